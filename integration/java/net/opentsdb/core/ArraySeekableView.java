// Drop-in for the OpenTSDB source tree (package net.opentsdb.core); see
// GpuAggregation.java.
package net.opentsdb.core;

import java.util.NoSuchElementException;

/**
 * SeekableView (SeekableView.java:37-71) over one group's GPU result.  Like
 * the iterators it replaces, next() returns one reused DataPoint; seek(t)
 * moves to the first point at or after t (a binary search: the timestamps
 * increase).
 */
final class ArraySeekableView implements SeekableView, DataPoint {
  private final long[] ts, val;
  private final byte[] is_int;
  private final int from, to;
  private int pos, cur = -1;

  ArraySeekableView(final long[] ts, final long[] val, final byte[] is_int,
      final int from, final int to) {
    this.ts = ts;
    this.val = val;
    this.is_int = is_int;
    this.from = from;
    this.to = to;
    this.pos = from;
  }

  public boolean hasNext() { return pos < to; }

  public DataPoint next() {
    if (pos >= to) {
      throw new NoSuchElementException("no more elements");
    }
    cur = pos++;
    return this;
  }

  public void remove() { throw new UnsupportedOperationException(); }

  public void seek(final long timestamp) {
    int lo = from, hi = to;
    while (lo < hi) {
      final int m = (lo + hi) >>> 1;
      if (ts[m] < timestamp) {
        lo = m + 1;
      } else {
        hi = m;
      }
    }
    pos = lo;
  }

  // DataPoint of the element next() returned
  public long timestamp() { return ts[cur]; }
  public boolean isInteger() { return is_int[cur] != 0; }

  public long longValue() {
    if (is_int[cur] == 0) {
      throw new ClassCastException("value is not a long");
    }
    return val[cur];
  }

  public double doubleValue() {
    if (is_int[cur] != 0) {
      throw new ClassCastException("value is not a float");
    }
    return Double.longBitsToDouble(val[cur]);
  }

  public double toDouble() {
    return is_int[cur] != 0 ? (double) val[cur] : Double.longBitsToDouble(val[cur]);
  }

  public long valueCount() { return 1; }
}
