// Drop-in for the OpenTSDB source tree (package net.opentsdb.core); see
// GpuAggregation.java.
package net.opentsdb.core;

import java.util.List;
import java.util.Map;

import org.hbase.async.Bytes.ByteMap;

import com.stumbleupon.async.Deferred;

import net.opentsdb.meta.Annotation;

/**
 * One group's result of a batched GPU evaluation: the points are slices of
 * the arrays otsdb_agg_run_cells filled (timestamp ms, long value or double
 * bits, is-integer flag per point, AggregationIterator.isInteger
 * AggregationIterator.java:612-625); names, tags, aggregated tags,
 * annotations and the query index come from the SpanGroup the reference
 * built (SpanGroup.java:348-600), so serializers see the same DataPoints.
 */
final class ArrayDataPoints implements DataPoints {
  private final SpanGroup group;
  private final long[] ts, val;
  private final byte[] is_int;
  private final int from, to;

  ArrayDataPoints(final SpanGroup group, final long[] ts, final long[] val,
      final byte[] is_int, final int from, final int to) {
    this.group = group;
    this.ts = ts;
    this.val = val;
    this.is_int = is_int;
    this.from = from;
    this.to = to;
  }

  public String metricName() { return group.metricName(); }
  public Deferred<String> metricNameAsync() { return group.metricNameAsync(); }
  public byte[] metricUID() { return group.metricUID(); }
  public Map<String, String> getTags() { return group.getTags(); }
  public Deferred<Map<String, String>> getTagsAsync() { return group.getTagsAsync(); }
  public ByteMap<byte[]> getTagUids() { return group.getTagUids(); }
  public List<String> getAggregatedTags() { return group.getAggregatedTags(); }
  public Deferred<List<String>> getAggregatedTagsAsync() {
    return group.getAggregatedTagsAsync();
  }
  public List<byte[]> getAggregatedTagUids() { return group.getAggregatedTagUids(); }
  public List<String> getTSUIDs() { return group.getTSUIDs(); }
  public List<Annotation> getAnnotations() { return group.getAnnotations(); }
  public int aggregatedSize() { return group.aggregatedSize(); }
  public int getQueryIndex() { return group.getQueryIndex(); }
  public boolean isPercentile() { return false; }
  public float getPercentile() {
    throw new UnsupportedOperationException("getPercentile not supported");
  }

  public int size() { return to - from; }

  public SeekableView iterator() {
    return new ArraySeekableView(ts, val, is_int, from, to);
  }

  private int idx(final int i) {
    if (i < 0 || i >= to - from) {
      throw new IndexOutOfBoundsException("index " + i + " >= " + size());
    }
    return from + i;
  }

  public long timestamp(final int i) { return ts[idx(i)]; }
  public boolean isInteger(final int i) { return is_int[idx(i)] != 0; }

  public long longValue(final int i) {
    final int k = idx(i);
    if (is_int[k] == 0) {
      throw new ClassCastException("value #" + i + " is not a long");
    }
    return val[k];
  }

  public double doubleValue(final int i) {
    final int k = idx(i);
    if (is_int[k] != 0) {
      throw new ClassCastException("value #" + i + " is not a float");
    }
    return Double.longBitsToDouble(val[k]);
  }

  @Override
  public String toString() {
    return "ArrayDataPoints(" + size() + " points of " + group + ")";
  }
}
