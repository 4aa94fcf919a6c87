// This file is a drop-in for the OpenTSDB source tree (package
// net.opentsdb.core, next to TsdbQuery.java).  It is not compiled in this
// repository (no JDK here); INTEGRATION.md shows the two-line hook in
// TsdbQuery.GroupByAndAggregateCB.call that uses it.
package net.opentsdb.core;

import java.lang.reflect.Field;
import java.util.ArrayList;
import java.util.Calendar;
import java.util.List;
import java.util.NoSuchElementException;
import java.util.TimeZone;

import net.opentsdb.utils.DateTime;

/**
 * Evaluates every {@link SpanGroup} of one query in a single call into
 * libotsdb_agg.so (the MI355X engine, include/otsdb_agg.h) instead of one
 * lazy AggregationIterator per group (SpanGroup.iterator(),
 * SpanGroup.java:525-530).  The spans' compacted RowSeq bytes go to the GPU
 * as they are (otsdb_agg_run_cells): decode, downsample / fill, rate,
 * interpolation and the cross-series aggregator run there.  The results are
 * served by {@link ArrayDataPoints}, which keeps the SpanGroup for names,
 * tags and annotations.
 *
 * <p>{@link #aggregate} returns {@code null} when the engine does not take
 * the query (rollup / histogram spans, scalar fill, a calendar grid that
 * depends on each series' first point, no library, no GPU): the caller then
 * keeps its SpanGroups and the Java iterators.  Exceptions the reference
 * path throws while iterating (IllegalDataException, IllegalStateException
 * "Got Infinity", ...) are thrown here, from the native status.
 */
public final class GpuAggregation {
  static final int OK = 0, ILLEGAL_DATA = 1, ILLEGAL_STATE = 2,
      ILLEGAL_ARGUMENT = 3, NO_SUCH_ELEMENT = 4, UNSUPPORTED = 5, DEVICE = 6,
      CAPACITY = 7;

  private static final boolean LOADED;
  private static final Field QUALIFIERS, VALUES;
  static {
    boolean ok;
    try {
      System.loadLibrary("otsdb_agg_jni");
      ok = true;
    } catch (UnsatisfiedLinkError e) {
      ok = false;
    }
    LOADED = ok;
    Field q = null, v = null;
    try {
      q = RowSeq.class.getDeclaredField("qualifiers");
      v = RowSeq.class.getDeclaredField("values");
      q.setAccessible(true);
      v.setAccessible(true);
    } catch (ReflectiveOperationException e) {
      q = v = null;
    }
    QUALIFIERS = q;
    VALUES = v;
  }

  /**
   * One engine context per thread (a context serialises its queries).  A
   * failed creation (library present, no usable GPU) is remembered: every
   * later query falls back to the Java iterators without retrying.
   */
  private static final ThreadLocal<Long> CTX = new ThreadLocal<Long>();
  private static volatile boolean CTX_FAILED = false;
  /** Contexts of every thread, destroyed at JVM exit. */
  private static final List<Long> ALL_CTX = new ArrayList<Long>();
  static {
    Runtime.getRuntime().addShutdownHook(new Thread() {
      @Override
      public void run() {
        synchronized (ALL_CTX) {
          for (final Long c : ALL_CTX) {
            nativeCtxDestroy(c);
          }
          ALL_CTX.clear();
        }
      }
    });
  }

  /** This thread's context, or 0 when no GPU context can be had. */
  private static long context() {
    if (CTX_FAILED) {
      return 0;
    }
    final Long c = CTX.get();
    if (c != null) {
      return c;
    }
    final long created;
    try {
      created = nativeCtxCreate(Integer.getInteger("tsd.gpu.device", 0));
    } catch (RuntimeException e) {
      CTX_FAILED = true;
      return 0;
    }
    if (created == 0) {
      CTX_FAILED = true;
      return 0;
    }
    CTX.set(created);
    synchronized (ALL_CTX) {
      ALL_CTX.add(created);
    }
    return created;
  }

  private GpuAggregation() {}

  // ---- natives (integration/jni/otsdb_agg_jni.c) -------------------------
  static native long nativeCtxCreate(int device);
  static native void nativeCtxDestroy(long ctx);
  /** otsdb_agg_id of the aggregator whose toString() is {@code name}, -1 if none. */
  static native int nativeAggId(String name);
  /**
   * otsdb_agg_run_cells.  spec = packed otsdb_query_spec (see SPEC_*).
   * Returns OK or CAPACITY (outputs too small: retry larger); every other
   * status is thrown as the reference's exception.
   */
  static native int nativeRunCells(long ctx, long[] spec, long[] calEdges,
      int nSeries, long[] rowSeries, long[] rowBase, long[] qualOff,
      byte[] qual, long[] valOff, byte[] val, long[] groupOffsets,
      long[] groupMembers, long[] outOffsets, long[] outTs, long[] outVal,
      byte[] outIsInt);

  // packed otsdb_query_spec
  static final int SPEC_START_MS = 0, SPEC_END_MS = 1, SPEC_QSTART_MS = 2,
      SPEC_QEND_MS = 3, SPEC_AGG = 4, SPEC_INTERP = 5, SPEC_DS_INTERVAL = 6,
      SPEC_DS_AGG = 7, SPEC_FILL = 8, SPEC_RUN_ALL = 9, SPEC_CALENDAR = 10,
      SPEC_RATE = 11, SPEC_COUNTER = 12, SPEC_DROP_RESETS = 13,
      SPEC_COUNTER_MAX = 14, SPEC_RESET_VALUE = 15, SPEC_LEN = 16;

  /**
   * The GroupByAndAggregateCB hook.  Arguments are what TsdbQuery hands the
   * SpanGroup constructor (TsdbQuery.java:1093-1101).
   */
  public static DataPoints[] aggregate(final SpanGroup[] groups,
      final long scan_start_s, final long scan_end_s,
      final Aggregator aggregator, final DownsamplingSpecification ds,
      final boolean rate, final RateOptions rate_options,
      final long query_start, final long query_end,
      final boolean split_rollup_raw_leg) {
    // the raw leg of a SplitRollupQuery must hand back SpanGroups
    // (SplitRollupQuery.RunCB.makeSpanGroupMap, SplitRollupQuery.java:436-441)
    if (!LOADED || QUALIFIERS == null || groups.length == 0
        || split_rollup_raw_leg) {
      return null;
    }
    final long[] spec = new long[SPEC_LEN];
    // SpanGroup normalises the window to ms (SpanGroup.java:267-270)
    spec[SPEC_START_MS] = scan_start_s * 1000;
    spec[SPEC_END_MS] = scan_end_s * 1000;
    spec[SPEC_QSTART_MS] = query_start;
    spec[SPEC_QEND_MS] = query_end;
    final int agg = nativeAggId(aggregator.toString());
    if (agg < 0) {
      return null;
    }
    spec[SPEC_AGG] = agg;
    spec[SPEC_INTERP] = -1;  // the aggregator's own interpolation
    long[] cal = null;
    if (ds != null && ds != DownsamplingSpecification.NO_DOWNSAMPLER) {
      final int ds_agg = nativeAggId(ds.getFunction().toString());
      if (ds_agg < 0 || ds.getFillPolicy() == FillPolicy.SCALAR) {
        return null;
      }
      spec[SPEC_DS_AGG] = ds_agg;
      spec[SPEC_FILL] = ds.getFillPolicy().ordinal();
      spec[SPEC_DS_INTERVAL] = ds.getInterval();
      // Downsampler.java:131-133: the deprecated (interval, function, fill)
      // constructor leaves the string interval null (not run-all)
      final String si = ds.getStringInterval();
      spec[SPEC_RUN_ALL] =
          si != null && si.toLowerCase().contains("all") ? 1 : 0;
      if (ds.useCalendar() && spec[SPEC_RUN_ALL] == 0) {
        cal = calendarEdges(ds, spec[SPEC_START_MS], spec[SPEC_END_MS]);
        if (cal == null) {
          return null;
        }
        spec[SPEC_CALENDAR] = 1;
      }
    }
    if (rate) {
      spec[SPEC_RATE] = 1;
      spec[SPEC_COUNTER] = rate_options.isCounter() ? 1 : 0;
      spec[SPEC_DROP_RESETS] = rate_options.getDropResets() ? 1 : 0;
      spec[SPEC_COUNTER_MAX] = rate_options.getCounterMax();
      spec[SPEC_RESET_VALUE] = rate_options.getResetValue();
    } else {
      spec[SPEC_COUNTER_MAX] = Long.MAX_VALUE;
    }

    // ---- the batch: series = spans in group order (each group lists its
    // spans in SpanCmp order), rows = the spans' RowSeqs in base-time order
    int n_series = 0, n_rows = 0, qbytes = 0, vbytes = 0;
    final List<List<RowSeq>> series_rows = new ArrayList<List<RowSeq>>();
    final long[] group_offsets = new long[groups.length + 1];
    for (int g = 0; g < groups.length; g++) {
      for (final Span span : groups[g].getSpans()) {
        if (span.getClass() != Span.class) {
          return null;  // rollup / histogram spans
        }
        span.iterator();  // checkRowOrder: rows sorted by base time
        final List<RowSeq> rs = new ArrayList<RowSeq>(span.rows.size());
        for (final iRowSeq r : span.rows) {
          if (!(r instanceof RowSeq)) {
            return null;
          }
          final RowSeq row = (RowSeq) r;
          qbytes += qualifiers(row).length;
          vbytes += values(row).length;
          rs.add(row);
        }
        n_rows += rs.size();
        series_rows.add(rs);
        n_series++;
      }
      group_offsets[g + 1] = n_series;
    }
    final long[] group_members = new long[n_series];
    for (int s = 0; s < n_series; s++) {
      group_members[s] = s;
    }
    final long[] row_series = new long[n_rows];
    final long[] row_base = new long[n_rows];
    final long[] qual_off = new long[n_rows + 1];
    final long[] val_off = new long[n_rows + 1];
    final byte[] qual = new byte[qbytes];
    final byte[] val = new byte[vbytes];
    int r = 0;
    for (int s = 0; s < n_series; s++) {
      for (final RowSeq row : series_rows.get(s)) {
        final byte[] q = qualifiers(row), v = values(row);
        row_series[r] = s;
        row_base[r] = row.baseTime();
        System.arraycopy(q, 0, qual, (int) qual_off[r], q.length);
        System.arraycopy(v, 0, val, (int) val_off[r], v.length);
        qual_off[r + 1] = qual_off[r] + q.length;
        val_off[r + 1] = val_off[r] + v.length;
        r++;
      }
    }

    // ---- outputs: one point per bucket (downsampled) or per raw point
    long cap = 1024;
    if (spec[SPEC_DS_INTERVAL] > 0) {
      final long nb = (spec[SPEC_END_MS] - spec[SPEC_START_MS])
          / spec[SPEC_DS_INTERVAL] + 4;
      cap = Math.max(cap, groups.length * nb);
    } else {
      cap = Math.max(cap, (long) vbytes + groups.length);
    }
    final long ctx = context();
    if (ctx == 0) {
      return null;  // no usable GPU: the Java iterators keep the query
    }
    while (true) {
      if (cap > Integer.MAX_VALUE - 8) {
        return null;
      }
      final long[] out_offsets = new long[groups.length + 1];
      final long[] out_ts = new long[(int) cap];
      final long[] out_val = new long[(int) cap];
      final byte[] out_is_int = new byte[(int) cap];
      final int st = nativeRunCells(ctx, spec, cal, n_series, row_series,
          row_base, qual_off, qual, val_off, val, group_offsets,
          group_members, out_offsets, out_ts, out_val, out_is_int);
      if (st == CAPACITY) {
        cap *= 2;
        continue;
      }
      if (st == UNSUPPORTED) {
        return null;
      }
      final DataPoints[] result = new DataPoints[groups.length];
      for (int g = 0; g < groups.length; g++) {
        result[g] = new ArrayDataPoints(groups[g], out_ts, out_val,
            out_is_int, (int) out_offsets[g], (int) out_offsets[g + 1]);
      }
      return result;
    }
  }

  private static byte[] qualifiers(final RowSeq row) {
    try {
      return (byte[]) QUALIFIERS.get(row);
    } catch (IllegalAccessException e) {
      throw new IllegalStateException(e);
    }
  }

  private static byte[] values(final RowSeq row) {
    try {
      return (byte[]) VALUES.get(row);
    } catch (IllegalAccessException e) {
      throw new IllegalStateException(e);
    }
  }

  /**
   * The calendar bucket grid the reference's Downsampler walks
   * (DateTime.previousInterval + Calendar.add, Downsampler.java:330-397),
   * from previousInterval(start) until two edges lie past end, or null when
   * a series could anchor its own grid off these edges (the engine then does
   * not take the query).
   */
  static long[] calendarEdges(final DownsamplingSpecification ds,
      final long start_ms, final long end_ms) {
    final String si = ds.getStringInterval();
    final int n = DateTime.getDurationInterval(si);
    final String units = DateTime.getDurationUnits(si);
    final int unit = DateTime.unitsToCalendarType(units);
    final TimeZone tz = ds.getTimezone();
    final Calendar c = DateTime.previousInterval(start_ms, n, unit, tz);
    final ArrayList<Long> edges = new ArrayList<Long>();
    edges.add(c.getTimeInMillis());
    int past = 0;
    while (past < 2) {
      if (unit == Calendar.DAY_OF_WEEK) {
        c.add(Calendar.DAY_OF_MONTH, 7 * n);
      } else {
        c.add(unit, n);
      }
      edges.add(c.getTimeInMillis());
      if (c.getTimeInMillis() > end_ms) {
        past++;
      }
      if (edges.size() > 10000000) {
        return null;
      }
    }
    final long[] out = new long[edges.size()];
    for (int i = 0; i < out.length; i++) {
      out[i] = edges.get(i);
    }
    // every anchor a series could start from must be an edge
    for (int i = 0; i + 1 < out.length && out[i] <= end_ms; i++) {
      final Calendar a = DateTime.previousInterval(out[i] + 1, n, unit, tz);
      if (a.getTimeInMillis() != out[i]) {
        return null;
      }
    }
    return out;
  }

  /** Maps a native status to the exception the reference path throws. */
  static void throwFor(final int status, final String msg) {
    switch (status) {
      case ILLEGAL_DATA: throw new IllegalDataException(msg);
      case ILLEGAL_STATE: throw new IllegalStateException(msg);
      case ILLEGAL_ARGUMENT: throw new IllegalArgumentException(msg);
      case NO_SUCH_ELEMENT: throw new NoSuchElementException(msg);
      default: throw new RuntimeException("GPU aggregation failed: " + msg);
    }
  }
}
