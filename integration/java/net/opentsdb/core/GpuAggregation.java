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
      long[] calAnchors, long[] calAnchorEdge,
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
    long[][] cal = null;
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
        cal = calendarTables(ds, groups, spec[SPEC_START_MS],
            spec[SPEC_END_MS]);
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
      final int st = nativeRunCells(ctx, spec, cal == null ? null : cal[0],
          cal == null ? null : cal[1], cal == null ? null : cal[2], n_series,
          row_series,
          row_base, qual_off, qual, val_off, val, group_offsets,
          group_members, out_offsets, out_ts, out_val, out_is_int);
      if (st == CAPACITY) {
        // the result's own shortfall fills the offsets with the size the
        // whole result needs (include/otsdb_agg.h); any other capacity
        // (decode / compaction workspace) leaves them zero: grow
        // geometrically so a retry never re-runs the query for +1
        cap = Math.max(cap * 2, out_offsets[groups.length]);
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

  /** Ends each chain of an anchored calendar table (otsdb_agg.h). */
  static final long CHAIN_END = Long.MAX_VALUE;

  /** The Downsampler's step of a calendar (Downsampler.java:387-394). */
  private static void step(final Calendar c, final int n, final int unit) {
    if (unit == Calendar.DAY_OF_WEEK) {
      c.add(Calendar.DAY_OF_MONTH, 7 * n);
    } else {
      c.add(unit, n);
    }
  }

  /**
   * The calendar tables of otsdb_query_spec, built with the reference's own
   * DateTime.previousInterval and Calendar.add.  {edges} alone when every
   * series' grid is the one anchored at previousInterval(start)
   * (previousInterval(first point) of every series in the window is one of
   * its edges); otherwise {chains, anchors, anchor edges}: the series' own
   * anchors previousInterval(first point after the seek) — each series'
   * first point decoded through its Span iterator — and the window's, each
   * with the chain the Downsampler steps from it (Downsampler.java:330-345,
   * :383-397).  Null when a table would be unreasonably large.
   */
  static long[][] calendarTables(final DownsamplingSpecification ds,
      final SpanGroup[] groups, final long start_ms, final long end_ms) {
    final String si = ds.getStringInterval();
    final int n = DateTime.getDurationInterval(si);
    final String units = DateTime.getDurationUnits(si);
    final int unit = DateTime.unitsToCalendarType(units);
    final TimeZone tz = ds.getTimezone();
    // the last point any span holds: chains run two edges past it
    long last = end_ms;
    for (final SpanGroup g : groups) {
      for (final Span span : g.getSpans()) {
        if (span.size() > 0) {
          last = Math.max(last, span.timestamp(span.size() - 1));
        }
      }
    }
    // the window's own grid
    final long[] global = chain(DateTime.previousInterval(start_ms, n, unit,
        tz), n, unit, last);
    if (global == null) {
      return null;
    }
    // ValuesInInterval.seekInterval(start) (Downsampler.java:419-429)
    long seek = global[0];
    if (start_ms > seek) {
      seek = global[1];
    }
    final java.util.TreeSet<Long> anchors = new java.util.TreeSet<Long>();
    anchors.add(global[0]);
    boolean shared = true;
    final java.util.HashSet<Long> on_global = new java.util.HashSet<Long>();
    for (final long e : global) {
      on_global.add(e);
    }
    for (final SpanGroup g : groups) {
      for (final Span span : g.getSpans()) {
        final SeekableView it = span.iterator();
        it.seek(seek);
        if (!it.hasNext()) {
          continue;
        }
        final long f = it.next().timestamp();
        final long a = DateTime.previousInterval(f, n, unit, tz)
            .getTimeInMillis();
        anchors.add(a);
        shared &= on_global.contains(a);
      }
    }
    if (shared) {
      return new long[][] {global, null, null};
    }
    // one chain per anchor not already on an earlier chain
    final ArrayList<Long> edges = new ArrayList<Long>();
    final java.util.HashMap<Long, Integer> pos =
        new java.util.HashMap<Long, Integer>();
    final long[] anchor_arr = new long[anchors.size()];
    final long[] anchor_edge = new long[anchors.size()];
    int j = 0;
    for (final long a : anchors) {
      Integer p = pos.get(a);
      if (p == null) {
        final Calendar c = Calendar.getInstance(tz);
        c.setTimeInMillis(a);
        final long[] ch = chain(c, n, unit, last);
        if (ch == null) {
          return null;
        }
        p = edges.size();
        for (int k = 0; k < ch.length; k++) {
          if (!pos.containsKey(ch[k])) {
            pos.put(ch[k], p + k);
          }
          edges.add(ch[k]);
        }
        edges.add(CHAIN_END);
        if (edges.size() > 4000000) {
          return null;
        }
      }
      anchor_arr[j] = a;
      anchor_edge[j] = p;
      j++;
    }
    final long[] out = new long[edges.size()];
    for (int i = 0; i < out.length; i++) {
      out[i] = edges.get(i);
    }
    return new long[][] {out, anchor_arr, anchor_edge};
  }

  /** A calendar's steps until two edges lie past `last`. */
  private static long[] chain(final Calendar c, final int n, final int unit,
      final long last) {
    final ArrayList<Long> edges = new ArrayList<Long>();
    edges.add(c.getTimeInMillis());
    int past = 0;
    while (past < 2) {
      step(c, n, unit);
      edges.add(c.getTimeInMillis());
      if (c.getTimeInMillis() > last) {
        past++;
      }
      if (edges.size() > 4000000) {
        return null;
      }
    }
    final long[] out = new long[edges.size()];
    for (int i = 0; i < out.length; i++) {
      out[i] = edges.get(i);
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
