/*
 * otsdb_agg.h — C-ABI of the MI355X-native OpenTSDB query-time aggregation
 * engine (libotsdb_agg.so).
 *
 * This is the drop-in boundary for ONE path of OpenTSDB: the query-time
 * aggregation that today runs as a chain of Java iterators
 *
 *   Span/RowSeq points -> Downsampler | FillingDownsampler -> RateSpan
 *                      -> AggregationIterator (cross-series group-by)
 *
 * created by SpanGroup.iterator() (src/core/SpanGroup.java:525-530) for every
 * group that TsdbQuery.GroupByAndAggregateCB.call builds
 * (src/core/TsdbQuery.java:992-1113).  A JNI shim replaces
 * the per-group lazy iterators with ONE batched call per query: every group of
 * the query is evaluated on the GPU and handed back as arrays, which a Java
 * array-backed SeekableView/DataPoints then serves to the unchanged callers
 * (HttpJsonSerializer.java:821-869, CliQuery.java:126).
 *
 * Conventions: plain C types only, no torch/HIP types in the signatures.
 * Every entry point returns an otsdb_status; on failure the thread-local
 * message is available from otsdb_last_error().  Status codes map 1:1 onto the
 * Java exceptions the reference path throws (see otsdb_status).
 */
#ifndef OTSDB_AGG_H
#define OTSDB_AGG_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OTSDB_ABI_VERSION 6

/* ------------------------------------------------------------------------ */
/* Status codes — 1:1 with the exceptions of the reference path.             */
/* ------------------------------------------------------------------------ */
typedef enum {
  OTSDB_OK = 0,
  /* IllegalDataException: corrupted cell (Internal.java:307-321), `none`
   * aggregator fed more than one value (Aggregators.java:446-460).          */
  OTSDB_E_ILLEGAL_DATA = 1,
  /* IllegalStateException: "Got Infinity" (AggregationIterator.java:640-643),
   * non-increasing timestamps in a rate (RateSpan.java:129-134), empty long
   * median (Aggregators.java:408-410).                                      */
  OTSDB_E_ILLEGAL_STATE = 2,
  /* IllegalArgumentException: bad spec (DownsamplingSpecification.java:116+,
   * Downsampler "cannot use the NONE aggregator for downsampling").        */
  OTSDB_E_ILLEGAL_ARGUMENT = 3,
  /* NoSuchElementException: unknown aggregator (Aggregators.java:222-228). */
  OTSDB_E_NO_SUCH_ELEMENT = 4,
  /* Valid in the reference but not implemented by this engine (calendar
   * downsampling, rollups, histograms, scalar fill): the Java side keeps its
   * own iterators for such queries.                                         */
  OTSDB_E_UNSUPPORTED = 5,
  /* HIP runtime failure / out of device memory.                            */
  OTSDB_E_DEVICE = 6,
  /* Caller-provided output capacity too small (otsdb_result.capacity).  The
   * host entries (otsdb_agg_run, otsdb_agg_run_cells, otsdb_agg_run_raw)
   * still fill result.offsets with the whole result's offsets, so
   * offsets[n_groups] is the capacity a retry needs; nothing else written. */
  OTSDB_E_CAPACITY = 7
} otsdb_status;

/* ------------------------------------------------------------------------ */
/* Aggregators registry (Aggregators.java:175-203).  Ids are stable.         */
/* ------------------------------------------------------------------------ */
typedef enum {
  OTSDB_AGG_SUM = 0,        /* "sum"       Sum(LERP)                 */
  OTSDB_AGG_PFSUM = 1,      /* "pfsum"     Sum(PREV)                 */
  OTSDB_AGG_MIN = 2,        /* "min"       Min(LERP)                 */
  OTSDB_AGG_MAX = 3,        /* "max"       Max(LERP)                 */
  OTSDB_AGG_AVG = 4,        /* "avg"       Avg(LERP)                 */
  OTSDB_AGG_MEDIAN = 5,     /* "median"    Median(LERP)              */
  OTSDB_AGG_NONE = 6,       /* "none"      None(ZIM), toString "raw" */
  OTSDB_AGG_MULT = 7,       /* "mult"      Multiply(LERP)            */
  OTSDB_AGG_DEV = 8,        /* "dev"       StdDev(LERP)              */
  OTSDB_AGG_DIFF = 9,       /* "diff"      Diff(LERP)                */
  OTSDB_AGG_ZIMSUM = 10,    /* "zimsum"    Sum(ZIM)                  */
  OTSDB_AGG_MIMMIN = 11,    /* "mimmin"    Min(MAX)                  */
  OTSDB_AGG_MIMMAX = 12,    /* "mimmax"    Max(MIN)                  */
  OTSDB_AGG_SQUARESUM = 13, /* "squareSum" SquareSum(ZIM)            */
  OTSDB_AGG_COUNT = 14,     /* "count"     Count(ZIM)                */
  OTSDB_AGG_FIRST = 15,     /* "first"     First(ZIM)                */
  OTSDB_AGG_LAST = 16,      /* "last"      Last(ZIM)                 */
  /* PercentileAgg(LERP), commons-math3 3.4.1 Percentile
   * (Aggregators.java:125-173, :657-708).  LEGACY estimation: */
  OTSDB_AGG_P999 = 17, OTSDB_AGG_P99 = 18, OTSDB_AGG_P95 = 19,
  OTSDB_AGG_P90 = 20, OTSDB_AGG_P75 = 21, OTSDB_AGG_P50 = 22,
  /* R_3 estimation (honoured by runLong only, Aggregators.java:690): */
  OTSDB_AGG_EP999R3 = 23, OTSDB_AGG_EP99R3 = 24, OTSDB_AGG_EP95R3 = 25,
  OTSDB_AGG_EP90R3 = 26, OTSDB_AGG_EP75R3 = 27, OTSDB_AGG_EP50R3 = 28,
  /* R_7 estimation (honoured by runLong only): */
  OTSDB_AGG_EP999R7 = 29, OTSDB_AGG_EP99R7 = 30, OTSDB_AGG_EP95R7 = 31,
  OTSDB_AGG_EP90R7 = 32, OTSDB_AGG_EP75R7 = 33, OTSDB_AGG_EP50R7 = 34,
  OTSDB_AGG_COUNT_IDS = 35
} otsdb_agg_id;

/* Aggregators.Interpolation (Aggregators.java:38-44), Java ordinal order. */
typedef enum {
  OTSDB_INTERP_DEFAULT = -1, /* use the aggregator's own method */
  OTSDB_INTERP_LERP = 0,
  OTSDB_INTERP_ZIM = 1,
  OTSDB_INTERP_MAX = 2,
  OTSDB_INTERP_MIN = 3,
  OTSDB_INTERP_PREV = 4
} otsdb_interp;

/* FillPolicy (FillPolicy.java:22-28), Java ordinal order. */
typedef enum {
  OTSDB_FILL_NONE = 0,
  OTSDB_FILL_ZERO = 1,
  OTSDB_FILL_NAN = 2,
  OTSDB_FILL_NULL = 3,
  OTSDB_FILL_SCALAR = 4 /* FillingDownsampler throws "unhandled fill policy" */
} otsdb_fill;

/* ------------------------------------------------------------------------ */
/* Query spec: one per query (all groups share it).                          */
/* ------------------------------------------------------------------------ */
#define OTSDB_SPEC_EXACT_ORDER 1
typedef struct {
  /* AggregationIterator window, ms, inclusive on both ends
   * (SpanGroup ctor normalises the scan bounds to ms, SpanGroup.java:267-270;
   * TsdbQuery passes getScanStartTimeSeconds/getScanEndTimeSeconds,
   * TsdbQuery.java:1092-1093).                                               */
  int64_t start_ms;
  int64_t end_ms;
  /* Raw query bounds (TsdbQuery.getStartTime/getEndTime, ms): used by the
   * "all" downsampler (Downsampler.java:354-379).                            */
  int64_t query_start_ms;
  int64_t query_end_ms;
  int32_t agg_id;          /* otsdb_agg_id — cross-series aggregator       */
  int32_t interp;          /* otsdb_interp, OTSDB_INTERP_DEFAULT normally  */
  int64_t ds_interval_ms;  /* 0 = no downsampling (raw path)               */
  int32_t ds_agg_id;       /* downsampling function (not NONE)             */
  int32_t fill;            /* otsdb_fill                                   */
  int32_t run_all;         /* "0all-<agg>" downsampling                    */
  int32_t use_calendar;    /* "<n><u>c-" downsampling: needs cal_edges     */
  int32_t rate;            /* RateSpan applied after downsampling          */
  int32_t counter;         /* RateOptions.counter                          */
  int32_t drop_resets;     /* RateOptions.drop_resets                      */
  /* OTSDB_SPEC_* bits (ABI 5; the padding word before, callers pass 0).
   * OTSDB_SPEC_EXACT_ORDER: an order-sensitive aggregator (dev) reduces
   * every (group, timestamp) in ONE sequential chain over the group's
   * members in SpanCmp order, whatever the group's size — StdDev.runDouble's
   * one Welford loop (Aggregators.java:547-568) bit for bit.  Without it a
   * group of more than 65,536 members on one device merges in-order chunk
   * states with Chan's formula: on well-conditioned contributions (counter
   * rates, C4) within 1e-12 of the loop, on offset gauges (~3e9 +- 1e4,
   * where the loop itself lies ~1e-11 from the exact sigma) measured
   * ~1e-11 off (tests/test_gpu_dev_large.py); the chain costs ~100-180 ns a
   * member per bucket (tools/chain_probe.hip: a 500k-member group ~50-90 ms).
   * A chain whose bucket rows (9 B per member and bucket) pass the engine's
   * fixed row budget is OTSDB_E_CAPACITY with the flag, merged without.    */
  int32_t flags;
  int64_t counter_max;     /* RateOptions.counter_max (default Long.MAX)   */
  int64_t reset_value;     /* RateOptions.reset_value (default 0)          */
  /* Calendar downsampling (use_calendar = 1): the bucket edges, ms, strictly
   * ascending, HOST memory (copied during the call).  cal_edges[0] =
   * DateTime.previousInterval(start_ms, n, unit, tz) (DateTime.java:450-610)
   * and cal_edges[k+1] = cal_edges[k] stepped once the way the Downsampler
   * steps its calendars (Calendar.add(unit, n), or 7n days for weeks,
   * Downsampler.java:387-394), continued until two edges lie past end_ms
   * (past the batch's last point if spans hold points beyond the window).
   * Bucket k is [cal_edges[k], cal_edges[k+1]) with timestamp cal_edges[k]
   * (ValuesInInterval.getIntervalTimestamp, :437-449).  The reference
   * anchors each series at previousInterval(its first point): when every
   * such anchor in the window is an edge of this one table (the grid does
   * not depend on the series: 1dc, 1hc, 1nc, 30mc, ... in any zone) the
   * caller passes it alone (n_cal_anchors = 0).  A point past the window
   * whose bucket end is not in the table is OTSDB_E_UNSUPPORTED.  NULL with
   * use_calendar = 1 -> OTSDB_E_UNSUPPORTED.  ds_interval_ms stays
   * DownsamplingSpecification's nominal interval (parseDuration), which the
   * scan bounds use.                                                       */
  const int64_t* cal_edges;
  int64_t n_cal_edges;
  /* Per-series calendar anchors (n_cal_anchors > 0; 7mc, 2wc, 6hc across a
   * DST change, ...): cal_edges then holds CHAINS, each the Downsampler's
   * calendar stepped from one anchor (Downsampler.java:330-345, :383-397)
   * until two edges lie past the window / the batch's last point, strictly
   * ascending and ended by INT64_MAX.  cal_anchors[j] (ascending) are
   * DateTime.previousInterval values and cal_anchor_edge[j] the index in
   * cal_edges of the chain edge equal to cal_anchors[j]; for every series'
   * first point f after the seek, previousInterval(f) must be the largest
   * anchor <= f (true when the anchors hold every previousInterval value of
   * the window, or just the ones the batch's series take), and so must
   * previousInterval(start_ms) (the seek, Downsampler.java:419-429).  Series
   * grids then differ, and the output timestamps are the union of the
   * series' bucket starts (AggregationIterator.next).  With fill != NONE
   * the FillingDownsampler's own grid is the chain from previousInterval(
   * start_ms) to previousInterval(end_ms) (FillingDownsampler.java:113-135):
   * previousInterval(end_ms) must then be the largest anchor <= end_ms too.
   * A point past its chain's last edge is OTSDB_E_UNSUPPORTED only when a
   * query reads it (rate queries; the first bucket past the window).  The
   * multi-GPU partial / selection entry points -> OTSDB_E_UNSUPPORTED.
   * HOST memory.                                                          */
  const int64_t* cal_anchors;
  const int64_t* cal_anchor_edge;
  int64_t n_cal_anchors;
} otsdb_query_spec;

/* ------------------------------------------------------------------------ */
/* Columnar batch.  Series are given in SpanCmp order (TsdbQuery.java:      */
/* 1862-1892); each group lists its member series in that order.            */
/* Within a series points must be sorted by timestamp (Span/RowSeq order).  */
/* Pointers are HOST pointers for otsdb_agg_run and DEVICE pointers for     */
/* otsdb_agg_run_device.                                                    */
/* ------------------------------------------------------------------------ */
typedef struct {
  int64_t n_series;             /* S                                       */
  int64_t n_points;             /* N = offsets[S]                          */
  const int64_t* offsets;       /* [S+1] CSR point offsets                 */
  const int64_t* ts_ms;         /* [N] timestamps, ms                      */
  const int64_t* val;           /* [N] raw value bits: int64 or IEEE f64   */
  /* Value type.  Exactly one of the following conventions:
   *  - is_float != NULL: per point, 1 = double, 0 = long;
   *  - else series_float != NULL: per series, 1 = double, 0 = long;
   *  - else all values are doubles.                                       */
  const uint8_t* is_float;      /* [N] or NULL                             */
  const uint8_t* series_float;  /* [S] or NULL                             */
  int64_t n_groups;             /* G                                       */
  const int64_t* group_offsets; /* [G+1] CSR into group_members            */
  const int64_t* group_members; /* [M] series indices, SpanCmp order       */
  /* Optional HOST copy of group_offsets (the same G+1 values) for the
   * device entries: the engine plans its tiles from it instead of reading
   * group_offsets back from the device (one copy + stream sync per call).
   * NULL = read it back.  Ignored by the host entries.  The engine plans
   * its tiles from this copy and trusts it: it must equal the device array
   * at the call (a stale copy makes the kernels read members past a group;
   * debug builds, -DOTSDB_DEBUG_SYNC, compare the last offset).            */
  const int64_t* group_offsets_host;
} otsdb_batch;

/* ------------------------------------------------------------------------ */
/* Result: caller-allocated (sizes from otsdb_agg_plan).  Group g's points   */
/* are [offsets[g], offsets[g+1]).  Value bits are a long when is_int=1,     */
/* else an IEEE double (AggregationIterator.isInteger, :612-625).            */
/* ------------------------------------------------------------------------ */
typedef struct {
  int64_t capacity;   /* max points the ts/val/is_int arrays can hold      */
  int64_t* offsets;   /* [G+1]                                              */
  int64_t* ts;        /* [capacity]                                         */
  int64_t* val;       /* [capacity] raw bits                                */
  uint8_t* is_int;    /* [capacity]                                         */
} otsdb_result;

typedef struct {
  int64_t n_buckets;        /* grid buckets per series (downsampled path)  */
  int64_t max_out_points;   /* upper bound of total output points          */
  int64_t workspace_bytes;  /* device scratch this query needs              */
} otsdb_sizes;

typedef struct otsdb_ctx otsdb_ctx;

/* ---- context ------------------------------------------------------------ */
int otsdb_abi_version(void);
/* Creates a context bound to HIP device `device` (one process per GPU).     */
otsdb_status otsdb_ctx_create(int device, otsdb_ctx** out);
void otsdb_ctx_destroy(otsdb_ctx* ctx);
/* Thread-local message of the last failing call on this thread.            */
const char* otsdb_last_error(void);

/* ---- registry (Aggregators.get / toString / interpolationMethod) -------- */
/* Aggregators.get(name): OTSDB_E_NO_SUCH_ELEMENT for unknown names.         */
otsdb_status otsdb_agg_lookup(const char* name, int32_t* agg_id);
const char* otsdb_agg_name(int32_t agg_id);         /* toString()          */
int32_t otsdb_agg_interpolation(int32_t agg_id);    /* otsdb_interp        */

/* ---- query -------------------------------------------------------------- */
/* Validates spec+batch shape and returns output/workspace sizes.            */
otsdb_status otsdb_agg_plan(otsdb_ctx* ctx, const otsdb_query_spec* spec,
                            const otsdb_batch* batch, otsdb_sizes* out);
/* Host-pointer entry (the JNI shim): copies the batch to HBM, runs, copies
 * the result back.  Synchronous.                                            */
otsdb_status otsdb_agg_run(otsdb_ctx* ctx, const otsdb_query_spec* spec,
                           const otsdb_batch* batch, otsdb_result* out);
/* Device-pointer entry: batch and result live in HBM; runs on `hip_stream`
 * (a hipStream_t passed as void*, NULL = the context's stream).  Returns
 * after the result is complete on the device (the status needs the device
 * error word).                                                               */
otsdb_status otsdb_agg_run_device(otsdb_ctx* ctx, const otsdb_query_spec* spec,
                                  const otsdb_batch* batch, otsdb_result* out,
                                  void* hip_stream);

/* ---- multi-GPU (series-sharded) ----------------------------------------- */
/* Partial per-(group, bucket) reduction state, the unit exchanged between
 * ranks over RCCL.  32 bytes, see DESIGN.md §Multi-GPU.                     */
typedef struct {
  double x, y, z;
  int64_t w;
} otsdb_partial;

/* Runs the local shard (downsample/rate/interpolate + chunked group reduce)
 * and writes one partial per (group, bucket) plus the emit mask into DEVICE
 * buffers partials[G*n_buckets], emit[G*n_buckets].  n_buckets from plan.   */
otsdb_status otsdb_agg_partials_device(otsdb_ctx* ctx,
                                       const otsdb_query_spec* spec,
                                       const otsdb_batch* batch,
                                       otsdb_partial* partials,
                                       uint8_t* emit, void* hip_stream);
/* The same, each (group, bucket) continuing from `init`/`init_emit` (DEVICE,
 * [G*n_buckets]): the state of the group's members on the ranks before this
 * one.  Handed from rank to rank in series order, the last rank's output is
 * the state ONE pass over every member in SpanCmp order reaches — for `dev`
 * the reference's single Welford loop (StdDev.runDouble,
 * src/core/Aggregators.java:547-568, fed by AggregationIterator.java:735-797)
 * bit for bit while each rank's share of a group is one chain
 * (<= 65,536 members), where merging per-rank partials (Chan's formula)
 * lands ~1e-11 from it on offset data.  Groups with no member on this rank
 * pass their state on unchanged; init may alias partials.  Finalise the last
 * rank's output with otsdb_agg_finalize_device(n_ranks = 1).              */
otsdb_status otsdb_agg_partials_chained_device(otsdb_ctx* ctx,
                                               const otsdb_query_spec* spec,
                                               const otsdb_batch* batch,
                                               const otsdb_partial* init,
                                               const uint8_t* init_emit,
                                               otsdb_partial* partials,
                                               uint8_t* emit, void* hip_stream);
/* Combines `n_ranks` partial sets laid out rank-major in DEVICE memory
 * ([n_ranks][G*n_buckets], combined in rank order = series order) and
 * writes the final result (DEVICE pointers).                                */
otsdb_status otsdb_agg_finalize_device(otsdb_ctx* ctx,
                                       const otsdb_query_spec* spec,
                                       int64_t n_groups, int64_t n_buckets,
                                       int32_t n_ranks,
                                       const otsdb_partial* partials,
                                       const uint8_t* emit,
                                       otsdb_result* out, void* hip_stream);

/* ---- multi-GPU median / percentiles (series-sharded) -------------------- */
/* Exact selection across ranks: digit histograms summed over
 * the ranks, at most two passes over each rank's local keys.  The protocol,
 * every rank in step:
 *
 *   otsdb_sel_prepare_device(ctx, spec, batch, counts, emit, krange)
 *       local shard -> per-(group, bucket) non-NaN contribution counts
 *       (int64 [G*n_buckets]), emit flags (u8) and key range (int64
 *       [G*n_buckets][2]) in DEVICE memory
 *   all-reduce counts (sum), emit (max), krange (min)
 *   for pass = 0, 1, ...:
 *       otsdb_sel_hist_device(ctx, pass, counts, emit, krange, hist_prev,
 *                             hist, &more)
 *           pass 0 reads the global counts / emit / krange; a later pass
 *           applies hist_prev, the global histogram of the pass before (it
 *           may be `hist` itself).  more == 0: the selection is resolved,
 *           leave the loop.  more == 1: `hist` holds this rank's histogram
 *           of the pass, u32 [G*n_buckets][OTSDB_SEL_BINS]; all-reduce it
 *           (sum)
 *   otsdb_sel_pick_device(ctx, picks)
 *       int64 [G*n_buckets][2]: the key of an order statistic whose bin
 *       holds one key over all ranks, from the rank holding it, else 0
 *   all-reduce picks (sum)
 *   otsdb_sel_finish_device(ctx, picks, result)
 *
 * Pass 0 bins an offset digit, (key >> s) - (min >> s) over the global key
 * range (2,048 bins); pass 1 the next 11 bits (2 x 10 when the estimator's
 * two order statistics sit in different bins) and compacts the local keys
 * still in play into a candidate pool; later passes and the pick read the
 * pool only.  Local key-matrix reads: two at most (otsdb_ctx_counters [3]).
 * otsdb_sel_hist_device reads its plan back (one stream sync) but returns
 * without waiting for the histogram kernels: the caller's collective must be
 * ordered after them on hip_stream (an RCCL all-reduce enqueued there is); a
 * binding that reads `hist` from the host or from another stream calls
 * otsdb_sel_hist_wait(ctx, hip_stream) first; the same holds for `picks`.
 * Every rank ends with the full result.  The batch's group_offsets span all
 * G global groups (empty where the rank holds no member).  Between prepare
 * and finish the context must not run other queries (the session lives in
 * its workspace).  Replaces PercentileAgg/Median.runDouble over the spans of
 * a group (Aggregators.java:397-431, :657-708) when the spans are spread
 * over GPUs.                                                               */
#define OTSDB_SEL_BINS 2048
otsdb_status otsdb_sel_prepare_device(otsdb_ctx* ctx,
                                      const otsdb_query_spec* spec,
                                      const otsdb_batch* batch,
                                      int64_t* counts, uint8_t* emit,
                                      int64_t* krange, void* hip_stream);
otsdb_status otsdb_sel_hist_device(otsdb_ctx* ctx, int32_t pass,
                                   const int64_t* counts, const uint8_t* emit,
                                   const int64_t* krange, uint32_t* hist_prev,
                                   uint32_t* hist, int32_t* more,
                                   void* hip_stream);
otsdb_status otsdb_sel_pick_device(otsdb_ctx* ctx, int64_t* picks,
                                   void* hip_stream);
otsdb_status otsdb_sel_finish_device(otsdb_ctx* ctx, const int64_t* picks,
                                     otsdb_result* out, void* hip_stream);
/* Blocks until the kernels otsdb_sel_hist_device / _pick_device enqueued on
 * hip_stream (NULL: the context's stream) are done.                         */
otsdb_status otsdb_sel_hist_wait(otsdb_ctx* ctx, void* hip_stream);

/* ---- compacted-cell decode (RowSeq) ------------------- */
/* The storage rows of a query as the scanner hands them to Span.addRow
 * (Span.java:177-220): one compacted column per (series, hour) row —
 * concatenated 2-byte (seconds) / 4-byte (ms) qualifiers and concatenated
 * big-endian values, plus the trailing meta byte of multi-value columns
 * (CompactionQueue.buildCompactedColumn, CompactionQueue.java:594-616).
 * Rows sorted by (series, base time).  DEVICE pointers.                     */
typedef struct {
  int64_t n_rows;            /* R                                          */
  const int64_t* row_series; /* [R] series index, nondecreasing            */
  const int64_t* row_base_s; /* [R] row base time, seconds                 */
  const int64_t* qual_off;   /* [R+1] offsets into qual                    */
  const uint8_t* qual;       /* qualifier bytes                            */
  const int64_t* val_off;    /* [R+1] offsets into val                     */
  const uint8_t* val;        /* value bytes                                */
} otsdb_cells;

/* Decodes the rows into a columnar batch (RowSeq.Iterator semantics,
 * RowSeq.java:552-643): offsets[S+1] (series point CSR), ts_ms/val/is_float
 * [capacity].  Pass ts_ms=NULL to only count (offsets filled, offsets[S] =
 * points).  A column whose value bytes do not match its qualifiers is
 * OTSDB_E_ILLEGAL_DATA (Internal.extractDataPoints, Internal.java:307-321). */
otsdb_status otsdb_decode_cells_device(otsdb_ctx* ctx, const otsdb_cells* cells,
                                       int64_t n_series, int64_t* offsets,
                                       int64_t* ts_ms, int64_t* val,
                                       uint8_t* is_float, int64_t capacity,
                                       void* hip_stream);

/* Test / bench infrastructure (not the query path): encodes a columnar
 * DEVICE batch into compacted RowSeq columns, the layout the write path and
 * compaction produce and otsdb_decode_cells_device reads (one row per
 * (series, hour); 2-byte qualifiers for whole seconds, 4-byte ms qualifiers
 * otherwise; doubles in 8 bytes, longs in the smallest of 1/2/4/8; the meta
 * byte on multi-value columns; Internal.java:848-863, TSDB.java:1051-1147,
 * CompactionQueue.java:594-616).  Two calls: with cells == NULL it writes
 * per-series counts (rows, qualifier bytes, value bytes) into series_rows /
 * series_qbytes / series_vbytes [S]; then, with those arrays turned into
 * exclusive prefix sums by the caller, it writes the cells (qual_off[R] and
 * val_off[R] are the caller's totals).  Values are typed by
 * batch->series_float (NULL = doubles).                                    */
typedef struct {
  int64_t* row_series;  /* [R] */
  int64_t* row_base_s;  /* [R] */
  int64_t* qual_off;    /* [R+1] */
  uint8_t* qual;
  int64_t* val_off;     /* [R+1] */
  uint8_t* val;
} otsdb_cells_out;

otsdb_status otsdb_encode_cells_device(otsdb_ctx* ctx, const otsdb_batch* batch,
                                       int64_t* series_rows,
                                       int64_t* series_qbytes,
                                       int64_t* series_vbytes,
                                       const otsdb_cells_out* cells,
                                       void* hip_stream);

/* The query straight from compacted columns (DEVICE pointers): the decode
 * runs fused into the downsample (no columnar copy).
 * `batch` supplies n_series and the groups only (its point arrays are not
 * read); series s owns the rows with row_series == s.  A corrupt column is
 * OTSDB_E_ILLEGAL_DATA.  Queries the fused path does not cover (raw
 * group-by, median / percentile or "all" downsampling, columns mixing 2-
 * and 4-byte qualifiers) are decoded into a context-owned columnar buffer
 * first and run through the columnar pipeline — same results.           */
otsdb_status otsdb_agg_run_cells_device(otsdb_ctx* ctx,
                                        const otsdb_query_spec* spec,
                                        const otsdb_cells* cells,
                                        const otsdb_batch* batch,
                                        otsdb_result* out, void* hip_stream);
/* The same with HOST pointers (the JNI entry at the TsdbQuery seam: the
 * Spans' RowSeq bytes, SpanGroup members); copies in, runs, copies the
 * result out.  Synchronous.  row_series must be nondecreasing.            */
otsdb_status otsdb_agg_run_cells(otsdb_ctx* ctx, const otsdb_query_spec* spec,
                                 const otsdb_cells* cells,
                                 const otsdb_batch* batch, otsdb_result* out);

/* ---- storage rows: query-time compaction + span assembly (§8a a3, a4) -- */
/* The storage rows of a query exactly as the scanner returns them, before
 * TSDB.compact (SaltScanner.java:849-881): each row (one series, one base
 * hour) is a list of columns — single-point cells, compacted columns, append
 * columns (qualifier {0x05,0,0}), annotations / histograms (skipped).        */
typedef struct {
  int64_t n_rows;               /* R                                        */
  const int64_t* row_series;    /* [R] series index, nondecreasing; a series'
                                 * rows in the order the scanner delivers them
                                 * (the Span.addRow call order)            */
  const int64_t* row_base_s;    /* [R] row base time, seconds (row key)     */
  const int64_t* row_col_off;   /* [R+1] CSR into the columns               */
  const int64_t* col_qual_off;  /* [C+1] offsets into qual                  */
  const uint8_t* qual;          /* column qualifiers                        */
  const int64_t* col_val_off;   /* [C+1] offsets into val                   */
  const uint8_t* val;           /* column values                            */
  const int64_t* col_ts;        /* [C] HBase cell timestamps (newest wins a
                                 * duplicate); NULL = ascending column order */
} otsdb_raw_rows;

/* CompactionQueue.compact of every row (CompactionQueue.java:340-616, with
 * ColumnDatapointIterator fix-ups :73-87 / Internal.java:535-591 and
 * AppendDataPoints.parseKeyValue :118-236): one compacted column per row,
 * rows without a data point dropped (as the scanner drops a null
 * compaction), kept rows packed in input order into `out` (DEVICE pointers,
 * caller-allocated: qual_capacity >= the input's qualifier + value bytes and
 * val_capacity >= its value bytes + n_rows always suffice).  *n_out_rows =
 * kept rows; out->qual_off[n] / val_off[n] hold the totals; out->row_series
 * may be NULL.  out == NULL: sizes only.  Duplicate offsets with different
 * values: OTSDB_E_ILLEGAL_DATA unless fix_duplicates
 * (tsd.storage.fix_duplicates); corrupt cells / appends: OTSDB_E_ILLEGAL_DATA;
 * an odd qualifier starting 0x05 that is not 3 bytes:
 * OTSDB_E_ILLEGAL_ARGUMENT; a row needing a merge of more than 8192 points
 * or 4096 data columns: OTSDB_E_UNSUPPORTED.  The first failing row (in row
 * order) decides the status.                                               */
otsdb_status otsdb_compact_rows_device(otsdb_ctx* ctx, const otsdb_raw_rows* raw,
                                       int32_t fix_duplicates,
                                       const otsdb_cells_out* out,
                                       int64_t qual_capacity,
                                       int64_t val_capacity,
                                       int64_t* n_out_rows, void* hip_stream);

/* Span.addRow of every series' compacted rows in arrival order
 * (Span.java:177-220, RowSeq.addRow RowSeq.java:91-222, checkRowOrder
 * :387-392): rows of the same key merge, rows end up sorted by base time.
 * `cells` rows carry nondecreasing row_series; out (DEVICE, caller-allocated,
 * capacities >= the input's bytes + n_rows) receives the span rows; NULL =
 * sizes only.  A row without a qualifier is OTSDB_E_ILLEGAL_ARGUMENT.       */
otsdb_status otsdb_span_assemble_device(otsdb_ctx* ctx, const otsdb_cells* cells,
                                        int64_t n_series,
                                        const otsdb_cells_out* out,
                                        int64_t qual_capacity,
                                        int64_t val_capacity,
                                        int64_t* n_out_rows, void* hip_stream);

/* The whole query from storage rows: compaction -> span assembly -> the
 * fused decode + aggregation of otsdb_agg_run_cells_device.  `batch`
 * supplies n_series and the groups.  _device: DEVICE pointers;
 * otsdb_agg_run_raw: HOST pointers (the JNI entry), synchronous.            */
otsdb_status otsdb_agg_run_raw_device(otsdb_ctx* ctx,
                                      const otsdb_query_spec* spec,
                                      const otsdb_raw_rows* raw,
                                      int32_t fix_duplicates,
                                      const otsdb_batch* batch,
                                      otsdb_result* out, void* hip_stream);
otsdb_status otsdb_agg_run_raw(otsdb_ctx* ctx, const otsdb_query_spec* spec,
                               const otsdb_raw_rows* raw, int32_t fix_duplicates,
                               const otsdb_batch* batch, otsdb_result* out);

/* ---- stage timing (bench roofline) ------------------------------------- */
/* When enabled, every query records HIP events around its pipeline stages
 * on the query's stream.  otsdb_prof_read returns, per stage, the summed
 * milliseconds and the number of launches since the last reset:
 * [0] k_bucketize  [1] k_transform  [2] k_group+k_combine  [3] k_prep
 * [4] k_compact+k_scan.  Synchronises the stream.                           */
otsdb_status otsdb_prof_enable(otsdb_ctx* ctx, int enable);
otsdb_status otsdb_prof_read(otsdb_ctx* ctx, double* ms, int64_t* launches,
                             int n, int reset);

/* ---- diagnostics ---------------------------------------------------------
 * Counters since the context was created (no reference counterpart: the
 * operator's view of which cells-fold kernel ran): out[0] cells folds run
 * with the uniform kernel (every kept series one value type and width),
 * out[1] with the general one, out[2] uniform folds that met a qualifier of
 * other flags and were re-run with the general kernel; out[3] passes over
 * the local key matrix and out[4] histogram passes of the last otsdb_sel_*
 * session.                                                                 */
otsdb_status otsdb_ctx_counters(otsdb_ctx* ctx, int64_t* out, int n);
/* Test hook: the one-pass compaction's epoch (1 .. 2^24 - 1, forward only)
 * the context's next call increments, so tests can drive it to its wrap.  */
otsdb_status otsdb_test_set_compact_epoch(otsdb_ctx* ctx, uint32_t epoch);

/* ---- synthetic workload generator (bench / tests) ----------- */
/* Generates the columnar batch of `n_series` series starting at global
 * series index `series0` directly in HBM.  Pass offsets=NULL first to get
 * the per-series point counts (written to `counts`, DEVICE [S]).            */
typedef struct {
  uint64_t seed;          /* 42                                              */
  int64_t t0_ms;          /* 1356998400000                                   */
  int64_t duration_ms;    /* 86400000 / 604800000                            */
  int64_t cadence_ms;     /* 10000                                           */
  int32_t kind;           /* 0 = gauge f64, 1 = gauge int64, 2 = counter int64 */
  int32_t flags;          /* 1 = whole-second phases (2-byte qualifiers)     */
} otsdb_gen_spec;

otsdb_status otsdb_gen_counts_device(otsdb_ctx* ctx, const otsdb_gen_spec* g,
                                     int64_t series0, int64_t n_series,
                                     int64_t* counts, void* hip_stream);
otsdb_status otsdb_gen_fill_device(otsdb_ctx* ctx, const otsdb_gen_spec* g,
                                   int64_t series0, int64_t n_series,
                                   const int64_t* offsets, int64_t* ts_ms,
                                   int64_t* val, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* OTSDB_AGG_H */
