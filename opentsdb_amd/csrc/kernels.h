// kernels.h — HIP kernels of the aggregation engine (gfx950, wave64).
//
// Pipeline for one downsampled query:
//   k_prep        per series: SpanGroup.add filter, seek/stop point bounds
//                 (binary search), first bucket beyond the window
//   k_bucketize   one wavefront per series streams its points from HBM
//                 (16-B loads, 2 points per lane) and reduces them into epoch
//                 aligned buckets with a segmented wave scan — Downsampler /
//                 ValuesInInterval semantics
//   k_transform   one wavefront per series sweeps its bucket row: fill policy
//                 (FillingDownsampler), RateSpan, and the per-series
//                 interpolation AggregationIterator applies (LERP/ZIM/MAX/
//                 MIN/PREV), marking each bucket real / interpolated / absent
//   k_group       one thread per (series chunk, bucket): the cross-series
//                 aggregator, sequential in SpanCmp order inside a chunk
//   k_combine     merges chunk partials in order, finalises, flags Infinity
//   k_compact1    per group: emitted buckets -> (ts, value) arrays (one pass)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "monoids.h"

namespace otsdb {

// row state of one (series, bucket)
enum : uint8_t {
  ST_ABSENT = 0,  // series does not contribute at this timestamp
  ST_INTERP = 1,  // contributes an interpolated / held value
  ST_REAL = 2,    // series has a real point here (emits the timestamp)
  ST_KEPT = 3     // transient: kept rate point (k_transform pass 1)
};

// device error word bits
enum : int {
  ERR_NONE_MULTI = 1,   // `none` fed >1 value  -> E_ILLEGAL_DATA
  ERR_INFINITY = 2,     // "Got Infinity"       -> E_ILLEGAL_STATE
  ERR_RATE_TS = 4,      // non-increasing ts    -> E_ILLEGAL_STATE
  ERR_SEL_TOO_BIG = 8,  // percentile group over the select limit
  ERR_X1_MASK = 16,     // interpolation toward x1 >= 2^44 ms (AssertionError
                        // in AggregationIterator.java:706-708, :776-778)
  ERR_RAW_DUP = 32,     // timestamps not increasing inside a raw span
  ERR_CAL_RANGE = 64,   // a point past the window outside the calendar table
  ERR_INTERNAL = 128,   // engine invariant broken          -> E_DEVICE
  // the storage-row query's verbatim speculation (Params.check_order) does
  // not hold: a series' points do not strictly increase, or a series is not
  // streamed whole -> the full compaction path runs instead
  ERR_NOT_SORTED = 1 << 22,
  ERR_SPEC_MISS = 1 << 23,
};

struct Params {
  int64_t gbase;         // timestamp of bucket 0
  int64_t interval;      // ms
  double inv_interval;   // 1.0 / interval
  int64_t nb;            // buckets per series row
  int64_t seek_ts;       // first point considered: ts >= seek_ts
  int64_t stop_ts;       // points with ts >= stop_ts are beyond the grid
  int64_t start_ms, end_ms;
  int64_t out_ts0;       // run_all: the single bucket's timestamp
  int64_t counter_max, reset_value;
  double fill_value;
  // previous point of RateSpan's first rate: (0, 0) normally; the
  // FillingDownsampler bucket align(start) when start is not aligned
  int64_t rate_origin_ts;
  double rate_origin_val;
  int32_t run_all, fill, rate, counter, drop_resets, interp;
  int32_t narrow;        // grid spans < 2^32 ms and interval < 2^31 ms
  double pct;            // percentile / 100.0 (PercentileAgg)
  int32_t pct_est;       // estimation type honoured by runLong: 0 LEGACY,
                         // 3 R_3, 7 R_7 (Aggregators.java:676-685)
  int32_t ds_sel;        // downsampling function: 0 monoid, 1 median,
                         // 2 percentile (k_ds_select)
  double ds_pct;         // its percentile / 100.0
  int32_t sentinel;      // rows written by the ring sink: k_bucketize left
                         // no state bytes; a bucket of [first, last] point
                         // bucket is absent iff its value is kAbsentBits
  int32_t _pad2;
  // calendar grid (otsdb_query_spec.cal_edges, device copy): bucket b is
  // [cal[b], cal[b+1]); valid indices cal_lo <= b < cal_n (cal_lo <= 0 when
  // the table starts before the grid's first bucket); null = fixed interval
  const int64_t* cal;
  int64_t cal_lo, cal_n;
  // rate queries with the RateSpan pass fused into k_bucketize's ring
  // flush: series the fused kernel hands back (a gap wider than its ring
  // inside one step) get redo[s] = 1; the fallback kernels, launched with
  // only_redo, skip every other series
  uint8_t* redo;
  int32_t only_redo;
  // buckets per window of the ordered fold (k_fold / k_fold_prep); 0: the
  // largest the aggregator state allows (fold_wb)
  int32_t fold_wb;
  // the cells query runs on storage rows taken verbatim (no compaction):
  // k_cells_prep flags a series not streamed whole, the cells fold a point
  // that does not follow its predecessor strictly (ERR_SPEC_MISS /
  // ERR_NOT_SORTED: the caller compacts and re-runs)
  int32_t check_order;
  // k_fold: every member context of a tile (at most this many members) is
  // loaded into LDS at workgroup start, all members at once; 0: each member
  // loads its own when a wavefront claims it
  int32_t fold_ctx;
};

// value bits of an absent bucket in sentinel rows: a signalling NaN, which
// no arithmetic produces and which the sink never stores for a real bucket
// (NaN results are stored as the canonical quiet NaN)
constexpr int64_t kAbsentBits = (int64_t)0x7FF4DEAD0BADF00DULL;

struct BatchDev {
  int64_t S;
  const int64_t* offsets;
  const int64_t* ts;
  const int64_t* val;
  const uint8_t* is_float;
  const uint8_t* series_float;
};

struct SeriesMeta {
  int64_t* lo;
  int64_t* hi;
  int32_t* kf;  // bucket of the first / last point in [lo, hi) (kf > kl:
  int32_t* kl;  // none) — the span sentinel rows are written over
  uint8_t* keep;
  uint8_t* of_has;  // bit 0: a bucket past the window (of_ts, of_val);
                    // rate queries, bits 1-2: kept rates after that
                    // bucket (0..2, capped), the first of them in of_rate
  int64_t* of_ts;
  double* of_val;
  double* of_rate;
};

struct Rows {
  double* val;     // [S * nb]
  uint8_t* state;  // [S * nb]
};

}  // namespace otsdb
