// calendar.hip — per-series calendar grids (otsdb_query_spec.cal_anchors).
//
// The reference anchors every series' calendar at DateTime.previousInterval
// (its first point after the seek) and steps it with Calendar.add
// (ValuesInInterval.initializeIfNotDone / resetEndOfInterval,
// Downsampler.java:330-345, :383-397).  For specs like 7mc, 2wc or 6hc
// across a DST change those grids differ between series, so the bucket
// timestamps AggregationIterator merges are the union of every series' own
// bucket starts.
//
// Stage A (here): each point's timestamp becomes the start of the bucket it
// falls in on its series' own chain (points before the seek, and series
// SpanGroup.add drops, get start_ms - 1: the stage-B seek skips them and a
// series left without points is dropped there too).  Stage B is the
// ordinary calendar pipeline over U, the union of every chain's edges:
// each series' bucket starts are edges of U, every point of one own bucket
// carries the same rewritten timestamp, so U's buckets hold exactly the
// series' own buckets (the downsampling function sees the same values in
// the same order) and the fold's "emit iff some member has a real point,
// interpolate between the member's own real buckets" is the union merge.
#pragma once
// (included by engine.hip after kernels.hip)

namespace otsdb {

struct AnchoredCal {
  const int64_t* edges;        // chains, each ended by INT64_MAX
  const int64_t* anchors;      // ascending previousInterval values
  const int64_t* anchor_edge;  // chain edge of each anchor
  const int64_t* chain_end;    // index of each anchor's chain terminator
  int64_t n_anchors;
};

// (last_le: raw.hip, the largest index k in [a, b) with e[k] <= t)

// One thread per series: the SpanGroup.add range filter (SpanGroup.java:
// 321-338), the seek (first point >= the window's calendar seek,
// Downsampler.java:419-429) and the series' chain: the anchor
// previousInterval(first point) = the largest anchor <= it.
__global__ void k_cal_anchor(int64_t start_ms, int64_t end_ms,
                             int64_t seek_ts, BatchDev B, AnchoredCal A,
                             int64_t* __restrict__ lo_out,
                             int64_t* __restrict__ pos_out,
                             int64_t* __restrict__ cend_out,
                             int* __restrict__ err_word) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= B.S) return;
  const int64_t p0 = B.offsets[s], p1 = B.offsets[s + 1];
  const bool keep = p1 > p0 && B.ts[p0] <= end_ms && B.ts[p1 - 1] >= start_ms;
  int64_t lo = p1, pos = 0, cend = 0;
  if (keep) {
    lo = lower_bound_interp(B.ts, p0, p1, seek_ts);
    if (lo < p1) {
      const int64_t j = last_le(A.anchors, 0, A.n_anchors, B.ts[lo]);
      if (j < 0) {
        atomicOr(err_word, ERR_CAL_RANGE);
        lo = p1;
      } else {
        pos = A.anchor_edge[j];
        cend = A.chain_end[j];
      }
    }
  }
  lo_out[s] = lo;
  pos_out[s] = pos;
  cend_out[s] = cend;
}

// One wavefront per series, lanes over its points: the bucket start on the
// series' chain [pos, cend) (a point past the chain's last edge has no
// known bucket end: ERR_CAL_RANGE, E_UNSUPPORTED like a global table's).
__global__ __launch_bounds__(256) void k_cal_vts(
    int64_t start_ms, BatchDev B, AnchoredCal A,
    const int64_t* __restrict__ lo_in, const int64_t* __restrict__ pos_in,
    const int64_t* __restrict__ cend_in, int64_t* __restrict__ vts,
    int* __restrict__ err_word) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= B.S) return;
  const int lane = threadIdx.x & 63;
  const int64_t p0 = B.offsets[s], p1 = B.offsets[s + 1];
  const int64_t lo = lo_in[s], pos = pos_in[s], cend = cend_in[s];
  int bad = 0;
  for (int64_t i = p0 + lane; i < p1; i += 64) {
    int64_t v = start_ms - 1;
    if (i >= lo) {
      const int64_t k = last_le(A.edges, pos, cend, B.ts[i]);
      if (k < pos || k + 1 >= cend) bad = 1;
      else v = A.edges[k];
    }
    vts[i] = v;
  }
  if (__ballot(bad) && lane == 0) atomicOr(err_word, ERR_CAL_RANGE);
}

}  // namespace otsdb
