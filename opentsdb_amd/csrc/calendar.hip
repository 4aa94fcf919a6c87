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
// series' chain [pos, cend).  A point past the chain's last edge has no
// known bucket: harmless when an earlier point of the series already lies
// in a bucket at or past stage B's stop bound `stop_b` (the first bucket
// past the window, the only one a non-rate query reads there, is then
// complete) — it gets kFarTs, past everything; otherwise ERR_CAL_RANGE
// (E_UNSUPPORTED, like a global table's).  Rate queries walk further
// buckets past the window (rates_beyond): every such point is an error.
constexpr int64_t kFarTs = INT64_MAX / 4;
__global__ __launch_bounds__(256) void k_cal_vts(
    int64_t start_ms, int64_t stop_b, int rate, BatchDev B, AnchoredCal A,
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
      if (k >= pos && k + 1 < cend) {
        v = A.edges[k];
      } else if (k < pos || rate) {
        bad = 1;
      } else {
        // the series' last point inside the chain (points ascend)
        const int64_t q = lower_bound(B.ts, lo, i, A.edges[cend - 1]) - 1;
        if (q >= lo && A.edges[last_le(A.edges, pos, cend, B.ts[q])] >= stop_b)
          v = kFarTs;
        else
          bad = 1;
      }
    }
    vts[i] = v;
  }
  if (__ballot(bad) && lane == 0) atomicOr(err_word, ERR_CAL_RANGE);
}

// ---- FillingDownsampler over per-series grids (fill != none).
// The FillingDownsampler walks its OWN grid — the chain from
// previousInterval(start) up to previousInterval(end), advanced once when
// both coincide (FillingDownsampler.java:113-135) — and matches each
// expected timestamp against the interval timestamp of the series' own
// Downsampler (anchored at previousInterval(first point), Downsampler.java:
// 330-397): a series bucket whose start equals the expected timestamp is
// emitted, series buckets before it are consumed and dropped, an expected
// timestamp with no such bucket is filled (:175-272).  So a series bucket
// reaches the output iff its start is an edge of the filling grid FD.
// Stage A' keeps exactly those points (timestamps rewritten to their own
// bucket start, hence to an FD edge) in a compacted copy of the batch, with
// two points that keep the series' SpanGroup.add verdict and lie outside
// every bucket: start_ms - 1 (before the seek) and the stage-B table's end
// (past the stop bound).  Stage B is the filling calendar pipeline over FD.

DEV bool keep_series(const BatchDev& B, int64_t s, int64_t start_ms,
                     int64_t end_ms) {
  const int64_t p0 = B.offsets[s], p1 = B.offsets[s + 1];
  return p1 > p0 && B.ts[p0] <= end_ms && B.ts[p1 - 1] >= start_ms;
}

// is t an edge of the sorted grid fd[0, n)?
DEV bool on_grid(const int64_t* fd, int64_t n, int64_t t) {
  const int64_t k = last_le(fd, 0, n, t);
  return k >= 0 && fd[k] == t;
}

// one wavefront per series: cnt[s] = the points stage A' keeps (+ 2 for a
// kept series); the rewritten timestamps go to vts
__global__ __launch_bounds__(256) void k_cal_fill_count(
    int64_t start_ms, int64_t end_ms, BatchDev B, AnchoredCal A,
    const int64_t* __restrict__ lo_in, const int64_t* __restrict__ pos_in,
    const int64_t* __restrict__ cend_in, const int64_t* __restrict__ fd,
    int64_t nfd, int64_t* __restrict__ vts, uint8_t* __restrict__ on,
    int64_t* __restrict__ cnt, int* __restrict__ err_word) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= B.S) return;
  const int lane = threadIdx.x & 63;
  const int64_t p0 = B.offsets[s], p1 = B.offsets[s + 1];
  const int64_t lo = lo_in[s], pos = pos_in[s], cend = cend_in[s];
  int bad = 0, n = 0;
  for (int64_t i = p0 + lane; i < p1; i += 64) {
    bool k_on = false;
    int64_t v = start_ms - 1;
    if (i >= lo) {
      const int64_t k = last_le(A.edges, pos, cend, B.ts[i]);
      if (k < pos) {
        bad = 1;
      } else if (k + 1 < cend) {
        v = A.edges[k];
        k_on = on_grid(fd, nfd, v);
      } else if (A.edges[cend - 1] <= fd[nfd - 1]) {
        // past its chain's last edge, and that edge is not past the filling
        // grid: the point's bucket starts at that edge or at some later one
        // the table does not hold — it may be an FD edge (emitted) or not
        // (dropped), so the engine cannot tell (the caller's chains end too
        // early: E_UNSUPPORTED, as for a global table's)
        bad = 1;
      }
      // (otherwise the point's bucket starts past every FD edge: it is never
      // emitted, and nothing else reads it)
    }
    vts[i] = v;
    on[i] = k_on;
    n += k_on ? 1 : 0;
  }
  for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d);
  if (__ballot(bad) && lane == 0) atomicOr(err_word, ERR_CAL_RANGE);
  if (lane == 0) cnt[s] = keep_series(B, s, start_ms, end_ms) ? n + 2 : 0;
}

// one wavefront per series: the compacted copy (offsets = exclusive scan of
// cnt): start_ms - 1, the kept points in order, then t_end
__global__ __launch_bounds__(256) void k_cal_fill_write(
    int64_t start_ms, int64_t t_end, BatchDev B,
    const int64_t* __restrict__ vts, const uint8_t* __restrict__ on,
    const int64_t* __restrict__ offs, int64_t* __restrict__ ts_out,
    int64_t* __restrict__ val_out, uint8_t* __restrict__ isf_out) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= B.S) return;
  const int lane = threadIdx.x & 63;
  const int64_t o0 = offs[s], o1 = offs[s + 1];
  if (o1 == o0) return;
  const int64_t p0 = B.offsets[s], p1 = B.offsets[s + 1];
  const uint8_t sf = B.series_float ? B.series_float[s] : 1;
  if (lane == 0) {
    ts_out[o0] = start_ms - 1;
    ts_out[o1 - 1] = t_end;
    val_out[o0] = val_out[o1 - 1] = 0;
    if (isf_out) isf_out[o0] = isf_out[o1 - 1] = sf;
  }
  int64_t o = o0 + 1;
  for (int64_t i0 = p0; i0 < p1; i0 += 64) {
    const int64_t i = i0 + lane;
    const bool k = i < p1 && on[i];
    const uint64_t m = __ballot(k);
    if (k) {
      const int64_t d = o + __popcll(m & ((1ULL << lane) - 1));
      ts_out[d] = vts[i];
      val_out[d] = B.val[i];
      if (isf_out) isf_out[d] = B.is_float[i];
    }
    o += __popcll(m);
  }
}

}  // namespace otsdb
