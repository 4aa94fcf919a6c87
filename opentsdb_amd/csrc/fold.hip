// fold.hip — the ordered group fold: downsample, per-series contribution
// (real bucket, interpolation inside gaps, FillingDownsampler fill) and the
// cross-series aggregator of one chunk of a group's members in ONE pass over
// the points, with the aggregator fed in SpanCmp order.
//
// Reference chain replaced (for every non-rate, non-selection query):
//   Downsampler / FillingDownsampler (Downsampler.java:162-228,
//   FillingDownsampler.java:172-298) -> AggregationIterator.next /
//   nextDoubleValue over the group's spans in span order
//   (AggregationIterator.java:514-567, :735-797) -> Aggregator.runDouble.
//
// Layout.  One workgroup per (chunk of <= 256 members of one group, window of
// WB buckets).  Its four wavefronts claim the chunk's members in member order
// and stream each member's points of the window (k_bucketize_k's reduce_step:
// K points per lane, DPP segmented scan).  Closed buckets go to a per-wave
// LDS ring; each flush turns a run of final buckets into the member's
// contributions and pushes them into the window's LDS aggregator states.
//
// Order.  Java pushes the values of one timestamp in span order, and the
// double sums / Welford steps are order-sensitive, so member i may push into
// bucket b only after member i-1 has pushed there.  Each member publishes a
// progress mark (LDS, one int per member): "all my pushes below p are done",
// and a member's mark is only ever raised after its own predecessor's
// effective mark reached the same point; a finished member publishes DONE
// and defers to its predecessor.  A flush up to bucket L waits until the
// nearest unfinished predecessor's mark is >= L.  Members are claimed in
// increasing order and a wavefront runs one member at a time, so the chain
// of waits always ends at a running member with a lower index: no deadlock.
// The results are the reference's SpanCmp-order sums, deterministic and
// independent of wavefront timing.
//
// Gaps.  A bucket after a member's latest real bucket stays pending until
// the next real bucket arrives (its interpolation needs both ends,
// AggregationIterator.java:772-793); the member's mark stops at the pending
// gap, so its successors wait for it.  Window edges: k_fold_prep gives each
// (series, inner window boundary) the first point of the window and the
// series' real buckets either side of it, so windows are independent.
#pragma once
#include "launch.h"

namespace otsdb {

// Every loop of the fold is bounded: past an absurd trip count it reports
// ERR_INTERNAL (E_DEVICE) and stops, so a broken invariant can never keep a
// wavefront spinning (debug builds also print where).
#ifdef OTSDB_DEBUG_SYNC
#define FOLD_GUARD(cnt, lim, err, ...)                 \
  if (++cnt > (lim)) {                                 \
    if (LANE == 0) {                                   \
      printf(__VA_ARGS__);                             \
      atomicOr(err, ERR_INTERNAL);                     \
    }                                                  \
    break;                                             \
  }
#else
#define FOLD_GUARD(cnt, lim, err, ...)                 \
  if (++cnt > (lim)) {                                 \
    if (LANE == 0) atomicOr(err, ERR_INTERNAL);        \
    break;                                             \
  }
#endif

#ifndef OTSDB_FOLD_FL
#define OTSDB_FOLD_FL 32
#endif
#ifndef OTSDB_FOLD_WAVES
#define OTSDB_FOLD_WAVES 1
#endif
#ifndef OTSDB_CELLS_FOLD_WAVES  // the cells fold: at most 128 VGPRs (23.7 vs 25.0 ms at 3 waves, C2)
#define OTSDB_CELLS_FOLD_WAVES 4
#endif
constexpr int FOLD_WIN = 128;  // per-wave ring of closed bucket values
#ifndef OTSDB_FOLD_WG_WAVES  // wavefronts per fold workgroup (A/B builds)
#define OTSDB_FOLD_WG_WAVES 4
#endif
constexpr int FOLD_WG = OTSDB_FOLD_WG_WAVES;
constexpr int FOLD_THREADS = 64 * FOLD_WG;
constexpr int FOLD_FL = OTSDB_FOLD_FL;  // flush once this many buckets are final
constexpr int32_t kProgDone = INT32_MAX;

// k_fold_prep: one thread per (series, inner boundary).  The boundary
// buckets' values are folded sequentially (Java order) from the points.
// (series s, boundary j) given the series' k_prep bounds
template <class M>
DEV void fold_prep_one(const Params& P, const BatchDev& B, int64_t s,
                       int64_t j, int64_t nbd, int64_t WB, bool keep,
                       int64_t lo_s, int64_t hi_s, WinCtx* __restrict__ wc) {
  WinCtx c{0, INT64_MIN, 0.0, INT64_MIN, 0.0};
  const int64_t lo = keep ? lo_s : 0, hi = keep ? hi_s : 0;
  if (lo >= hi) {
    c.bnd = lo;
    wc[s * nbd + j - 1] = c;
    return;
  }
  const int sf = B.series_float ? (int)B.series_float[s] : 1;
  const int64_t p = lower_bound_near(B.ts, lo, hi, bucket_ts(P, j * WB));
  c.bnd = p;
  int err = 0;
  // the buckets either side, reduced in point order.  The 8 points either
  // side of the boundary are read in ONE round of loads (a bucket of up to 8
  // points needs nothing else; longer ones continue point-chunk by chunk):
  // each dependent load round costs this latency-bound kernel ~2 us
  constexpr int C8 = 8;
  int64_t t[2 * C8], v[2 * C8];
#pragma unroll
  for (int u = 0; u < 2 * C8; ++u) {
    const int64_t i = p - C8 + u;
    const bool in = i >= lo && i < hi;
    t[u] = in ? B.ts[i] : (i < lo ? INT64_MIN : INT64_MAX);
    v[u] = in ? B.val[i] : 0;
  }
  if (p > lo) {
    const int64_t k = bucket_of(P, t[C8 - 1]);
    const int64_t bt = bucket_ts(P, k);
    M st = M::init();
    // the bucket starts before the chunk: its earlier points first
    if (t[0] >= bt && p - C8 > lo) {
      const int64_t q = lower_bound_interp(B.ts, lo, p - C8, bt);
      for (int64_t i0 = q; i0 < p - C8; i0 += C8) {
        int64_t w[C8];
#pragma unroll
        for (int u = 0; u < C8; ++u) w[u] = i0 + u < p - C8 ? B.val[i0 + u] : 0;
#pragma unroll
        for (int u = 0; u < C8; ++u)
          if (i0 + u < p - C8) st.push(point_value(B, i0 + u, w[u], sf));
      }
    }
#pragma unroll
    for (int u = 0; u < C8; ++u)
      if (t[u] >= bt && t[u] != INT64_MAX)
        st.push(point_value(B, p - C8 + u, v[u], sf));
    c.prev_ts = bt;
    c.prev_val = st.finish(&err);
  }
  if (p < hi) {
    const int64_t k = bucket_of(P, t[C8]);
    const int64_t bt = bucket_ts(P, k), be = bucket_ts(P, k + 1);
    M st = M::init();
    bool more = true;
#pragma unroll
    for (int u = C8; u < 2 * C8; ++u) {
      more = more && t[u] < be;  // (INT64_MAX past hi)
      if (more) st.push(point_value(B, p - C8 + u, v[u], sf));
    }
    for (int64_t i0 = p + C8; more && i0 < hi; i0 += C8) {
      int64_t tt[C8], w[C8];
#pragma unroll
      for (int u = 0; u < C8; ++u) {
        const bool in = i0 + u < hi;
        tt[u] = in ? B.ts[i0 + u] : INT64_MAX;
        w[u] = in ? B.val[i0 + u] : 0;
      }
#pragma unroll
      for (int u = 0; u < C8; ++u) {
        more = more && tt[u] < be;
        if (more) st.push(point_value(B, i0 + u, w[u], sf));
      }
    }
    c.next_ts = bt;
    c.next_val = st.finish(&err);
  }
  wc[s * nbd + j - 1] = c;
}

template <class M>
__global__ __launch_bounds__(256) void k_fold_prep(Params P, BatchDev B,
                                                   SeriesMeta SM, int64_t NW,
                                                   int64_t WB,
                                                   WinCtx* __restrict__ wc) {
  const int64_t nbd = NW - 1;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t s = idx / nbd;
  if (s >= B.S) return;
  const bool keep = SM.keep[s];
  fold_prep_one<M>(P, B, s, idx - s * nbd + 1, nbd, WB, keep, SM.lo[s],
                   SM.hi[s], wc);
}

// k_prep and k_fold_prep in one launch for small queries (C1: 1,000 series
// x 7 boundaries; one launch and one dependent round of SeriesMeta loads
// fewer): every (series, boundary) thread finds the series' bounds itself,
// the series' first thread also does the rest of k_prep
template <class M>
__global__ __launch_bounds__(256) void k_prep_fold(Params P, BatchDev B,
                                                   SeriesMeta SM, int* err_word,
                                                   int64_t NW, int64_t WB,
                                                   WinCtx* __restrict__ wc) {
  const int64_t nbd = NW - 1;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t s = idx / nbd;
  if (s >= B.S) return;
  const int64_t j0 = idx - s * nbd;
  bool keep;
  int64_t lo, hi;
  prep_series<M>(P, B, SM, err_word, s, j0 == 0, &keep, &lo, &hi);
  fold_prep_one<M>(P, B, s, j0 + 1, nbd, WB, keep, lo, hi, wc);
}

// One wavefront's view of the fold (wave-uniform except the pointers).
// Bucket indices are 32-bit (run_pipeline rejects wider grids).
template <class A>
struct FoldSink {
  A* st;              // LDS aggregator states of the window
  uint8_t* emit;      // LDS: some member has a real point there
  double* ring;       // this wave's LDS ring
  int32_t* prog;      // LDS progress marks of the chunk's members
  int* err;           // device error word (watchdog)
  int32_t mi;         // this member's index in the chunk
  int32_t eff;        // cached effective mark of the predecessors
  int32_t W0, W1;     // window buckets [W0, W1)
  int32_t flushed;    // buckets below are pushed or pending
  int32_t pend;       // start of the pending gap, -1: none
  int64_t x0;         // the latest real bucket before `pend`
  double y0;
};

// Waits until every member before this one has pushed all its contributions
// to buckets < need.
template <class A>
DEV void fold_wait(FoldSink<A>& F, int32_t need) {
#ifdef OTSDB_FOLD_NOWAIT  // debug build: no ordering
  return;
#endif
  if (F.eff >= need) return;
  const int lane = LANE;
  for (uint32_t spin = 0;; ++spin) {
    int32_t e = INT32_MAX;  // no unfinished predecessor
    for (int j0 = F.mi - 1; j0 >= 0; j0 -= 64) {
      const int j = j0 - lane;
      const int32_t v =
          j >= 0 ? __hip_atomic_load(&F.prog[j], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP)
                 : kProgDone;
      const uint64_t nd = __ballot(v != kProgDone);
      if (nd) {  // nearest unfinished predecessor (lowest lane)
        e = __builtin_amdgcn_readlane(v, __builtin_ctzll(nd));
        break;
      }
    }
    F.eff = e;
    if (e >= need) break;
    if (spin > (1u << 24)) {
      // watchdog: an invariant is broken (never expected); report it and
      // let the grid drain instead of spinning forever
      if (lane == 0) atomicOr(F.err, ERR_INTERNAL);
      F.eff = INT32_MAX;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <class A>
DEV void fold_publish(FoldSink<A>& F, int32_t p) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (LANE == 0)
    __hip_atomic_store(&F.prog[F.mi], p, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}

// pushes the member's interpolated contribution to every bucket of [a, e)
// (between its real buckets x0 -> x1, or toward the point past the window)
template <class A>
DEV void fold_fill_gap(const Params& P, FoldSink<A>& F, int32_t a, int32_t e,
                       int64_t x1, double y1) {
  const int lane = LANE;
  for (int32_t j0 = a; j0 < e; j0 += 64) {
    const int32_t b = j0 + lane;
    if (b < e)
      F.st[b - F.W0].push(
          interp_value(P.interp, bucket_ts(P, b), F.x0, F.y0, x1, y1));
  }
}

// Turns the ring's buckets [flushed, limit) (all final) into contributions.
#ifdef OTSDB_FLUSH_NOINLINE  // tuning builds: the flush as a real call
#define FLUSH_FN __device__ __attribute__((noinline))
#else
#define FLUSH_FN DEV
#endif
template <class A>
FLUSH_FN void fold_flush(const Params& P, FoldSink<A>& F, int32_t limit) {
  if (limit <= F.flushed) return;
#ifdef OTSDB_FOLD_ABL_NOFLUSH  // timing ablation: no contributions
  F.flushed = limit;
  return;
#endif
  fold_wait(F, limit);
  const int lane = LANE;
  const bool fill = P.fill != 0;
  int dbg_n = 0;
  for (int32_t f = F.flushed; f < limit; f += 64) {
    FOLD_GUARD(dbg_n, 1 << 26, F.err, "flush loop mi=%d f=%d limit=%d\n", F.mi, f, limit)
    const int32_t b = f + lane;
    const bool inb = b < limit;
    double v = absent_value();
    if (inb) {
      const int i = b & (FOLD_WIN - 1);
      v = F.ring[i];
      F.ring[i] = absent_value();
    }
    const bool real = inb && __double_as_longlong(v) != kAbsentBits;
    if (fill) {  // FillingDownsampler: every bucket is a point
      if (inb) {
        F.st[b - F.W0].push(real ? v : P.fill_value);
        F.emit[b - F.W0] = 1;
      }
      continue;
    }
    const uint64_t rm = __ballot(real);
    if (!rm) continue;  // pending gap goes on (or absent before any real)
    if (rm == __ballot(inb)) {
      // every bucket of the run is real (dense series): no gap inside it
      if (F.pend >= 0 && F.pend < f)
        fold_fill_gap(P, F, F.pend, f, bucket_ts(P, f), readlane_d(v, 0));
      if (inb) {
        F.st[b - F.W0].push(v);
        F.emit[b - F.W0] = 1;
      }
      const int lr = 63 - __builtin_clzll(rm);
      F.x0 = bucket_ts(P, f + lr);
      F.y0 = readlane_d(v, lr);
      F.pend = f + lr + 1;
      continue;
    }
    const int fr = __builtin_ctzll(rm);
    const double vfr = readlane_d(v, fr);
    if (F.pend >= 0) fold_fill_gap(P, F, F.pend, f + fr, bucket_ts(P, f + fr), vfr);
    // gaps inside the chunk: both ends are lanes of this chunk
    const uint64_t below = rm & ((1ULL << lane) - 1);
    const uint64_t above = lane == 63 ? 0ULL : (rm & (~0ULL << (lane + 1)));
    const int pl = below ? 63 - __builtin_clzll(below) : 0;
    const int nl = above ? __builtin_ctzll(above) : 0;
    const double yp = __shfl(v, pl), yn = __shfl(v, nl);
    if (real) {
      F.st[b - F.W0].push(v);
      F.emit[b - F.W0] = 1;
    } else if (inb && below && above) {
      F.st[b - F.W0].push(interp_value(P.interp, bucket_ts(P, b),
                                       bucket_ts(P, f + pl), yp,
                                       bucket_ts(P, f + nl), yn));
    }
    const int lr = 63 - __builtin_clzll(rm);
    F.x0 = bucket_ts(P, f + lr);
    F.y0 = readlane_d(v, lr);
    F.pend = f + lr + 1;
  }
  F.flushed = limit;
  fold_publish(F, (fill || F.pend < 0) ? limit : F.pend);
}

// wave-uniform copies (SGPRs): the member loop and the stream loop branch on
// these, so the compiler must see them as uniform, not as per-lane values
DEV int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
DEV int64_t uni(int64_t x) { return readlane_l(x, 0); }
DEV double uni(double x) { return readlane_d(x, 0); }

// sum of a per-lane count over the wavefront
DEV int wave_sum(int x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
  return x;
}

// timestamp of point `idx` (wave-uniform): a scalar load.  Only steps that
// are not full (a member's first / last step, a cut) need it; picking the
// element out of t[] by a computed index would put t[] in scratch memory.
DEV int64_t point_ts(const BatchDev& B, int64_t idx) { return uni(B.ts[idx]); }

// bucket of a wave-uniform timestamp
DEV int32_t fold_bucket(const Params& P, int64_t ts) {
  return P.narrow ? bucket_narrow(P, ts) : (int32_t)bucket_of(P, ts);
}

// One member's points [pa, pb) of the window (the member's wave).
// Context: the latest real bucket before the window (has_prev: x0/y0) and
// where its contribution goes past its last real bucket of the window
// (has_next: toward (nx, ny) — the next real bucket, or the point past the
// grid, AggregationIterator.java:760-775).
// A member's window context, kept in LDS while its points stream (only the
// member prologue and the tail read it: not held in SGPRs across the loop).
struct FoldMember {
  int64_t pa, pb;    // its points of the window
  int64_t px, nx;    // previous / next real bucket timestamps
  double py, ny;
  int32_t kept, sf, has_prev, has_next;
};
// the dynamic LDS a k_fold workgroup may take and still run 4 to a CU (160 KB)
// beside its static arrays (rings, marks, contexts: ~5.6 KB)
constexpr size_t kFoldDynBudget = 40960 - 6144;

template <class A>
DEV void fold_member_init(const Params& P, FoldSink<A>& F,
                          const FoldMember* mc) {
  F.flushed = F.W0;
  F.pend = uni(mc->has_prev) ? F.W0 : -1;
  F.x0 = uni(mc->px);
  F.y0 = uni(mc->py);
}

// A member's buckets after its last point: FillingDownsampler fill, or the
// interpolation toward the point past the window.
template <class A>
DEV void fold_member_tail(const Params& P, FoldSink<A>& F,
                          const FoldMember* mc) {
  const int lane = LANE;
  if (P.fill) {
    if (F.flushed < F.W1) {
      fold_wait(F, F.W1);
      for (int32_t j0 = F.flushed; j0 < F.W1; j0 += 64) {
        const int32_t b = j0 + lane;
        if (b < F.W1) {
          F.st[b - F.W0].push(P.fill_value);
          F.emit[b - F.W0] = 1;
        }
      }
    }
  } else if (F.pend >= 0 && F.pend < F.W1 && uni(mc->has_next)) {
    fold_wait(F, F.W1);
    fold_fill_gap(P, F, F.pend, F.W1, uni(mc->nx), uni(mc->ny));
  }
}

template <class M, class A, int K>
DEV void fold_member(const Params& P, const BatchDev& B, FoldSink<A>& F,
                     const FoldMember* mc) {
  constexpr int PTS = 64 * K;
  const int lane = LANE;
  const bool kept = uni(mc->kept) != 0;
  const int sf = uni(mc->sf);
  const int64_t pa = uni(mc->pa), pb = uni(mc->pb);
  fold_member_init(P, F, mc);
  if (!kept) return;  // contributes nowhere (SpanGroup.add dropped it)
  RowSink S{nullptr, nullptr, F.ring, FOLD_WIN - 1, 0, 0, 0, 0};
  int err = 0;
  int carry_key = INT32_MIN;
  M carry = M::init();
  int64_t lo_eff = pa;
  int32_t prev_hi = -1;  // bucket of the previous step's last point
  int dbg_n = 0;
  L2Touch pt_, pv_;
  // (no points in the window: no step — an aligned base below an odd pa
  // would stream the point before the window and read bucket bounds past it)
  for (int64_t base = pa & ~(int64_t)1; pa < pb && base < pb;) {
    FOLD_GUARD(dbg_n, 1 << 30, F.err, "stream loop mi=%d base=%ld pa=%ld pb=%ld\n", F.mi, (long)base, (long)pa, (long)pb)
    const int64_t i0 = base + (int64_t)K * lane;
    int64_t t[K], v[K];
    if (i0 + K <= pb) {
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        const ll2_t tt = *reinterpret_cast<const ll2_t*>(B.ts + i0 + j);
        const ll2_t vv = *reinterpret_cast<const ll2_t*>(B.val + i0 + j);
        t[j] = tt.x; t[j + 1] = tt.y;
        v[j] = vv.x; v[j + 1] = vv.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        t[j] = (i0 + j < pb) ? B.ts[i0 + j] : 0;
        v[j] = (i0 + j < pb) ? B.val[i0 + j] : 0;
      }
    }
    if (OTSDB_PF_FOLD) {
      pt_.retire();
      pv_.retire();
      if (base + (OTSDB_PF_FOLD + 1) * PTS <= pb) {
        pt_.touch(B.ts + i0 + OTSDB_PF_FOLD * PTS);
        pv_.touch(B.val + i0 + OTSDB_PF_FOLD * PTS);
      }
    }
#ifdef OTSDB_FOLD_ABL_STREAM  // timing ablation: the loads alone
    {
      int64_t x = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) x ^= t[j] + v[j];
      if (x == 42) F.emit[0] = 1;
      base += PTS;
      continue;
    }
#endif
    // buckets below the open one are final (every bucket of the previous
    // step when it ended on a bucket boundary): drain them while this
    // step's loads are in flight (nothing below reads t[] / v[])
    const bool carry_ok = carry_key >= 0 && carry_key < P.nb;
    int32_t limit = carry_ok ? carry_key : prev_hi + 1;
#ifndef OTSDB_FOLD_FLUSH_LATE
    if (limit - F.flushed >= FOLD_FL) fold_flush(P, F, limit);
#endif
    const bool full = base >= lo_eff && base + PTS <= pb;
    const int64_t last_i = (base + PTS < pb ? base + PTS : pb) - 1;
    // the step's last bucket: lane 63's last point when the step is full
    const int32_t k_hi = fold_bucket(
        P, full ? readlane_l(t[K - 1], 63) : point_ts(B, last_i));
    int64_t hi_step = pb;
    if (k_hi >= F.flushed + FOLD_WIN) {
      // ring pressure (a gap or sparse buckets inside the step): close the
      // open bucket if the step starts past it, drain, and cut the step
      // where the ring ends (a bucket boundary) if it still does not fit
      const int64_t first_i = base > lo_eff ? base : lo_eff;
      const int32_t k_first = fold_bucket(P, point_ts(B, first_i));
      if (carry_ok && carry_key < k_first) {
        if (lane == 0) S.put(carry_key, carry.finish(&err));
        carry_key = INT32_MIN;
        limit = k_first;
      } else if (!carry_ok) {
        limit = k_first;
      }
      fold_flush(P, F, limit);
      if (k_hi >= F.flushed + FOLD_WIN) {
        const int64_t T = bucket_ts(P, F.flushed + FOLD_WIN);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < K; ++j)
          cnt += (i0 + j >= first_i && i0 + j <= last_i && t[j] < T) ? 1 : 0;
        hi_step = first_i + uni((int32_t)wave_sum(cnt));
      }
    }
#ifdef OTSDB_FOLD_ABL_NOREDUCE  // timing ablation: stream + ring bookkeeping
    {
      int64_t x = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) x ^= t[j] + v[j];
      if (x == 42) F.emit[0] = 1;
    }
#else
    reduce_step<M, K, 1>(P, B, sf, lo_eff, hi_step, base, i0, t, v, S, err,
                         carry_key, carry);
#endif
    if (hi_step < pb) {
      prev_hi = fold_bucket(P, point_ts(B, hi_step - 1));
      lo_eff = hi_step;
      base = hi_step & ~(int64_t)1;
    } else {
      prev_hi = k_hi;
      base += PTS;
    }
#ifdef OTSDB_FOLD_FLUSH_LATE
    {
      const int32_t lim = (carry_key >= 0 && carry_key < P.nb) ? carry_key
                                                                 : prev_hi + 1;
      if (lim - F.flushed >= FOLD_FL) fold_flush(P, F, lim);
    }
#endif
  }
  if (carry_key >= 0 && carry_key < P.nb && lane == 0)
    S.put(carry_key, carry.finish(&err));
  if (prev_hi >= 0) fold_flush(P, F, prev_hi + 1);
  // the window's remaining buckets
  fold_member_tail(P, F, mc);
}

// the kernel's own arguments the member loop and the finalisation read,
// stashed in LDS so they do not occupy SGPRs across the point stream
struct FoldKernel {
  SeriesMeta SM;
  const int64_t* members;
  const WinCtx* wc;
  const uint8_t* series_float;
  int64_t nbd, win, m0, m1, g, t;
  Packed* partial;
  uint8_t* tile_emit;
  double* out_val;
  uint8_t* out_emit;
  int32_t fin;
};

// k_fold: see the file header.  Single-chunk groups finish here (out_val /
// out_emit); chunks of larger groups (and every chunk with always_partial,
// the multi-GPU partials) leave their window of partials for k_combine.
// A cells member's stream context (CELLS = 1, cellfold.hip), kept in LDS
struct CellsMember {
  int64_t qb;     // qualifier byte offset of the series' point 0
  int64_t vb0;    // value byte offset of its first row
  int64_t vcur;   // value byte offset of point pa
  int64_t rlo;    // row holding point pa
  int64_t r1;     // one past the series' last row
  int64_t qend, vend;  // readable bytes of the pools
  int32_t qw, vl0;
  int32_t uf;     // the uniform series' flags nibble (CellsFold.uf)
};

template <class M, class A, int K, int QW>
DEV void fold_member_cells(const Params& P, const CellsDev& C, FoldSink<A>& F,
                           const FoldMember* mc, const CellsMember* cm);
template <class M, class A, int K, int QW>
DEV void fold_member_cells_u(const Params& P, const CellsDev& C, FoldSink<A>& F,
                             const FoldMember* mc, const CellsMember* cm);

template <class M, class A, int K, int CELLS = 0>
__global__ __launch_bounds__(FOLD_THREADS, CELLS ? OTSDB_CELLS_FOLD_WAVES
                                        : OTSDB_FOLD_WAVES) void k_fold(
    Params P, BatchDev B, SeriesMeta SM, int64_t n_tiles,
    const int64_t* __restrict__ tile_g, const int64_t* __restrict__ tile_m0,
    const int64_t* __restrict__ tile_m1,
    const uint8_t* __restrict__ tile_single,
    const int64_t* __restrict__ members, const WinCtx* __restrict__ wc,
    int64_t NW, Packed* __restrict__ partial, uint8_t* __restrict__ tile_emit,
    double* __restrict__ out_val, uint8_t* __restrict__ out_emit,
    int* err_word, int always_partial, CellsFold CF) {
  constexpr int WB = fold_wb<A>();
  // the window's aggregator states and emit flags: dynamic LDS sized for
  // min(WB, nb) buckets (fold_lds_bytes), so a short grid leaves room for
  // more workgroups per CU
  extern __shared__ __attribute__((aligned(16))) unsigned char fold_dyn[];
  A* st = reinterpret_cast<A*>(fold_dyn);
  uint8_t* emit = fold_dyn + fold_lds_states<A>(P);
  __shared__ double ring[FOLD_WG][FOLD_WIN];
  __shared__ int32_t prog[256];
  __shared__ int s_next;
  __shared__ FoldKernel kc;
  __shared__ FoldMember mc[FOLD_WG];
  __shared__ CellsMember cm[CELLS ? FOLD_WG : 1];
  const int tid = threadIdx.x, lane = LANE, w = tid >> 6;
  const int64_t nb = P.nb;
  int32_t W0, W1;
  {
    const int64_t t = (int64_t)blockIdx.x % n_tiles;
    const int64_t win = (int64_t)blockIdx.x / n_tiles;
    const int64_t wb = fold_window<A>(P);  // <= WB
    W0 = (int32_t)(win * wb);
    W1 = (int32_t)((W0 + wb < nb) ? W0 + wb : nb);
    if (tid == 0) {
      kc.SM = SM;
      kc.members = members;
      kc.wc = wc;
      kc.series_float = B.series_float;
      kc.nbd = NW - 1;
      kc.win = win;
      kc.m0 = tile_m0[t];
      kc.m1 = tile_m1[t];
      kc.g = tile_g[t];
      kc.t = t;
      kc.partial = partial;
      kc.tile_emit = tile_emit;
      kc.out_val = out_val;
      kc.out_emit = out_emit;
      kc.fin = tile_single[t] && !always_partial;
      // a cells fold whose prep already sent the batch to the generic path
      // (mixed qualifier widths: the engine rewrites them and runs again)
      s_next = (CELLS && (__hip_atomic_load(err_word, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT) &
                          ERR_CELLS_GENERIC)) ? -1 : 0;
    }
  }
  const int nw = W1 - W0;
  for (int b = tid; b < nw; b += FOLD_THREADS) {
    st[b] = A::init();
    emit[b] = 0;
  }
  for (int j = tid; j < 256; j += FOLD_THREADS) prog[j] = 0;
  for (int i = lane; i < FOLD_WIN; i += 64) ring[w][i] = absent_value();
  __syncthreads();
  if (CELLS && s_next < 0) return;  // (block-uniform)
  int dbg_n = 0;
  FoldSink<A> F{st, emit, ring[w], prog, err_word, 0, 0, W0, W1, W0, -1, 0, 0.0};
  // a member's window context (k_prep / k_fold_prep's results for series s)
  auto member_ctx = [&](int64_t s) {
    const SeriesMeta& sm = kc.SM;
    const int64_t nbd = kc.nbd, win = kc.win;
    FoldMember m;
    m.kept = sm.keep[s] != 0;
    m.pa = m.kept ? sm.lo[s] : 0;
    m.pb = m.kept ? sm.hi[s] : 0;
    m.has_prev = m.has_next = 0;
    m.px = m.nx = 0;
    m.py = m.ny = 0.0;
    if (win > 0) {
      const WinCtx& c = kc.wc[s * nbd + win - 1];
      m.pa = c.bnd;
      if (c.prev_ts != INT64_MIN) {
        m.has_prev = 1;
        m.px = c.prev_ts;
        m.py = c.prev_val;
      }
    }
    if (win < nbd) {
      const WinCtx& c = kc.wc[s * nbd + win];
      m.pb = c.bnd;
      if (c.next_ts != INT64_MIN) {
        m.has_next = 1;
        m.nx = c.next_ts;
        m.ny = c.next_val;
      }
    }
    if (!m.has_next && sm.of_has[s]) {  // toward the point past the grid
      m.has_next = 1;
      m.nx = sm.of_ts[s];
      m.ny = sm.of_val[s];
    }
    m.sf = kc.series_float ? (int)kc.series_float[s] : 1;
    return m;
  };
  // tiles of at most P.fold_ctx members (the host sized the dynamic LDS for
  // them): every context loaded here at once — two dependent load rounds per
  // workgroup instead of two per member on the path of each wavefront
  const int64_t n_mem = kc.m1 - kc.m0;
  const bool ctx_on = !CELLS && P.fold_ctx > 0 && n_mem <= P.fold_ctx;
  FoldMember* ctx = reinterpret_cast<FoldMember*>(fold_dyn + fold_lds_bytes<A>(P));
  if (ctx_on) {
    for (int64_t j = tid; j < n_mem; j += FOLD_THREADS) ctx[j] = member_ctx(kc.members[kc.m0 + j]);
    __syncthreads();
  }
  for (;;) {
    int i = 0;
    if (lane == 0) i = atomicAdd(&s_next, 1);
    i = __builtin_amdgcn_readlane(i, 0);
    const int64_t m0 = uni(kc.m0);
    if (m0 + i >= uni(kc.m1)) break;
    FOLD_GUARD(dbg_n, 1 << 20, err_word, "claim loop i=%d\n", i)
    F.mi = i;
    F.eff = 0;
    // the member's window context, lane 0 -> LDS (preloaded: a copy)
    if (lane == 0 && ctx_on) {
      mc[w] = ctx[i];
    } else if (lane == 0) {
      const int64_t s = kc.members[m0 + i];
      mc[w] = member_ctx(s);
      if (CELLS) {
        const int64_t nbd = kc.nbd, win = kc.win;
        CellsMember c;
        c.qb = CF.C.qual_off[CF.series_row[s]];
        c.vb0 = CF.C.val_off[CF.series_row[s]];
        c.r1 = CF.series_row[s + 1];
        if (win > 0) {  // the cursor at the window's first point
          const int64_t o = s * nbd + win - 1;
          c.rlo = CF.wrlo[o];
          c.vcur = CF.wvlo[o];
          c.vl0 = CF.wvl0[o];
        } else {
          c.rlo = CF.rlo[s];
          c.vcur = CF.vlo[s];
          c.vl0 = CF.vl0[s];
        }
        c.qw = CF.qw[s];
        c.uf = CF.uf ? CF.uf[s] : 0xFF;
        c.qend = CF.C.qual_off[CF.C.R];
        c.vend = CF.C.val_off[CF.C.R];
        cm[CELLS ? w : 0] = c;
      }
    }
    if constexpr (CELLS >= 8)  // every kept series uniform (k_cells_uniform)
      fold_member_cells_u<M, A, K, CELLS - 8>(P, CF.C, F, &mc[w], &cm[w]);
    else if constexpr (CELLS != 0)
      fold_member_cells<M, A, K, CELLS == 1 ? 0 : CELLS>(P, CF.C, F, &mc[w], &cm[w]);
    else
      fold_member<M, A, K>(P, B, F, &mc[w]);
    fold_publish(F, kProgDone);
  }
  __syncthreads();
  const bool fin = kc.fin;
  const int64_t g = kc.g, t = kc.t;
  int e = 0;
  for (int b = tid; b < nw; b += FOLD_THREADS) {
    const int64_t gb = W0 + b;
    if (fin) {
      double r = 0.0;
      if (emit[b]) {
        r = st[b].finish(&e);
        if (is_inf(r)) e |= ERR_INFINITY;
      }
      kc.out_val[g * nb + gb] = r;
      kc.out_emit[g * nb + gb] = emit[b];
    } else {
      kc.partial[t * nb + gb] = st[b].pack();
      kc.tile_emit[t * nb + gb] = emit[b];
    }
  }
  if (e) atomicOr(err_word, e);
}

}  // namespace otsdb
