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

constexpr int FOLD_WIN = 128;  // per-wave ring of closed bucket values
constexpr int FOLD_FL = 32;    // flush once this many buckets are final
constexpr int32_t kProgDone = INT32_MAX;

// k_fold_prep: one thread per (series, inner boundary).  The boundary
// buckets' values are folded sequentially (Java order) from the points.
template <class M>
__global__ __launch_bounds__(256) void k_fold_prep(Params P, BatchDev B,
                                                   SeriesMeta SM, int64_t NW,
                                                   int64_t WB,
                                                   WinCtx* __restrict__ wc) {
  const int64_t nbd = NW - 1;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t s = idx / nbd;
  if (s >= B.S) return;
  const int64_t j = idx - s * nbd + 1;
  WinCtx c{0, INT64_MIN, 0.0, INT64_MIN, 0.0};
  const bool keep = SM.keep[s];
  const int64_t lo = keep ? SM.lo[s] : 0, hi = keep ? SM.hi[s] : 0;
  if (lo >= hi) {
    c.bnd = lo;
    wc[s * nbd + j - 1] = c;
    return;
  }
  const int sf = B.series_float ? (int)B.series_float[s] : 1;
  const int64_t p = lower_bound_ends(B.ts, lo, hi, bucket_ts(P, j * WB));
  c.bnd = p;
  int err = 0;
  if (p > lo) {
    const int64_t k = bucket_of(P, B.ts[p - 1]);
    const int64_t bt = bucket_ts(P, k);
    const int64_t q = lower_bound_ends(B.ts, lo, p - 1, bt);
    M st = M::init();
    for (int64_t i = q; i < p; ++i) st.push(point_value(B, i, B.val[i], sf));
    c.prev_ts = bt;
    c.prev_val = st.finish(&err);
  }
  if (p < hi) {
    const int64_t k = bucket_of(P, B.ts[p]);
    const int64_t bt = bucket_ts(P, k), be = bucket_ts(P, k + 1);
    M st = M::init();
    for (int64_t i = p; i < hi && B.ts[i] < be; ++i)
      st.push(point_value(B, i, B.val[i], sf));
    c.next_ts = bt;
    c.next_val = st.finish(&err);
  }
  wc[s * nbd + j - 1] = c;
}

// One wavefront's view of the fold (wave-uniform except the pointers).
template <class A>
struct FoldSink {
  A* st;              // LDS aggregator states of the window
  uint8_t* emit;      // LDS: some member has a real point there
  double* ring;       // this wave's LDS ring
  int32_t* prog;      // LDS progress marks of the chunk's members
  int* err;           // device error word (watchdog)
  int32_t mi;         // this member's index in the chunk
  int32_t eff;        // cached effective mark of the predecessors
  int64_t W0, W1;     // window buckets [W0, W1)
  int64_t flushed;    // buckets below are pushed or pending
  int64_t pend;       // start of the pending gap, -1: none
  int64_t x0;         // the latest real bucket before `pend`
  double y0;
};

// Waits until every member before this one has pushed all its contributions
// to buckets < need.
template <class A>
DEV void fold_wait(FoldSink<A>& F, int64_t need) {
#ifdef OTSDB_FOLD_NOWAIT  // debug build: no ordering
  return;
#endif
  if ((int64_t)F.eff >= need) return;
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
    if ((int64_t)e >= need) break;
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
DEV void fold_publish(FoldSink<A>& F, int64_t p) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (LANE == 0)
    __hip_atomic_store(&F.prog[F.mi], (int32_t)p, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}

// pushes the member's interpolated contribution to every bucket of [a, e)
// (between its real buckets x0 -> x1, or toward the point past the window)
template <class A>
DEV void fold_fill_gap(const Params& P, FoldSink<A>& F, int64_t a, int64_t e,
                       int64_t x1, double y1) {
  const int lane = LANE;
  for (int64_t j0 = a; j0 < e; j0 += 64) {
    const int64_t b = j0 + lane;
    if (b < e)
      F.st[b - F.W0].push(
          interp_value(P.interp, bucket_ts(P, b), F.x0, F.y0, x1, y1));
  }
}

// Turns the ring's buckets [flushed, limit) (all final) into contributions.
template <class A>
DEV void fold_flush(const Params& P, FoldSink<A>& F, int64_t limit) {
  if (limit <= F.flushed) return;
  fold_wait(F, limit);
  const int lane = LANE;
  const bool fill = P.fill != 0;
  int dbg_n = 0;
  for (int64_t f = F.flushed; f < limit; f += 64) {
    FOLD_GUARD(dbg_n, 1 << 26, F.err, "flush loop mi=%d f=%ld limit=%ld\n", F.mi, (long)f, (long)limit)
    const int64_t b = f + lane;
    const bool inb = b < limit;
    double v = absent_value();
    if (inb) {
      const int i = (int)(b & (FOLD_WIN - 1));
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

// t[] element holding point `idx` of the step at `base` (idx wave-uniform)
template <int K>
DEV int64_t step_ts(const int64_t* t, int64_t base, int64_t idx) {
  const int64_t r = idx - base;
  const int j = (int)(r % K);
  int64_t x = t[0];
#pragma unroll
  for (int q = 1; q < K; ++q)
    if (q == j) x = t[q];
  return readlane_l(x, (int)(r / K));
}

// One member's points [pa, pb) of the window (the member's wave).
// Context: the latest real bucket before the window (has_prev: x0/y0) and
// where its contribution goes past its last real bucket of the window
// (has_next: toward (nx, ny) — the next real bucket, or the point past the
// grid, AggregationIterator.java:760-775).
template <class M, class A, int K>
DEV void fold_member(const Params& P, const BatchDev& B, FoldSink<A>& F,
                     int sf, bool kept, int64_t pa, int64_t pb, bool has_prev,
                     int64_t px, double py, bool has_next, int64_t nx,
                     double ny) {
  constexpr int PTS = 64 * K;
  const int lane = LANE;
  F.flushed = F.W0;
  F.pend = has_prev ? F.W0 : -1;
  F.x0 = px;
  F.y0 = py;
  if (!kept) return;  // contributes nowhere (SpanGroup.add dropped it)
  RowSink S{nullptr, nullptr, F.ring, FOLD_WIN - 1, 0, 0, 0, 0};
  int err = 0;
  int carry_key = INT32_MIN;
  M carry = M::init();
  int64_t lo_eff = pa;
  int64_t k_last = -1;
  int dbg_n = 0;
  for (int64_t base = pa & ~(int64_t)1; base < pb;) {
    FOLD_GUARD(dbg_n, 1 << 30, F.err, "stream loop mi=%d base=%ld pa=%ld pb=%ld lo_eff=%ld\n", F.mi, (long)base, (long)pa, (long)pb, (long)lo_eff)
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
    const int64_t first_i = base > lo_eff ? base : lo_eff;
    const int64_t last_i = (base + PTS < pb ? base + PTS : pb) - 1;
    const int64_t k_first = bucket_of(P, step_ts<K>(t, base, first_i));
    const int64_t k_hi = bucket_of(P, step_ts<K>(t, base, last_i));
    k_last = k_hi;
    const bool carry_ok = carry_key >= 0 && carry_key < P.nb;
    if (carry_ok && carry_key < k_first) {
      // the open bucket ends before this step: close it now
      if (lane == 0) S.put(carry_key, carry.finish(&err));
      carry_key = INT32_MIN;
    }
    const int64_t k_open = (carry_key >= 0 && carry_key < P.nb) ? carry_key : k_first;
    if (k_open - F.flushed >= FOLD_FL || k_hi >= F.flushed + FOLD_WIN)
      fold_flush(P, F, k_open);
    int64_t hi_step = pb;
    if (k_hi >= F.flushed + FOLD_WIN) {
      // the step spans more buckets than the ring: cut it where the ring
      // ends (a bucket boundary) and resume from there
      const int64_t T = bucket_ts(P, F.flushed + FOLD_WIN);
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < K; ++j)
        cnt += (i0 + j >= first_i && i0 + j <= last_i && t[j] < T) ? 1 : 0;
      hi_step = first_i + uni((int32_t)wave_sum(cnt));
    }
    reduce_step<M, K, 1>(P, B, sf, lo_eff, hi_step, base, i0, t, v, S, err,
                         carry_key, carry);
    if (hi_step < pb) {
      lo_eff = hi_step;
      base = hi_step & ~(int64_t)1;
    } else {
      base += PTS;
    }
  }
  if (carry_key >= 0 && carry_key < P.nb && lane == 0)
    S.put(carry_key, carry.finish(&err));
  if (k_last >= 0) fold_flush(P, F, k_last + 1);
  // the window's remaining buckets
  if (P.fill) {
    if (F.flushed < F.W1) {
      fold_wait(F, F.W1);
      for (int64_t j0 = F.flushed; j0 < F.W1; j0 += 64) {
        const int64_t b = j0 + lane;
        if (b < F.W1) {
          F.st[b - F.W0].push(P.fill_value);
          F.emit[b - F.W0] = 1;
        }
      }
    }
  } else if (F.pend >= 0 && has_next && F.pend < F.W1) {
    fold_wait(F, F.W1);
    fold_fill_gap(P, F, F.pend, F.W1, nx, ny);
  }
}

// k_fold: see the file header.  Single-chunk groups finish here (out_val /
// out_emit); chunks of larger groups (and every chunk with always_partial,
// the multi-GPU partials) leave their window of partials for k_combine.
template <class M, class A, int K>
__global__ __launch_bounds__(256) void k_fold(
    Params P, BatchDev B, SeriesMeta SM, int64_t n_tiles,
    const int64_t* __restrict__ tile_g, const int64_t* __restrict__ tile_m0,
    const int64_t* __restrict__ tile_m1,
    const uint8_t* __restrict__ tile_single,
    const int64_t* __restrict__ members, const WinCtx* __restrict__ wc,
    int64_t NW, Packed* __restrict__ partial, uint8_t* __restrict__ tile_emit,
    double* __restrict__ out_val, uint8_t* __restrict__ out_emit,
    int* err_word, int always_partial) {
  constexpr int WB = fold_wb<A>();
  __shared__ A st[WB];
  __shared__ uint8_t emit[WB];
  __shared__ double ring[4][FOLD_WIN];
  __shared__ int32_t prog[256];
  __shared__ int s_next;
  const int tid = threadIdx.x, lane = LANE, w = tid >> 6;
  const int64_t t = (int64_t)blockIdx.x % n_tiles;
  const int64_t win = (int64_t)blockIdx.x / n_tiles;
  const int64_t nb = P.nb;
  const int64_t W0 = win * WB, W1 = (W0 + WB < nb) ? W0 + WB : nb;
  const int nw = (int)(W1 - W0);
  for (int b = tid; b < nw; b += 256) {
    st[b] = A::init();
    emit[b] = 0;
  }
  prog[tid] = 0;
  for (int i = lane; i < FOLD_WIN; i += 64) ring[w][i] = absent_value();
  if (tid == 0) s_next = 0;
  __syncthreads();
  const int64_t m0 = tile_m0[t], m1 = tile_m1[t];
  const int64_t nbd = NW - 1;
  int dbg_n = 0;
  FoldSink<A> F{st, emit, ring[w], prog, err_word, 0, 0, W0, W1, W0, -1, 0, 0.0};
  for (;;) {
    int i = 0;
    if (lane == 0) i = atomicAdd(&s_next, 1);
    i = __builtin_amdgcn_readlane(i, 0);
    if (m0 + i >= m1) break;
    FOLD_GUARD(dbg_n, 1 << 20, err_word, "claim loop i=%d m0=%ld m1=%ld\n", i, (long)m0, (long)m1)
    const int64_t s = uni(members[m0 + i]);
    F.mi = i;
    F.eff = 0;
    const bool kept = uni((int32_t)SM.keep[s]) != 0;
    const int64_t lo = kept ? uni(SM.lo[s]) : 0, hi = kept ? uni(SM.hi[s]) : 0;
    int64_t pa = lo, pb = hi;
    bool has_prev = false, has_next = false;
    int64_t px = 0, nx = 0;
    double py = 0.0, ny = 0.0;
    if (win > 0) {
      const WinCtx* c = wc + s * nbd + win - 1;
      pa = uni(c->bnd);
      const int64_t pt = uni(c->prev_ts);
      if (pt != INT64_MIN) {
        has_prev = true;
        px = pt;
        py = uni(c->prev_val);
      }
    }
    if (win < nbd) {
      const WinCtx* c = wc + s * nbd + win;
      pb = uni(c->bnd);
      const int64_t nt = uni(c->next_ts);
      if (nt != INT64_MIN) {
        has_next = true;
        nx = nt;
        ny = uni(c->next_val);
      }
    }
    if (!has_next && uni((int32_t)SM.of_has[s])) {  // toward the point past the grid
      has_next = true;
      nx = uni(SM.of_ts[s]);
      ny = uni(SM.of_val[s]);
    }
    const int sf = B.series_float ? uni((int32_t)B.series_float[s]) : 1;
    fold_member<M, A, K>(P, B, F, sf, kept, pa, pb, has_prev, px, py,
                         has_next, nx, ny);
    fold_publish(F, kProgDone);
  }
  __syncthreads();
  const bool fin = tile_single[t] && !always_partial;
  const int64_t g = tile_g[t];
  int e = 0;
  for (int b = tid; b < nw; b += 256) {
    const int64_t gb = W0 + b;
    if (fin) {
      double r = 0.0;
      if (emit[b]) {
        r = st[b].finish(&e);
        if (is_inf(r)) e |= ERR_INFINITY;
      }
      out_val[g * nb + gb] = r;
      out_emit[g * nb + gb] = emit[b];
    } else {
      partial[t * nb + gb] = st[b].pack();
      tile_emit[t * nb + gb] = emit[b];
    }
  }
  if (e) atomicOr(err_word, e);
}

}  // namespace otsdb
