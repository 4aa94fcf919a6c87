// select.hip — median / percentile across the series of large groups
// (PercentileAgg.runDouble, Aggregators.java:687-706, commons-math3 3.4.1
// LEGACY estimator; Median.runDouble, :412-431) by MSB radix select over
// order-preserving 64-bit keys.
//
//  k_keys_transpose  bucket rows [S][B] -> key columns [B][M] (members in
//                    group order; non-contributing / NaN -> KEY_NONE), via
//                    64x64 LDS tiles so both the read and the write coalesce
//  k_sel_init        per (group, bucket): n (non-NaN contributions) -> the
//                    one or two target ranks the estimator needs
//  k_seg_select      one workgroup per (group, bucket) segment: min / max,
//                    11-bit digit passes, LDS gather + count select
//  k_xsel_*          the cross-rank protocol (otsdb_sel_*): offset digit,
//                    one more digit pass that also compacts the candidates,
//                    pool passes, the unique key picked by its rank
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace otsdb {

constexpr uint64_t KEY_NONE = ~0ULL;
constexpr int SEL_CHUNK = 1 << 17;  // keys per k_xsel_scan block
#ifndef OTSDB_KT_M  // members per k_keys_transpose tile: 64 (4 waves) or 128
#define OTSDB_KT_M 128  // (8 waves, 1 KB key runs per bucket; C5 4.48 -> 4.42 ms)
#endif
constexpr int KT_M = OTSDB_KT_M;
constexpr int KT_WAVES = KT_M / 16;  // each wave loads 16 members' rows
constexpr int KT_THREADS = 64 * KT_WAVES;
static_assert(KT_M == 64 || KT_M == 128, "keys transpose tile");

DEV uint64_t dkey(double v) {  // total order, -0.0 < 0.0 (Double.compareTo)
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
DEV double key_value(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k;
  return __longlong_as_double((long long)u);
}

// Fill-mode selection without k_transform / k_group (percentiles over a
// FillingDownsampler grid, every group large): the transpose applies the
// fill itself (a kept series contributes every bucket, its real value or the
// fill value; FillingDownsampler.java:258-272), counts the non-NaN keys per
// (bucket, tile) and flags the groups that hold a kept series (they emit
// every bucket); k_seg_select derives n and the targets from that.
struct SelFill {
  const uint8_t* keep;     // null: the rows are final (k_transform ran)
  const int32_t* kf;       // sentinel rows: buckets [kf, kl] written
  const int32_t* kl;
  double fill_value;
  uint32_t* cnt;           // [nb][ntiles] non-NONE keys per (bucket, tile)
  const int64_t* lg_off;   // every group is large: member ranges
  int64_t n_lg;
  uint32_t* kept;          // [n_lg] the group has a kept series
};

#ifndef OTSDB_KT_SLICES  // bucket slices per KT_M members (grid.y): C5's
#define OTSDB_KT_SLICES 4  // 977 member tiles alone are ~1.9 rounds of the
#endif                     // 512 workgroups its LDS lets the chip hold
// One workgroup per KT_M members and bucket slice (blockIdx.y) sweeps their
// rows tile by tile (64 buckets):
// the members' row offsets are read once, and the next tile's values and
// states are loaded into registers before the current tile leaves LDS, so
// each wave keeps a tile's loads in flight while it stores the previous one.
// mm (optional): per (bucket, tile) min / max non-NONE key, k_seg_select's
// first pass.
template <bool FILL>
__global__ __launch_bounds__(KT_THREADS) void k_keys_transpose(
    int64_t nb, int64_t M, const int64_t* __restrict__ members, Rows R,
    uint64_t* __restrict__ keys, uint64_t* __restrict__ mm, SelFill F) {
  __shared__ uint64_t tile[KT_M][65];
  __shared__ int64_t s_row[KT_M];
  __shared__ int32_t s_kf[KT_M], s_kl[KT_M];
  __shared__ uint64_t s_mm[KT_WAVES][64][2];
  __shared__ uint32_t s_cnt[KT_WAVES][64];
  const int64_t ntiles = gridDim.x;
  const int tid = threadIdx.x;
  const int64_t m0 = (int64_t)blockIdx.x * KT_M;
  const int bi = tid & 63, w = tid >> 6;
  if (tid < KT_M) {
    const int64_t m = m0 + tid;
    const int64_t sr = m < M ? members[m] : -1;
    s_row[tid] = sr >= 0 ? sr * nb : -1;
    if (FILL) {
      const bool kp = sr >= 0 && F.keep[sr];
      // not kept: contributes nowhere (kf > kl and no fill)
      s_kf[tid] = kp ? F.kf[sr] : 1;
      s_kl[tid] = kp ? F.kl[sr] : 0;
      if (!kp) s_row[tid] = -1;
      int64_t g = 0;  // the member's group: the last lg_off <= m
      if (kp) {
        int64_t hi = F.n_lg;
        while (hi - g > 1) {
          const int64_t mid = (g + hi) >> 1;
          if (F.lg_off[mid] <= m) g = mid;
          else hi = mid;
        }
      }
      // one flag write per distinct group of the wave (all of one group,
      // mostly): a flag every member raised would be 64 atomics per tile on
      // one word
      uint64_t todo = __ballot(kp);
      while (todo) {
        const int lead = __builtin_ctzll(todo);
        const int64_t gl = readlane_l(g, lead);
        if (bi == lead && !F.kept[gl]) atomicOr(&F.kept[gl], 1u);
        todo &= ~__ballot(kp && g == gl);
      }
    }
  }
  __syncthreads();
  double v[16];
  uint8_t st[16];
  auto load = [&](int64_t b0) {
    const int64_t b = b0 + bi;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t ro = s_row[r * KT_WAVES + w];
      const bool in = ro >= 0 && b < nb;
      // loads unconditional in shape: the 16 rows' loads all go out at once
      const int64_t off = in ? ro + b : 0;
      v[r] = R.val[off];
      if (!FILL) st[r] = in ? R.state[off] : (uint8_t)0;
    }
  };
  // this workgroup's bucket slice: whole 64-bucket tiles
  const int64_t ntb = (nb + 63) / 64;
  const int64_t tps = (ntb + gridDim.y - 1) / gridDim.y;
  const int64_t bs = (int64_t)blockIdx.y * tps * 64;
  const int64_t be = bs + tps * 64 < nb ? bs + tps * 64 : nb;
  if (bs < be) load(bs);
  for (int64_t b0 = bs; b0 < be; b0 += 64) {
    // the keys of this thread's 16 members at bucket b0 + bi, and their
    // min / max / count (the tile's per-bucket partial, from registers)
    uint64_t mn = KEY_NONE, mx = 0;
    uint32_t nk = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mi = r * KT_WAVES + w;
      uint64_t k;
      if (FILL) {
        const int64_t b = b0 + bi;
        const bool real = b >= s_kf[mi] && b <= s_kl[mi] &&
                          __double_as_longlong(v[r]) != kAbsentBits;
        const double x = real ? v[r] : F.fill_value;
        k = (s_row[mi] >= 0 && b < nb && !is_nan(x)) ? dkey(x) : KEY_NONE;
      } else {
        k = (st[r] && !is_nan(v[r])) ? dkey(v[r]) : KEY_NONE;
      }
      tile[mi][bi] = k;
      if (k != KEY_NONE) {
        mn = k < mn ? k : mn;
        mx = k > mx ? k : mx;
        ++nk;
      }
    }
    if (mm) {
      s_mm[w][bi][0] = mn;
      s_mm[w][bi][1] = mx;
      s_cnt[w][bi] = nk;
    }
    __syncthreads();
    if (b0 + 64 < be) load(b0 + 64);
    // stores: KT_M consecutive members per bucket, 4 buckets at a time
    const int sm = tid % KT_M, sg = tid / KT_M;
    const int64_t m = m0 + sm;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int bj = r * 4 + sg;
      const int64_t b = b0 + bj;
      if (m < M && b < nb) keys[b * M + m] = tile[sm][bj];
    }
    if (mm && tid < 64 && b0 + tid < nb) {
#pragma unroll
      for (int q = 1; q < KT_WAVES; ++q) {
        mn = s_mm[q][tid][0] < mn ? s_mm[q][tid][0] : mn;
        mx = s_mm[q][tid][1] > mx ? s_mm[q][tid][1] : mx;
        nk += s_cnt[q][tid];
      }
      const int64_t oi = (b0 + tid) * ntiles + blockIdx.x;
      mm[2 * oi] = mn;
      mm[2 * oi + 1] = mx;
      if (FILL) F.cnt[oi] = nk;
    }
    __syncthreads();
  }
}

struct SelState {
  uint64_t prefix[2];
  int64_t rank[2];
  int64_t n;
  int32_t ntarget;
  int32_t _pad;
};

// the one or two order statistics Median / PercentileAgg.runDouble read
// over n non-NaN values (Aggregators.java:412-431, :687-706)
DEV SelState sel_state_of(int64_t n, int median, double p) {
  SelState s;
  s.prefix[0] = s.prefix[1] = 0;
  s.n = n;
  s.ntarget = 0;
  s._pad = 0;
  s.rank[0] = s.rank[1] = 0;
  if (s.n > 0) {
    if (median) {
      s.rank[0] = s.rank[1] = s.n / 2;
    } else if (s.n == 1) {
      s.rank[0] = s.rank[1] = 0;
    } else {
      const double pos = p * (double)(s.n + 1);
      if (pos < 1) {
        s.rank[0] = s.rank[1] = 0;
      } else if (pos >= (double)s.n) {
        s.rank[0] = s.rank[1] = s.n - 1;
      } else {
        const int64_t ip = (int64_t)__builtin_floor(pos);
        s.rank[0] = ip - 1;
        s.rank[1] = ip;
      }
    }
    s.ntarget = (s.rank[0] == s.rank[1]) ? 1 : 2;
  }
  return s;
}

// segments: seg = lg * nb + b for large group lg (group id lg_g[lg])
__global__ void k_sel_init(int64_t nb, int64_t n_lg,
                           const int64_t* __restrict__ lg_g,
                           const double* __restrict__ count_val,
                           const uint8_t* __restrict__ count_emit,
                           SelState* __restrict__ sel, int median, double p) {
  const int64_t seg = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (seg >= n_lg * nb) return;
  const int64_t lg = seg / nb, b = seg - lg * nb;
  const int64_t o = lg_g[lg] * nb + b;
  sel[seg] = sel_state_of(count_emit[o] ? (int64_t)count_val[o] : 0, median, p);
}

// cross-rank protocol (otsdb_sel_*): dense (group, bucket) non-NaN counts
// as doubles <-> the int64 counts ranks all-reduce
__global__ void k_dense_to_counts(int64_t GB, const double* __restrict__ val,
                                  const uint8_t* __restrict__ emit,
                                  int64_t* __restrict__ counts,
                                  uint8_t* __restrict__ emit_out) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= GB) return;
  counts[o] = emit[o] ? (int64_t)val[o] : 0;
  emit_out[o] = emit[o];
}
__global__ void k_counts_to_dense(int64_t GB, const int64_t* __restrict__ counts,
                                  const uint8_t* __restrict__ emit,
                                  double* __restrict__ val,
                                  uint8_t* __restrict__ emit_out) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= GB) return;
  val[o] = (double)counts[o];
  emit_out[o] = emit[o] ? 1 : 0;
}

// ------------------------------------------------------------------------
// r-th smallest (0-based) of n keys, key_at(i) for i in [0, n), by one
// wavefront (the block must be exactly one wavefront: the LDS histogram is
// fenced with __syncthreads): 8 MSB passes of 8 bits.
// ------------------------------------------------------------------------
template <class F>
DEV uint64_t wave_select(int64_t n, int64_t r, uint32_t* hist, F key_at) {
  const int lane = LANE;
  uint64_t prefix = 0, mask = 0;
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int j = lane; j < 256; j += 64) hist[j] = 0;
    __syncthreads();
    for (int64_t i = lane; i < n; i += 64) {
      const uint64_t k = key_at(i);
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1u);
    }
    __syncthreads();
    uint32_t c[4];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c[j] = hist[4 * lane + j];
      sum += c[j];
    }
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    const int64_t excl = (int64_t)incl - sum;
    const bool mine = r >= excl && r < (int64_t)incl;
    int digit = 0;
    int64_t rem = 0;
    if (mine) {
      int64_t cum = excl;
      int j = 0;
      for (; j < 3; ++j) {
        if (r < cum + c[j]) break;
        cum += c[j];
      }
      digit = 4 * lane + j;
      rem = r - cum;
    }
    const uint64_t who = __ballot(mine);
    const int src = who ? __builtin_ctzll(who) : 0;
    digit = __shfl(digit, src);
    rem = __shfl(rem, src);
    r = rem;
    prefix |= (uint64_t)digit << shift;
    mask |= (uint64_t)0xFF << shift;
    __syncthreads();
  }
  return prefix;
}

// Median.runDouble (Aggregators.java:412-431) / PercentileAgg.runDouble
// (:687-706, LEGACY whatever the name) over n non-NaN values given as the
// one or two order statistics the estimator reads.
DEV void sel_ranks(int median, double p, int64_t n, int64_t* r0, int64_t* r1,
                   double* pos) {
  *r0 = *r1 = 0;
  *pos = 0.0;
  if (n <= 0) return;
  if (median) {
    *r0 = *r1 = n / 2;
  } else if (n > 1) {
    *pos = p * (double)(n + 1);
    if (*pos < 1) {
      *r0 = *r1 = 0;
    } else if (*pos >= (double)n) {
      *r0 = *r1 = n - 1;
    } else {
      const int64_t ip = (int64_t)__builtin_floor(*pos);
      *r0 = ip - 1;
      *r1 = ip;
    }
  }
}
DEV double sel_value(int median, int64_t n, double pos, double lo, double hi) {
  if (n <= 0) return qnan();
  if (median || n == 1) return lo;
  if (pos >= 1 && pos < (double)n) return lo + (pos - __builtin_floor(pos)) * (hi - lo);
  return lo;
}

// ------------------------------------------------------------------------
// k_seg_select: the whole selection of one segment (large group, bucket) in
// one workgroup, for rank-local groups.  (1) min / max key of the segment: bits above
// the highest differing bit are common to every key and need no pass; (2)
// 11-bit digit passes (2,048-bin LDS histograms per target) only while a
// target still has more than SS_CAP candidates; (3) the <= SS_CAP candidates
// of each target are gathered into LDS and the target's order statistic is
// picked by counting.  Exact: the same keys, the same order statistics.
// ------------------------------------------------------------------------
constexpr int SS_BITS = 11;
constexpr int SS_BINS = 1 << SS_BITS;
constexpr int SS_CAP = 1024;
constexpr int SS_THREADS = 1024;

DEV uint64_t block_min_max_u64(uint64_t v, bool is_max, uint64_t* red) {
  // wave reduce then across the 4 waves of the block
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t o = __shfl_xor(v, d);
    v = is_max ? (o > v ? o : v) : (o < v ? o : v);
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if (LANE == 0) red[w] = v;
  __syncthreads();
  uint64_t r = red[0];
  for (int j = 1; j < SS_THREADS / 64; ++j)
    r = is_max ? (red[j] > r ? red[j] : r) : (red[j] < r ? red[j] : r);
  return r;
}

DEV uint64_t block_sum_u64(uint64_t v, uint64_t* red) {
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if (LANE == 0) red[w] = v;
  __syncthreads();
  uint64_t r = 0;
  for (int j = 0; j < SS_THREADS / 64; ++j) r += red[j];
  return r;
}

__global__ __launch_bounds__(SS_THREADS) void k_seg_select(
    int64_t nb, int64_t M, int64_t n_lg, const int64_t* __restrict__ lg_g,
    const int64_t* __restrict__ lg_off, const int64_t* __restrict__ lg_k,
    const uint64_t* __restrict__ keys, const SelState* __restrict__ sel,
    const uint8_t* __restrict__ emit, double* __restrict__ out_val,
    int* err_word, int median, double p, const uint64_t* __restrict__ mm,
    const uint32_t* __restrict__ cnt_p, const uint32_t* __restrict__ kept,
    uint8_t* __restrict__ out_emit) {
  __shared__ uint32_t h[2][SS_BINS];
  __shared__ uint64_t cand[2][SS_CAP];
  __shared__ uint64_t red[SS_THREADS / 64];
  __shared__ uint32_t s_nc[2];
  __shared__ uint64_t s_pick[2];
  __shared__ int s_digit[2];
  __shared__ int64_t s_below[2], s_cnt[2];
  const int tid = threadIdx.x;
  const int64_t seg = blockIdx.x;
  if (seg >= n_lg * nb) return;
  const int64_t lg = seg / nb, b = seg - lg * nb;
  const int64_t o = lg_g[lg] * nb + b;
  const bool fused = cnt_p != nullptr;
  if (fused) {  // FillingDownsampler grid: every bucket of a group holding a
                // kept series is emitted
    const bool e = kept[lg] != 0;
    if (tid == 0) out_emit[o] = e;
    if (!e) return;
  } else if (!emit[o]) {
    return;
  }
  SelState s0;
  if (!fused) s0 = sel[seg];
  double r = qnan();
  const uint64_t* col = keys + b * M + lg_off[lg];
  const int64_t k = lg_k[lg];
  // every key of the segment: 16-byte loads (two keys), 4 in flight per
  // thread; a key before the first 16-byte boundary and an odd last one
  // singly
  auto for_keys = [&](auto&& f) {
    const int64_t head = ((uintptr_t)col & 15) ? 1 : 0;
    if (head && k > 0 && tid == 0) f(col[0]);
    const int64_t np = (k - head) >> 1;  // pairs
    const ulonglong2* c2 = reinterpret_cast<const ulonglong2*>(col + head);
    int64_t i = tid;
    for (; i + 3 * SS_THREADS < np; i += 4 * SS_THREADS) {
      const ulonglong2 a0 = c2[i], a1 = c2[i + SS_THREADS],
                       a2 = c2[i + 2 * SS_THREADS],
                       a3 = c2[i + 3 * SS_THREADS];
      f(a0.x);
      f(a0.y);
      f(a1.x);
      f(a1.y);
      f(a2.x);
      f(a2.y);
      f(a3.x);
      f(a3.y);
    }
    for (; i < np; i += SS_THREADS) {
      const ulonglong2 a = c2[i];
      f(a.x);
      f(a.y);
    }
    if (((k - head) & 1) && tid == 0) f(col[k - 1]);
  };
  // (1) min / max (fused: and count) over the non-NONE keys: from
  // k_keys_transpose's per-(KT_M-member tile, bucket) partials for the tiles
  // wholly inside the segment, the keys of the partial tiles at its ends
  // directly
  uint64_t mn = ~0ULL, mx = 0;
  if (fused || s0.ntarget > 0) {
    uint64_t nn = 0;
    auto fold = [&](uint64_t key) {
      if (key == KEY_NONE) return;
      mn = key < mn ? key : mn;
      mx = key > mx ? key : mx;
      ++nn;
    };
    const int64_t o0 = lg_off[lg], ntiles = (M + KT_M - 1) / KT_M;
    const int64_t t_lo = (o0 + KT_M - 1) / KT_M, t_hi = (o0 + k) / KT_M;
    if (mm && t_hi > t_lo) {
      const uint64_t* pm = mm + 2 * (b * ntiles);
      for (int64_t t = t_lo + tid; t < t_hi; t += SS_THREADS) {
        mn = pm[2 * t] < mn ? pm[2 * t] : mn;
        mx = pm[2 * t + 1] > mx ? pm[2 * t + 1] : mx;
        if (fused) nn += cnt_p[b * ntiles + t];
      }
      const int64_t e0 = t_lo * KT_M - o0, e1 = t_hi * KT_M - o0;
      for (int64_t i = tid; i < e0; i += SS_THREADS) fold(col[i]);
      for (int64_t i = e1 + tid; i < k; i += SS_THREADS) fold(col[i]);
    } else {
      for_keys(fold);
    }
    mn = block_min_max_u64(mn, false, red);
    mx = block_min_max_u64(mx, true, red);
    if (fused) s0 = sel_state_of((int64_t)block_sum_u64(nn, red), median, p);
  }
  const int nt = s0.ntarget;
  if (nt > 0) {
    uint64_t prefix[2], mask[2];
    int64_t rank[2], cnt[2];
    int shift = 0;
    if (mn != mx) shift = 64 - __builtin_clzll(mn ^ mx);  // bits left to resolve
    for (int t = 0; t < 2; ++t) {
      mask[t] = shift >= 64 ? 0ULL : ~0ULL << shift;
      prefix[t] = mn & mask[t];
      rank[t] = s0.rank[t];
      cnt[t] = s0.n;
    }
    // (2a) the first pass bins by an OFFSET digit, (key >> s1) - (mn >> s1)
    // with the smallest s1 whose range fits the 2,048 bins, instead of the
    // top 11 bits below the common prefix: for doubles of one sign those are
    // mostly exponent bits (cpu% values 1..100 use 7 of the 2,048 bins and
    // a p99 target keeps ~1/3 of the keys), while the offset digit resolves
    // the exponent and the leading mantissa bits in one pass — one pass over
    // the keys less before the gather.  Monotone in the key, so the target's
    // bin is again a bit prefix (bits >= s1) for the passes below.
    if (shift > 0 && (cnt[0] > SS_CAP || (nt == 2 && cnt[1] > SS_CAP))) {
      int s1 = 64 - __builtin_clzll(mx - mn) - SS_BITS;
      if (s1 < 0) s1 = 0;
      while (s1 < 64 && (mx >> s1) - (mn >> s1) >= (uint64_t)SS_BINS) ++s1;
      const uint64_t b1 = mn >> s1;
      for (int j = tid; j < SS_BINS; j += SS_THREADS) h[0][j] = 0;
      __syncthreads();
      for_keys([&](uint64_t key) {
        if (key == KEY_NONE) return;
        atomicAdd(&h[0][(uint32_t)((key >> s1) - b1)], 1u);
      });
      __syncthreads();
      if (nt == 2)
        for (int j = tid; j < SS_BINS; j += SS_THREADS) h[1][j] = h[0][j];
      __syncthreads();
      const int wv = tid >> 6, lane = LANE;
      if (wv < nt) {
        const int per = SS_BINS / 64;
        uint32_t sum = 0;
        for (int j = 0; j < per; ++j) sum += h[wv][lane * per + j];
        uint32_t incl = sum;
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(incl, d);
          if (lane >= d) incl += y;
        }
        const int64_t excl = (int64_t)incl - sum;
        const int64_t rr = rank[wv];
        if (rr >= excl && rr < (int64_t)incl) {
          int64_t cum = excl;
          int j = 0;
          for (; j < per - 1; ++j) {
            const uint32_t c = h[wv][lane * per + j];
            if (rr < cum + c) break;
            cum += c;
          }
          s_digit[wv] = lane * per + j;
          s_below[wv] = cum;
          s_cnt[wv] = h[wv][lane * per + j];
        }
      }
      __syncthreads();
      for (int t = 0; t < nt; ++t) {
        mask[t] = s1 >= 64 ? 0ULL : ~0ULL << s1;
        prefix[t] = s1 >= 64 ? 0ULL : (b1 + (uint64_t)s_digit[t]) << s1;
        rank[t] -= s_below[t];
        cnt[t] = s_cnt[t];
      }
      shift = s1;
      __syncthreads();
    }
    // (2b) digit passes while some target has too many candidates
    while (shift > 0 && (cnt[0] > SS_CAP || (nt == 2 && cnt[1] > SS_CAP))) {
      const int w = shift < SS_BITS ? shift : SS_BITS;
      shift -= w;
      const uint32_t dm = (1u << w) - 1;
      // targets still sharing their prefix (the two order statistics of an
      // interpolating estimator usually do) share one histogram
      const bool two = nt == 2 && prefix[1] != prefix[0];
      for (int j = tid; j < (two ? 2 : 1) * SS_BINS; j += SS_THREADS)
        (&h[0][0])[j] = 0;
      __syncthreads();
      if (two) {
        for_keys([&](uint64_t key) {
          if (key == KEY_NONE) return;
          const uint32_t d = (uint32_t)(key >> shift) & dm;
          if ((key & mask[0]) == prefix[0]) atomicAdd(&h[0][d], 1u);
          if ((key & mask[1]) == prefix[1]) atomicAdd(&h[1][d], 1u);
        });
      } else {
        for_keys([&](uint64_t key) {
          if (key == KEY_NONE) return;
          if ((key & mask[0]) == prefix[0])
            atomicAdd(&h[0][(uint32_t)(key >> shift) & dm], 1u);
        });
      }
      __syncthreads();
      if (nt == 2 && !two)
        for (int j = tid; j < SS_BINS; j += SS_THREADS) h[1][j] = h[0][j];
      __syncthreads();
      // per target: the digit whose cumulative count passes the rank (one
      // wave per target scans its bins, 32 per lane)
      const int wv = tid >> 6, lane = LANE;
      if (wv < nt) {
        const int per = SS_BINS / 64;
        uint32_t sum = 0;
        for (int j = 0; j < per; ++j) sum += h[wv][lane * per + j];
        uint32_t incl = sum;
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(incl, d);
          if (lane >= d) incl += y;
        }
        const int64_t excl = (int64_t)incl - sum;
        const int64_t rr = rank[wv];
        if (rr >= excl && rr < (int64_t)incl) {
          int64_t cum = excl;
          int j = 0;
          for (; j < per - 1; ++j) {
            const uint32_t c = h[wv][lane * per + j];
            if (rr < cum + c) break;
            cum += c;
          }
          s_digit[wv] = lane * per + j;
          s_below[wv] = cum;
          s_cnt[wv] = h[wv][lane * per + j];
        }
      }
      __syncthreads();
      for (int t = 0; t < nt; ++t) {
        prefix[t] |= (uint64_t)s_digit[t] << shift;
        mask[t] |= (uint64_t)dm << shift;
        rank[t] -= s_below[t];
        cnt[t] = s_cnt[t];
      }
      __syncthreads();
    }
    // (3) both targets' candidates gathered in one pass over the keys, then
    // each target's rank-th picked by counting
    uint64_t val[2];
    bool need[2] = {false, false};
    for (int t = 0; t < nt; ++t) {
      if (shift == 0) val[t] = prefix[t];  // every bit resolved
      else need[t] = true;
    }
    if (need[0] || need[1]) {
      // targets with the same remaining prefix gather one candidate set
      const bool same = need[0] && need[1] && prefix[0] == prefix[1];
      if (tid < 2) s_nc[tid] = 0;
      __syncthreads();
      for_keys([&](uint64_t key) {
        if (key == KEY_NONE) return;
        for (int t = 0; t < (same ? 1 : 2); ++t) {
          if (need[t] && (key & mask[t]) == prefix[t]) {
            const uint32_t q = atomicAdd(&s_nc[t], 1u);
            if (q < SS_CAP) cand[t][q] = key;
          }
        }
      });
      __syncthreads();
      for (int t = 0; t < 2; ++t) {
        if (!need[t]) continue;
        const int src = same ? 0 : t;
        const int nc = (int)(s_nc[src] < SS_CAP ? s_nc[src] : SS_CAP);
        const int64_t rr = rank[t];
        for (int j = tid; j < nc; j += SS_THREADS) {
          const uint64_t x = cand[src][j];
          int less = 0, eq = 0;
          for (int q = 0; q < nc; ++q) {
            less += cand[src][q] < x;
            eq += cand[src][q] == x;
          }
          if (rr >= less && rr < less + eq) s_pick[t] = x;  // ties: same key
        }
      }
      __syncthreads();
      for (int t = 0; t < 2; ++t)
        if (need[t]) val[t] = s_pick[t];
    }
    if (nt == 1) val[1] = val[0];
    // PercentileAgg / Median estimator over the order statistics
    double pos = 0.0;
    int64_t r0, r1;
    sel_ranks(median, p, s0.n, &r0, &r1, &pos);
    r = sel_value(median, s0.n, pos, key_value(val[0]), key_value(val[1]));
  }
  if (tid == 0) {
    if (is_inf(r)) atomicOr(err_word, ERR_INFINITY);
    out_val[o] = r;
  }
}

// ------------------------------------------------------------------------
// k_ds_select: median / percentile DOWNSAMPLING (Downsampler.java:162-228:
// function.runDouble over the values of each interval).  One wavefront per
// series (block = 64); lanes take consecutive buckets, find each bucket's
// points by binary search, and select over the non-NaN values: buckets of
// up to DS_SMALL values by an insertion sort in LDS, larger ones by a
// wave-wide radix select.  Bucket index nb stands for the first bucket past
// the window (k_prep's of_val).
// ------------------------------------------------------------------------
constexpr int DS_SMALL = 16;

__global__ __launch_bounds__(64) void k_ds_select(Params P, BatchDev B,
                                                  SeriesMeta SM, Rows R) {
  __shared__ uint64_t sk[DS_SMALL][64];
  __shared__ uint32_t hist[256];
  const int lane = LANE;
  const int64_t s = blockIdx.x;
  if (s >= B.S || !SM.keep[s]) return;
  const int64_t lo = SM.lo[s], hi = SM.hi[s], p1 = B.offsets[s + 1];
  const int sf = B.series_float ? (int)B.series_float[s] : 1;
  const int median = P.ds_sel == 1;
  const double p = P.ds_pct;
  double* rowv = R.val + s * P.nb;
  uint8_t* rows = R.state + s * P.nb;
  auto value = [&](int64_t i) {
    const int64_t b = B.val[i];
    const int f = B.is_float ? (int)B.is_float[i] : sf;
    return f ? __longlong_as_double(b) : (double)b;
  };
  // the percentile of the points [a, e) of each active lane's bucket (NaN
  // when every value is NaN): buckets of up to DS_SMALL values by a per-lane
  // insertion sort, larger ones by the whole wave, one bucket at a time
  auto select_buckets = [&](bool act, int64_t a, int64_t e) -> double {
    const int64_t cnt = act ? e - a : 0;
    double res = qnan();
    if (cnt > 0 && cnt <= DS_SMALL) {
      int n = 0;
      for (int64_t i = a; i < e; ++i) {
        const double v = value(i);
        if (is_nan(v)) continue;
        const uint64_t k = dkey(v);
        int q = n++;
        while (q > 0 && sk[q - 1][lane] > k) {
          sk[q][lane] = sk[q - 1][lane];
          --q;
        }
        sk[q][lane] = k;
      }
      int64_t r0, r1;
      double pos;
      sel_ranks(median, p, n, &r0, &r1, &pos);
      if (n)
        res = sel_value(median, n, pos, key_value(sk[r0][lane]),
                        key_value(sk[r1][lane]));
    }
    uint64_t big = __ballot(cnt > DS_SMALL);
    while (big) {
      const int l = __builtin_ctzll(big);
      big &= big - 1;
      const int64_t la = __shfl(a, l), le = __shfl(e, l);
      // non-NaN count
      int64_t nn = 0;
      for (int64_t i = la + lane; i < le; i += 64) nn += !is_nan(value(i));
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) nn += __shfl_xor(nn, d);
      // NaNs (either sign) take the largest key: ranks below nn never
      // reach them
      auto key_at = [&](int64_t i) {
        const double v = value(la + i);
        return is_nan(v) ? ~0ULL : dkey(v);
      };
      int64_t r0, r1;
      double pos;
      sel_ranks(median, p, nn, &r0, &r1, &pos);
      double v = qnan();
      if (nn > 0) {
        const uint64_t k0 = wave_select(le - la, r0, hist, key_at);
        const uint64_t k1 = (r1 == r0) ? k0 : wave_select(le - la, r1, hist, key_at);
        v = sel_value(median, nn, pos, key_value(k0), key_value(k1));
      }
      if (lane == l) res = v;
    }
    return res;
  };
  // buckets that can hold points: [b_first, b_last] (+ nb for of_val)
  int64_t b_first = 0, b_last = -1;
  if (lo < hi) {
    b_first = bucket_of(P, B.ts[lo]);
    b_last = bucket_of(P, B.ts[hi - 1]);
  }
  const bool of = SM.of_has[s] != 0;
  const int64_t n_b = (b_last - b_first + 1) + (of ? 1 : 0);
  double of_v = 0.0;
  int64_t of_e = hi;
  for (int64_t c0 = 0; c0 < n_b; c0 += 64) {
    const int64_t j = c0 + lane;
    const bool act = j < n_b;
    const bool is_of = act && of && j == n_b - 1;
    const int64_t b = is_of ? P.nb : b_first + j;
    int64_t a = 0, e = 0;
    if (act) {
      if (is_of) {
        a = hi;
        const int64_t of_end =
            P.cal ? P.cal[cal_bucket(P, SM.of_ts[s]) + 1]
                  : SM.of_ts[s] + P.interval;
        e = lower_bound(B.ts, hi, p1, of_end);
      } else if (P.run_all) {
        a = lo;
        e = hi;
      } else {
        a = lower_bound(B.ts, lo, hi, bucket_ts(P, b));
        e = lower_bound(B.ts, a, hi, bucket_ts(P, b + 1));
      }
    }
    const double v = select_buckets(act, a, e);
    if (act && e > a) {
      if (is_of) {
        SM.of_val[s] = v;
      } else {
        rowv[b] = v;
        rows[b] = ST_REAL;
      }
    }
    const uint64_t om = __ballot(is_of);
    if (om) {
      const int l = __builtin_ctzll(om);
      of_v = __shfl(v, l);
      of_e = __shfl(e, l);
    }
  }
  if (!(P.rate && of)) return;
  // rate queries: the kept rates past the bucket past the window (k_prep's
  // rates_beyond, here over percentile buckets).  Lane j takes the j-th
  // bucket from the one holding the next unread point; the rates then chain
  // through the lanes in order until two are kept or the points run out.
  int64_t t = SM.of_ts[s], pos = of_e;
  double v = of_v, r1 = 0.0;
  int nk = 0;
  while (nk < 2 && pos < p1) {
    const int64_t t_pos = B.ts[pos];
    int64_t bt = 0, be = 0;
    bool act = true;
    if (P.cal) {
      const int64_t k = cal_bucket(P, t_pos) + lane;
      act = k >= P.cal_lo && k + 1 < P.cal_n;
      if (act) {
        bt = P.cal[k];
        be = P.cal[k + 1];
      }
    } else {
      bt = align_ts(t_pos, P.interval) + lane * P.interval;
      be = bt + P.interval;
    }
    int64_t a = pos, e = pos;
    if (act) {
      a = lower_bound(B.ts, pos, p1, bt);
      e = lower_bound(B.ts, a, p1, be);
    }
    const double bv = select_buckets(act, a, e);
    const uint64_t hm = __ballot(act && e > a);
    if (!hm) break;  // the calendar table ends here
    for (uint64_t m = hm; m && nk < 2; m &= m - 1) {
      const int l = __builtin_ctzll(m);
      const int64_t tn = __shfl(bt, l);
      const double vn = __shfl(bv, l);
      bool kept;
      const double r = rate_between(P, t, v, tn, vn, &kept);
      if (kept && nk++ == 0) r1 = r;
      t = tn;
      v = vn;
    }
    pos = __shfl(e, 63 - __builtin_clzll(hm));
  }
  if (lane == 0) {
    SM.of_has[s] = (uint8_t)(1 | (nk << 1));
    SM.of_rate[s] = r1;
  }
}

// ------------------------------------------------------------------------
// Cross-rank median / percentile (otsdb_sel_*).  The members of
// a (group, bucket) segment are spread over the ranks; each rank holds its
// members' keys as [B][M] columns (k_keys_transpose).  Exact selection with
// at most two reads of the local key matrix:
//   prepare  local non-NaN counts and each segment's min / max key (krange,
//            from k_keys_transpose's tile partials); the caller all-reduces
//   pass 0   an OFFSET digit, (key >> s1) - (min >> s1) with s1 the smallest
//            shift whose range fits 2,048 bins (k_seg_select's first pass):
//            one histogram both targets share              [key read 1]
//   pass 1   the next digit of each open target (11 bits, or 2 x 10 bits
//            when the two targets' bins differ); the keys still matching a
//            target are appended to a candidate pool       [key read 2]
//   pass 2+  histograms over the pool only
// A target is resolved when its prefix covers every bit, or when its bin
// holds ONE key over all ranks: the rank holding that key writes it into
// `picks` (the caller sums them) — from the pool, or from the key matrix
// when no pass 1 ran [key read 2].  Every decision is taken from all-reduced
// data, so the ranks plan the same passes.  The pool's capacity is bounded
// per segment by min(local members, the global counts of the targets' bins).
// Segment index = dense (group, bucket) index: the protocol lists every
// group as large (build_tiles sel_all), lg_g the identity.
// ------------------------------------------------------------------------
constexpr int XS_BINS = 2048;
constexpr uint64_t XS_SIGN = 0x8000000000000000ULL;
enum : uint32_t { XS_MORE = 1, XS_PICK = 2, XS_BROKEN = 4 };

struct XSel {
  uint64_t prefix[2];  // the target's resolved bits (those >= shift)
  int64_t rank[2];     // its rank inside that bin
  int64_t cnt[2];      // keys in that bin over all ranks
  int64_t n;           // non-NaN contributions over all ranks
  uint64_t base;       // offset pass: min >> s1
  int32_t shift[2];    // bits below the prefix (64: none resolved)
  int32_t w[2];        // the planned pass's digit width (0: not in it)
  int32_t ntarget;
  int32_t split;       // planned pass: two 1,024-bin halves (else one 2,048)
  int32_t offset;      // planned pass is the offset digit
  int32_t s1;
  uint8_t done[2];     // 0 open, 1 the prefix is the key, 2 one key in its bin
  uint8_t _pad[6];
};

DEV bool xs_match(const XSel& s, int t, uint64_t key) {
  return s.shift[t] >= 64 || (key >> s.shift[t]) == (s.prefix[t] >> s.shift[t]);
}
DEV uint32_t xs_digit(const XSel& s, int t, uint64_t key) {
  return (uint32_t)(key >> (s.shift[t] - s.w[t])) & ((1u << s.w[t]) - 1u);
}
// keys the pool keeps: those of a target not yet resolved to its prefix
DEV bool xs_keep(const XSel& s, uint64_t key) {
  return (s.ntarget > 0 && s.done[0] != 1 && xs_match(s, 0, key)) ||
         (s.ntarget > 1 && s.done[1] != 1 && xs_match(s, 1, key));
}
// the bin a key counts in for the planned pass, or -1
DEV int xs_bin(const XSel& s, uint64_t key) {
  if (s.offset) return (int)((key >> s.s1) - s.base);
  if (!s.split) {
    const int t = s.w[0] ? 0 : 1;
    return xs_match(s, t, key) ? (int)xs_digit(s, t, key) : -1;
  }
  return -1;  // split: per target (xs_bins2)
}
// plans the next digit pass of the open targets; false: none is open
DEV bool xs_plan(XSel& s) {
  s.w[0] = s.w[1] = 0;
  s.offset = 0;
  s.split = 0;
  const bool o0 = s.ntarget > 0 && s.done[0] == 0;
  const bool o1 = s.ntarget > 1 && s.done[1] == 0;
  if (!o0 && !o1) return false;
  const bool same = o0 && o1 && s.prefix[0] == s.prefix[1] && s.shift[0] == s.shift[1];
  s.split = (o0 && o1 && !same) ? 1 : 0;
  const int wmax = s.split ? 10 : 11;
  if (o0) s.w[0] = s.shift[0] < wmax ? s.shift[0] : wmax;
  if (o1) s.w[1] = s.shift[1] < wmax ? s.shift[1] : wmax;
  return true;
}
// one key of the pass: LDS (or global) histogram h of the segment
DEV void xs_count(const XSel& s, uint64_t key, uint32_t* h) {
  if (!s.split) {
    const int d = xs_bin(s, key);
    if (d >= 0) atomicAdd(&h[d], 1u);
    return;
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
    if (s.w[t] && xs_match(s, t, key)) atomicAdd(&h[t * 1024 + xs_digit(s, t, key)], 1u);
}

// prepare: the segment's local min / max non-NONE key as all-reducible
// int64 (min of key ^ sign, and of ~(max ^ sign)); empty: INT64_MAX twice.
// cnt_p (fill mode, k_keys_transpose<true>): also the segment's non-NaN
// count and emit flag (every bucket of a group holding a kept series)
__global__ __launch_bounds__(256) void k_xsel_range(
    int64_t nb, int64_t M, int64_t n_lg, const int64_t* __restrict__ lg_off,
    const int64_t* __restrict__ lg_k, const uint64_t* __restrict__ keys,
    const uint64_t* __restrict__ mm, int64_t* __restrict__ krange,
    const uint32_t* __restrict__ cnt_p, const uint32_t* __restrict__ kept,
    int64_t* __restrict__ counts, uint8_t* __restrict__ emit) {
  __shared__ uint64_t red[3][4];
  const int tid = threadIdx.x;
  const int64_t seg = blockIdx.x;
  if (seg >= n_lg * nb) return;
  const int64_t lg = seg / nb, b = seg - lg * nb;
  const int64_t o0 = lg_off[lg], k = lg_k[lg];
  const uint64_t* col = keys + b * M + o0;
  uint64_t mn = ~0ULL, mx = 0, nn = 0;
  auto fold = [&](uint64_t key) {
    if (key == KEY_NONE) return;
    mn = key < mn ? key : mn;
    mx = key > mx ? key : mx;
    ++nn;
  };
  // k_keys_transpose's per-(bucket, KT_M-member tile) partials for the
  // tiles wholly inside the segment, the keys of the partial tiles directly
  const int64_t ntiles = (M + KT_M - 1) / KT_M;
  const int64_t t_lo = (o0 + KT_M - 1) / KT_M, t_hi = (o0 + k) / KT_M;
  if (t_hi > t_lo) {
    const uint64_t* pm = mm + 2 * (b * ntiles);
    for (int64_t t = t_lo + tid; t < t_hi; t += 256) {
      mn = pm[2 * t] < mn ? pm[2 * t] : mn;
      mx = pm[2 * t + 1] > mx ? pm[2 * t + 1] : mx;
      if (cnt_p) nn += cnt_p[b * ntiles + t];
    }
    const int64_t e0 = t_lo * KT_M - o0, e1 = t_hi * KT_M - o0;
    for (int64_t i = tid; i < e0; i += 256) fold(col[i]);
    for (int64_t i = e1 + tid; i < k; i += 256) fold(col[i]);
  } else {
    for (int64_t i = tid; i < k; i += 256) fold(col[i]);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t a = __shfl_xor(mn, d), z = __shfl_xor(mx, d);
    mn = a < mn ? a : mn;
    mx = z > mx ? z : mx;
    nn += __shfl_xor(nn, d);
  }
  if (LANE == 0) {
    red[0][tid >> 6] = mn;
    red[1][tid >> 6] = mx;
    red[2][tid >> 6] = nn;
  }
  __syncthreads();
  if (tid == 0) {
    for (int j = 1; j < 4; ++j) {
      mn = red[0][j] < mn ? red[0][j] : mn;
      mx = red[1][j] > mx ? red[1][j] : mx;
      nn += red[2][j];
    }
    krange[2 * seg] = (int64_t)(mn ^ XS_SIGN);
    krange[2 * seg + 1] = ~(int64_t)(mx ^ XS_SIGN);
    if (cnt_p) {
      const bool e = kept[lg] != 0;
      counts[seg] = e ? (int64_t)nn : 0;
      emit[seg] = e ? 1 : 0;
    }
  }
}

// pass 0: the global counts and key range -> targets, the offset pass
__global__ void k_xsel_init(int64_t n_seg, const int64_t* __restrict__ counts,
                            const uint8_t* __restrict__ emit,
                            const int64_t* __restrict__ krange,
                            XSel* __restrict__ sel, int median, double p,
                            uint32_t* __restrict__ flags) {
  const int64_t seg = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (seg >= n_seg) return;
  const int64_t n = emit[seg] ? counts[seg] : 0;
  const SelState ss = sel_state_of(n, median, p);
  XSel x;
  x.n = n;
  x.ntarget = ss.ntarget;
  x.base = 0;
  x.s1 = 0;
  x.offset = 0;
  x.split = 0;
  x._pad[0] = x._pad[1] = x._pad[2] = x._pad[3] = x._pad[4] = x._pad[5] = 0;
  for (int t = 0; t < 2; ++t) {
    x.prefix[t] = 0;
    x.rank[t] = ss.rank[t];
    x.cnt[t] = n;
    x.shift[t] = 64;
    x.w[t] = 0;
    x.done[t] = 0;
  }
  if (x.ntarget > 0) {
    const uint64_t mn = (uint64_t)krange[2 * seg] ^ XS_SIGN;
    const uint64_t mx = (uint64_t)~krange[2 * seg + 1] ^ XS_SIGN;
    if (mn >= mx) {  // one distinct key (mn > mx: counted keys but none seen)
      if (mn > mx) atomicOr(flags, (uint32_t)XS_BROKEN);
      for (int t = 0; t < x.ntarget; ++t) {
        x.prefix[t] = mn;
        x.shift[t] = 0;
        x.done[t] = 1;
      }
    } else {
      int s1 = 64 - __builtin_clzll(mx - mn) - 11;
      if (s1 < 0) s1 = 0;
      while ((mx >> s1) - (mn >> s1) >= (uint64_t)XS_BINS) ++s1;
      x.s1 = s1;
      x.base = mn >> s1;
      x.offset = 1;
      atomicOr(flags, (uint32_t)XS_MORE);
    }
  }
  sel[seg] = x;
}

// the keys of one (segment, SEL_CHUNK chunk) per block: the planned pass's
// histogram (mode 1), candidates appended to the pool (mode 2), the unique
// key of a target picked (mode 4)
// the pool: one region per segment, [off[seg], off[seg + 1]) sized by the
// apply's bound and filled through a per-segment counter; unfilled slots
// keep seg = -1
struct XPool {
  uint64_t* key;
  int64_t* seg;
  const int64_t* off;  // [n_seg + 1] exclusive scan of the bounds
  uint32_t* fill;      // [n_seg]
  int64_t cap;
  uint32_t* flags;
};

constexpr int XS_THREADS = 1024;
__global__ __launch_bounds__(XS_THREADS) void k_xsel_scan(
    int mode, int64_t nb, int64_t M, int64_t n_lg,
    const int64_t* __restrict__ lg_off, const int64_t* __restrict__ lg_k,
    const int64_t* __restrict__ lg_ch0, const uint64_t* __restrict__ keys,
    const XSel* __restrict__ sel, uint32_t* __restrict__ hist, XPool pool,
    int64_t* __restrict__ picks) {
  __shared__ uint32_t h[XS_BINS];
  const int tid = threadIdx.x, lane = LANE;
  const int64_t bid = blockIdx.x;
  int64_t a = 0, z = n_lg;
  while (z - a > 1) {
    const int64_t mid = (a + z) >> 1;
    if (lg_ch0[mid] * nb <= bid) a = mid;
    else z = mid;
  }
  const int64_t lg = a;
  const int64_t k = lg_k[lg];
  const int64_t nch = (k + SEL_CHUNK - 1) / SEL_CHUNK;
  const int64_t local = bid - lg_ch0[lg] * nb;
  const int64_t b = local / nch, c = local - b * nch;
  const int64_t seg = lg * nb + b;
  const XSel s = sel[seg];
  const bool hon = (mode & 1) && (s.offset || s.w[0] || s.w[1]);
  const bool app = (mode & 2) && s.ntarget > 0 && (s.done[0] != 1 ||
                                                   (s.ntarget > 1 && s.done[1] != 1));
  const bool pk = (mode & 4) && (s.done[0] == 2 || (s.ntarget > 1 && s.done[1] == 2));
  if (!hon && !app && !pk) return;  // block-uniform
  if (hon)
    for (int j = tid; j < XS_BINS; j += XS_THREADS) h[j] = 0;
  __syncthreads();
  const uint64_t* col = keys + b * M + lg_off[lg];
  const int64_t i0 = c * SEL_CHUNK;
  const int64_t i1 = i0 + SEL_CHUNK < k ? i0 + SEL_CHUNK : k;
  auto one = [&](uint64_t key) {
    const bool valid = key != KEY_NONE;
    if (hon && valid) xs_count(s, key, h);
    if (app) {  // wave ballot: one pool atomic per wave and key slot
      const bool cand = valid && xs_keep(s, key);
      const uint64_t m = __ballot(cand);
      if (m) {
        const int lead = __builtin_ctzll(m);
        uint32_t at = 0;
        if (lane == lead) at = atomicAdd(&pool.fill[seg], (uint32_t)__popcll(m));
        at = (uint32_t)__builtin_amdgcn_readlane((int)at, lead);
        if (cand) {
          const int64_t q = pool.off[seg] + at + __popcll(m & ((1ULL << lane) - 1));
          if (q < pool.off[seg + 1]) {
            pool.key[q] = key;
            pool.seg[q] = seg;
          } else {
            atomicOr(pool.flags, (uint32_t)XS_BROKEN);
          }
        }
      }
    }
    if (pk && valid) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (t < s.ntarget && s.done[t] == 2 && xs_match(s, t, key))
          picks[2 * seg + t] = (int64_t)key;
    }
  };
  // XS_UNROLL keys a lane in flight (wave-strided, so each load is 512
  // coalesced bytes); every lane runs the same trip count (the ballots)
  constexpr int XS_UNROLL = 8;
  const int64_t w0 = i0 + (tid - lane) * XS_UNROLL;
  for (int64_t i = w0; i < i1; i += XS_THREADS * XS_UNROLL) {
    uint64_t kk[XS_UNROLL];
#pragma unroll
    for (int j = 0; j < XS_UNROLL; ++j) {
      const int64_t x = i + 64 * j + lane;
      kk[j] = x < i1 ? col[x] : KEY_NONE;
    }
#pragma unroll
    for (int j = 0; j < XS_UNROLL; ++j) one(kk[j]);
  }
  if (!hon) return;
  __syncthreads();
  uint32_t* g = hist + seg * XS_BINS;
  for (int j = tid; j < XS_BINS; j += XS_THREADS)
    if (h[j]) atomicAdd(&g[j], h[j]);
}

// passes 2+ and the pick over the pool: a few keys per segment, global
// atomics
__global__ __launch_bounds__(256) void k_xsel_pool(
    int mode, XPool pool, const XSel* __restrict__ sel, uint32_t* __restrict__ hist,
    int64_t* __restrict__ picks) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pool.cap;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t seg = pool.seg[i];
    if (seg < 0) continue;  // an unfilled slot
    const uint64_t key = pool.key[i];
    const XSel& s = sel[seg];
    if ((mode & 1) && (s.w[0] || s.w[1])) xs_count(s, key, hist + seg * XS_BINS);
    if (mode & 4) {
      for (int t = 0; t < 2; ++t)
        if (t < s.ntarget && s.done[t] == 2 && xs_match(s, t, key))
          picks[2 * seg + t] = (int64_t)key;
    }
  }
}

// one wave per segment: the global histogram of the pass just run -> each
// target's digit, rank and bin count; resolution; the next pass planned.
// flags: XS_MORE a pass is planned, XS_PICK a target waits for its key
// (set once: a flag word every segment hits is read before its atomic);
// bnd[seg] = the segment's pool bound
__global__ __launch_bounds__(256) void k_xsel_apply(
    int64_t n_seg, const int64_t* __restrict__ seg_k,  // local members (lg_k)
    int64_t nb, const uint32_t* __restrict__ hist, XSel* __restrict__ sel,
    uint32_t* __restrict__ flags, int64_t* __restrict__ bnd) {
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg >= n_seg) return;  // wave-uniform
  const int lane = LANE;
  XSel s = sel[seg];
  const bool ran = s.offset || s.w[0] || s.w[1];
  if (ran) {
    const uint32_t* h = hist + seg * XS_BINS;
    for (int t = 0; t < 2; ++t) {
      const bool in = s.offset ? (t < s.ntarget && s.done[t] == 0) : s.w[t] > 0;
      if (!in) continue;
      const uint32_t* ht = h + (s.split ? t * 1024 : 0);
      const int per = (s.split ? 1024 : XS_BINS) / 64;  // 16 / 32 bins a lane
      // the lane's bins in registers (16-byte loads), summed and searched
      // there
      uint32_t cb[32];
      const uint4* hv = reinterpret_cast<const uint4*>(ht + lane * per);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (q < per / 4) v = hv[q];
        cb[4 * q] = v.x;
        cb[4 * q + 1] = v.y;
        cb[4 * q + 2] = v.z;
        cb[4 * q + 3] = v.w;
      }
      uint32_t sum = 0;
#pragma unroll
      for (int j = 0; j < 32; ++j) sum += cb[j];
      uint32_t incl = sum;
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d);
        if (lane >= d) incl += y;
      }
      const int64_t excl = (int64_t)incl - sum;
      const int64_t rr = s.rank[t];
      const bool mine = rr >= excl && rr < (int64_t)incl;
      int64_t below = 0, cnt = 0;
      int dig = 0;
      if (mine) {
        int64_t cum = excl;
        int jj = per - 1;
        bool found = false;
#pragma unroll
        for (int j = 0; j < 31; ++j) {
          if (!found && j < per - 1) {
            if (rr < cum + cb[j]) {
              jj = j;
              found = true;
            } else {
              cum += cb[j];
            }
          }
        }
        uint32_t cj = 0;
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if (j == jj) cj = cb[j];
        dig = lane * per + jj;
        below = cum;
        cnt = cj;
      }
      const uint64_t who = __ballot(mine);
      if (!who) {  // the rank is past the bins: the ranks' data disagree
        if (lane == 0) atomicOr(flags, (uint32_t)XS_BROKEN);
        s.done[t] = 1;
        s.shift[t] = 0;
        continue;
      }
      const int src = __builtin_ctzll(who);
      dig = __shfl(dig, src);
      below = readlane_l(below, src);
      cnt = readlane_l(cnt, src);
      s.rank[t] = rr - below;
      s.cnt[t] = cnt;
      if (s.offset) {
        s.prefix[t] = (s.base + (uint64_t)dig) << s.s1;
        s.shift[t] = s.s1;
      } else {
        s.shift[t] -= s.w[t];
        s.prefix[t] |= (uint64_t)dig << s.shift[t];
      }
      if (s.shift[t] == 0) s.done[t] = 1;
      else if (cnt == 1) s.done[t] = 2;
    }
  }
  const bool more = xs_plan(s);
  if (lane == 0) {
    sel[seg] = s;
    uint32_t f = more ? (uint32_t)XS_MORE : 0u;
    if (s.done[0] == 2 || (s.ntarget > 1 && s.done[1] == 2)) f |= XS_PICK;
    if (f && (__hip_atomic_load(flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
              f) != f)
      atomicOr(flags, f);
    // the pool's bound: local keys matching a target not resolved to its
    // prefix (one bin when the two share it)
    int64_t cb = 0;
    const bool k0 = s.ntarget > 0 && s.done[0] != 1;
    const bool k1 = s.ntarget > 1 && s.done[1] != 1;
    if (k0) cb += s.cnt[0];
    if (k1 && !(k0 && s.prefix[0] == s.prefix[1] && s.shift[0] == s.shift[1]))
      cb += s.cnt[1];
    const int64_t lk = seg_k[seg / nb];
    if (cb > lk) cb = lk;
    bnd[seg] = cb;
  }
}

// the estimator over the resolved order statistics (k_seg_select's tail)
__global__ void k_xsel_finish(int64_t n_seg, const XSel* __restrict__ sel,
                              const int64_t* __restrict__ picks,
                              const uint8_t* __restrict__ emit,
                              double* __restrict__ out_val, int* err_word,
                              int median, double p,
                              const uint32_t* __restrict__ broken) {
  const int64_t seg = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (seg == 0 && *broken) atomicOr(err_word, ERR_INTERNAL);  // pool overflow
  if (seg >= n_seg || !emit[seg]) return;
  const XSel s = sel[seg];
  double r = qnan();
  if (s.ntarget > 0) {
    uint64_t v[2] = {0, 0};
    for (int t = 0; t < s.ntarget; ++t) {
      if (s.done[t] == 1) v[t] = s.prefix[t];
      else if (s.done[t] == 2) v[t] = (uint64_t)picks[2 * seg + t];
      else atomicOr(err_word, ERR_INTERNAL);
    }
    if (s.ntarget == 1) v[1] = v[0];
    double pos = 0.0;
    int64_t r0, r1;
    sel_ranks(median, p, s.n, &r0, &r1, &pos);
    r = sel_value(median, s.n, pos, key_value(v[0]), key_value(v[1]));
  }
  if (is_inf(r)) atomicOr(err_word, ERR_INFINITY);
  out_val[seg] = r;
}

}  // namespace otsdb
