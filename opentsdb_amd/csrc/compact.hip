// compact.hip — the last stage of a query: dense (group, bucket) results ->
// the per-group (timestamp, value) arrays of otsdb_result (offsets[G+1]),
// plus the call's {error word, total points} for finish's single read.
// Included by engine.hip only (the pipeline's other kernels never call it).
#pragma once
// (included after kernels.hip: Params, bucket_ts, LANE)

namespace otsdb {

// ------------------------------------------------------------------------
// k_compact1: dense (group, bucket) results -> per-group (ts, value) arrays
// in ONE pass (count, exclusive scan across groups, scatter), the scan by
// decoupled look-back.  One wavefront per
// group, groups taken in ticket order (a block's logical index is an atomic
// ticket, so every group it waits for belongs to a block that has already
// started: no dependence on dispatch order or co-residency beyond that).  Each wave publishes its
// group's count as an 8-byte granule {epoch:24, status:2, value:38} — the
// data is the flag (status 1 = this group's count, 2 = the inclusive
// prefix) — reads up to 64 predecessors' granules at once, sums back to the
// nearest inclusive one, publishes its own inclusive prefix and scatters.
// The epoch (per call, never 0) retires the previous call's granules
// without a memset; the last group also writes offsets[G] and the call's
// {error word, total points} pair for one read-back, and zeroes the error
// word for the next call (the engine's memset of it is skipped then).
// ------------------------------------------------------------------------
constexpr int kCmpSlots = 4;  // ticket counters, one per call in rotation
constexpr int kCmpStatusShift = 38;
constexpr int kCmpEpochShift = 40;
constexpr uint64_t kCmpValueMask = (1ULL << kCmpStatusShift) - 1;
constexpr int kCmpRegChunks = 32;  // k_compact1 holds grids of 64 x this
constexpr int64_t kCmpRegBuckets = 64 * kCmpRegChunks;

// emitted buckets of one group's row of nb emit bytes (0 / 1), by the whole
// wavefront: 16-byte loads aligned down from the row start (rows of nb bytes
// start anywhere; the named query's 10,081-byte rows read byte by byte took
// 0.24 ms), the bytes outside the row masked off
DEV int compact_count(const uint8_t* __restrict__ em, int64_t nb, int lane) {
  const uint8_t* a0 =
      reinterpret_cast<const uint8_t*>((uintptr_t)em & ~(uintptr_t)15);
  const int64_t head = em - a0;  // 0 .. 15
  const int64_t span = head + nb;
  auto nz = [](uint32_t w) {  // non-zero bytes of w
    return __builtin_popcount((((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) &
                              0x80808080u);
  };
  // the bytes [lo, hi) of a 4-byte word as a mask
  auto bytes = [](int lo, int hi) -> uint32_t {
    const uint32_t l = lo <= 0 ? ~0u : (lo >= 4 ? 0u : (~0u << (8 * lo)));
    const uint32_t h = hi >= 4 ? ~0u : (hi <= 0 ? 0u : (~0u >> (32 - 8 * hi)));
    return l & h;
  };
  int n = 0;
  for (int64_t c0 = 0; c0 < span; c0 += 1024) {
    const int64_t o = c0 + 16 * lane;
    if (o < span) {
      const uint4 x = *reinterpret_cast<const uint4*>(a0 + o);
      const uint32_t w[4] = {x.x, x.y, x.z, x.w};
      const int lo = o < head ? (int)(head - o) : 0;
      const int hi = span - o < 16 ? (int)(span - o) : 16;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        n += nz((lo == 0 && hi == 16) ? w[i]
                                      : w[i] & bytes(lo - 4 * i, hi - 4 * i));
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d);
  return n;
}

// Long grids (more than 2,048 buckets: the named query's 10,081) take three
// launches instead: the single pass's count phase is long enough there that
// most waves reach the look-back together and walk far back for an
// inclusive prefix (the named query's compaction: 1.2 ms).
// k_compact_count (each wave counts its group's emitted buckets) -> k_scan
// (offsets) -> k_compact_scatter.
// zeroes is_int[a, min(e, cap)) — every compacted point is a double — with
// 16-byte stores between the aligned ends (64 one-byte stores a wave
// instruction cost the scatter more than its 16 bytes of ts and value)
DEV void zero_bytes(uint8_t* __restrict__ r, int64_t a, int64_t e, int64_t cap,
                    int lane) {
  if (e > cap) e = cap;
  if (a >= e) return;
  uint8_t* pa = r + a;
  uint8_t* pe = r + e;
  uint8_t* qa = reinterpret_cast<uint8_t*>(((uintptr_t)pa + 15) & ~(uintptr_t)15);
  uint8_t* qe = reinterpret_cast<uint8_t*>((uintptr_t)pe & ~(uintptr_t)15);
  if (qa > pe) qa = pe;
  if (qe < qa) qe = qa;
  for (uint8_t* x = pa + lane; x < qa; x += 64) *x = 0;
  for (uint8_t* x = qa + 16 * lane; x < qe; x += 1024)
    *reinterpret_cast<uint4*>(x) = make_uint4(0, 0, 0, 0);
  for (uint8_t* x = qe + lane; x < pe; x += 64) *x = 0;
}

__global__ __launch_bounds__(256) void k_compact_count(
    Params P, int64_t G, const uint8_t* __restrict__ out_emit,
    int64_t* __restrict__ counts, unsigned long long* __restrict__ ticket,
    uint32_t epoch) {
  const int lane = LANE;
  // k_compact1's ticket slots rotate with the epoch whichever path a call
  // takes: clear the next call's slot as its last block would
  if (blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(ticket + ((epoch + 1) & (kCmpSlots - 1)), 0ULL,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t g = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (g >= G) return;
  const int64_t n = compact_count(out_emit + g * P.nb, P.nb, lane);
  if (lane == 0) counts[g] = n;
}

__global__ __launch_bounds__(256) void k_compact_scatter(
    Params P, int64_t G, const double* __restrict__ out_val,
    const uint8_t* __restrict__ out_emit, const int64_t* __restrict__ counts,
    const int64_t* __restrict__ offsets, int64_t cap,
    int64_t* __restrict__ r_ts, int64_t* __restrict__ r_val,
    uint8_t* __restrict__ r_isint, int* err_word, int64_t* __restrict__ small) {
  const int lane = LANE;
  const int64_t g = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (g >= G) return;
  const int64_t nb = P.nb;
  const int64_t prefix = offsets[g];
  if (lane == 0 && g == G - 1) {
    small[1] = offsets[G];
    small[0] = (int64_t)(uint32_t)__hip_atomic_exchange(
        err_word, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const uint8_t* em = out_emit + g * nb;
  constexpr int U = 16;
  zero_bytes(r_isint, prefix, prefix + counts[g], cap, lane);
  if (counts[g] == nb) {
    // every bucket emitted (dense series): a straight copy, no flags read
    const double* src = out_val + g * nb;
    for (int64_t c0 = 0; c0 < nb; c0 += 64 * U) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t b = c0 + 64 * u + lane;
        v[u] = b < nb ? src[b] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t b = c0 + 64 * u + lane;
        const int64_t p = prefix + b;
        if (b < nb && p < cap) {
          r_ts[p] = bucket_ts(P, b);
          r_val[p] = __double_as_longlong(v[u]);
        }
      }
    }
    return;
  }
  int64_t pos = prefix;
  for (int64_t c0 = 0; c0 < nb; c0 += 64 * U) {
    bool e[U];
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t b = c0 + 64 * u + lane;
      e[u] = b < nb && em[b];
      v[u] = b < nb ? out_val[g * nb + b] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t b = c0 + 64 * u + lane;
      const uint64_t m = __ballot(e[u]);
      if (e[u]) {
        const int64_t p = pos + __popcll(m & ((1ULL << lane) - 1));
        if (p < cap) {
          r_ts[p] = bucket_ts(P, b);
          r_val[p] = __double_as_longlong(v[u]);
        }
      }
      pos += __popcll(m);
    }
  }
}

__global__ __launch_bounds__(256) void k_compact1(
    Params P, int64_t G, const double* __restrict__ out_val,
    const uint8_t* __restrict__ out_emit, unsigned long long* __restrict__ flags,
    unsigned long long* __restrict__ ticket, uint32_t epoch,
    int64_t* __restrict__ offsets, int64_t cap,
    int64_t* __restrict__ r_ts, int64_t* __restrict__ r_val,
    uint8_t* __restrict__ r_isint, int* err_word, int64_t* __restrict__ small) {
  __shared__ unsigned long long s_blk;
  const int lane = LANE, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    // this call's ticket counter: slot epoch % kCmpSlots (zero: the previous
    // call's last block cleared it); the last block clears the next call's
    unsigned long long* tk = ticket + (epoch & (kCmpSlots - 1));
    const unsigned long long t = __hip_atomic_fetch_add(
        tk, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 == gridDim.x)
      __hip_atomic_store(ticket + ((epoch + 1) & (kCmpSlots - 1)), 0ULL,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_blk = t;
  }
  __syncthreads();
  const int64_t g = (int64_t)s_blk * (blockDim.x >> 6) + w;
  if (g >= G) return;
  const int64_t nb = P.nb;
  const uint8_t* em = out_emit + g * nb;
  // grids of up to 2,048 buckets (C1's 1,440, C2's 2,017; the engine sends
  // longer ones to the three-launch path above): every emit flag and value
  // read ONCE (lane = bucket, coalesced) and held in registers across the
  // look-back, the count from the ballots
  constexpr int U2 = kCmpRegChunks;
  uint64_t bm[U2];
  double vv[U2];
  int64_t n = 0;
#pragma unroll
  for (int u = 0; u < U2; ++u) {
    const int64_t b = 64 * u + lane;
    const bool in = b < nb;
    vv[u] = in ? out_val[g * nb + b] : 0.0;
    bm[u] = __ballot(in && em[b]);
    n += __popcll(bm[u]);
  }
  const uint64_t tag = (uint64_t)epoch << kCmpEpochShift;
  if (lane == 0)
    __hip_atomic_store(&flags[g], tag | (1ULL << kCmpStatusShift) | (uint64_t)n,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // look back: lane l reads group j - l; sum every published count down to
  // (and including) the nearest inclusive prefix
  int64_t prefix = 0;
  int64_t j = g - 1;
  unsigned spins = 0;
  while (j >= 0) {
    const int64_t k = j - lane;
    uint64_t v = 0;
    if (k >= 0)
      v = __hip_atomic_load(&flags[k], __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
    const bool cur = k < 0 || (v >> kCmpEpochShift) == epoch;
    const uint32_t st = k < 0 ? 2u : (uint32_t)((v >> kCmpStatusShift) & 3);
    const uint64_t incl = __ballot(cur && st == 2);
    const int stop = incl ? __builtin_ctzll(incl) : 64;  // nearest inclusive
    const uint64_t upto = stop == 64 ? ~0ULL : ((2ULL << stop) - 1);
    if (__ballot(!cur) & upto) {  // a predecessor not published yet
      if (++spins > (1u << 22)) {  // (bounded: never expected)
        // reported through host memory: the last group may have swapped
        // the error word out already (finish reads small[2])
        if (lane == 0) {
          atomicOr(err_word, ERR_INTERNAL);
          __hip_atomic_store(&small[2], (int64_t)1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    int64_t x = (k >= 0 && (uint64_t)lane <= (uint64_t)stop)
                    ? (int64_t)(v & kCmpValueMask) : 0;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
    prefix += x;
    if (stop < 64) break;
    j -= 64;
  }
  if (lane == 0) {
    __hip_atomic_store(&flags[g],
                       tag | (2ULL << kCmpStatusShift) | (uint64_t)(prefix + n),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    offsets[g] = prefix;
    if (g == G - 1) {
      offsets[G] = prefix + n;
      small[1] = prefix + n;
      // every kernel that reports into the error word ran before this one
      small[0] = (int64_t)(uint32_t)__hip_atomic_exchange(
          err_word, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  zero_bytes(r_isint, prefix, prefix + n, cap, lane);
  int64_t pos = prefix;
#pragma unroll
  for (int u = 0; u < U2; ++u) {
    const int64_t b = 64 * u + lane;
    const uint64_t m = bm[u];
    if ((m >> lane) & 1) {
      const int64_t p = pos + __popcll(m & ((1ULL << lane) - 1));
      if (p < cap) {
        r_ts[p] = bucket_ts(P, b);
        r_val[p] = __double_as_longlong(vv[u]);
      }
    }
    pos += __popcll(m);
  }
}

}  // namespace otsdb
