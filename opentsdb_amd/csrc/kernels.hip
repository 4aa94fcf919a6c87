// kernels.hip — device code of the aggregation engine (gfx950, wave64).
// See kernels.h for the pipeline.  Reference semantics cited per kernel
// (paths under /root/reference).
//
// Compiled with -ffp-contract=off: Java evaluates `y0 + (x-x0)*(y1-y0)/(x1-x0)`
// and every aggregator loop with separate roundings, so no FMA may be formed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace otsdb {

#define LANE (threadIdx.x & 63)

DEV double bits_to_double(int64_t b) { return __longlong_as_double(b); }

// Java `t - t % interval` (Downsampler.alignTimestamp, Downsampler.java:452)
DEV int64_t align_ts(int64_t t, int64_t iv) { return t - t % iv; }

// floor(rel / interval) for rel >= 0 without a 64-bit divide: double
// reciprocal estimate + one correction step each way.
// calendar grid: the b with cal[b] <= ts < cal[b+1] (binary search over the
// table; clamped to [cal_lo - 1, cal_n - 1] outside it)
DEV int64_t cal_bucket(const Params& P, int64_t ts) {
  int64_t lo = P.cal_lo, hi = P.cal_n;  // first index with cal[i] > ts
  while (lo < hi) {
    const int64_t m = lo + ((hi - lo) >> 1);
    if (P.cal[m] <= ts) lo = m + 1;
    else hi = m;
  }
  return lo - 1;
}

DEV int64_t bucket_of(const Params& P, int64_t ts) {
  if (P.run_all) return 0;
  if (P.cal) return cal_bucket(P, ts);
  const int64_t rel = ts - P.gbase;
  int64_t q = (int64_t)((double)rel * P.inv_interval);
  int64_t r = rel - q * P.interval;
  if (r < 0) { --q; r += P.interval; }
  if (r < 0) { --q; r += P.interval; }
  if (r >= P.interval) { ++q; r -= P.interval; }
  if (r >= P.interval) { ++q; }
  return q;
}

DEV int64_t bucket_ts(const Params& P, int64_t b) {
  return P.run_all ? P.out_ts0 : P.cal ? P.cal[b] : P.gbase + b * P.interval;
}

DEV double point_value(const BatchDev& B, int64_t i, int64_t bits, int sf) {
  const int f = B.is_float ? (int)B.is_float[i] : sf;
  return f ? bits_to_double(bits) : (double)bits;
}

// first index in [a, b) with ts >= t (the seek of Span.Iterator /
// MockSeekableView on sorted points)
DEV int64_t lower_bound(const int64_t* ts, int64_t a, int64_t b, int64_t t) {
  while (a < b) {
    const int64_t m = a + ((b - a) >> 1);
    if (ts[m] < t) a = m + 1;
    else b = m;
  }
  return a;
}

// lower_bound over [a, b) that first tests the ends: when the whole series
// lies on one side of t (every series of a whole-range query) no search runs
// — the dependent-load chain of the binary search was most of k_prep.
// Otherwise an interpolated first probe: series sampled at a near-regular
// interval put the answer within a few points of the linear guess, so a
// gallop from it brackets the answer in 2-3 dependent loads instead of
// log2(n) ≈ 12 (k_fold_prep's window edges).  Same result as lower_bound
// for any sorted input: the guess only picks where the bracketing starts.
DEV int64_t lower_bound_interp(const int64_t* ts, int64_t a, int64_t b,
                               int64_t t) {
  if (a >= b) return a;
  const int64_t ta = ts[a];
  if (ta >= t) return a;
  const int64_t tb = ts[b - 1];
  if (tb < t) return b;
  int64_t lo = a, hi = b - 1;  // ts[lo] < t <= ts[hi]
  if (hi - lo > 1) {
    const double f = (double)(t - ta) / (double)(tb - ta);
    int64_t g = lo + (int64_t)(f * (double)(hi - lo));
    g = g <= lo ? lo + 1 : (g >= hi ? hi - 1 : g);
    if (ts[g] < t) {
      lo = g;
      for (int64_t step = 1;; step <<= 1) {
        const int64_t h = lo + step;
        if (h >= hi) break;
        if (ts[h] >= t) { hi = h; break; }
        lo = h;
      }
    } else {
      hi = g;
      for (int64_t step = 1;; step <<= 1) {
        const int64_t l = hi - step;
        if (l <= lo) break;
        if (ts[l] < t) { lo = l; break; }
        hi = l;
      }
    }
  }
  return lower_bound(ts, lo + 1, hi, t);
}

// lower_bound over [a, b) in two rounds of loads for near-regular series:
// the ends, then the 8 points around the interpolated guess, which hold the
// answer unless the cadence is irregular there (then lower_bound_interp's
// gallop).  k_fold_prep's window edges: a chain of 4-6 dependent loads was
// most of that latency-bound kernel.
DEV int64_t lower_bound_near(const int64_t* ts, int64_t a, int64_t b,
                             int64_t t) {
  if (a >= b) return a;
  const int64_t ta = ts[a];
  if (ta >= t) return a;
  const int64_t tb = ts[b - 1];
  if (tb < t) return b;
  // ts[a] < t <= ts[b - 1]
  const double f = (double)(t - ta) / (double)(tb - ta);
  const int64_t g = a + (int64_t)(f * (double)(b - 1 - a));
  int64_t base = g - 4;
  if (base > b - 8) base = b - 8;
  if (base < a) base = a;
  int cnt = 0;
  bool last_ge = false;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int64_t i = base + u;
    const int64_t x = i < b ? ts[i] : INT64_MAX;
    cnt += x < t ? 1 : 0;
    if (u == 0 && x >= t && base > a) last_ge = true;  // answer before base
  }
  if (!last_ge && cnt < 8) return base + cnt;
  return lower_bound_interp(ts, a, b, t);
}

// lower bound of t in [a, b) found by galloping back from b - 1: the start
// of the bucket that holds ts[b - 1] lies a few points before it
DEV int64_t lower_bound_back(const int64_t* ts, int64_t a, int64_t b,
                             int64_t t) {
  if (a >= b || ts[b - 1] < t) return b;
  int64_t hi = b - 1, lo = a - 1;  // ts[hi] >= t; ts[lo] < t (lo = a-1: none)
  for (int64_t step = 1;; step <<= 1) {
    const int64_t l = hi - step;
    if (l <= lo) break;
    if (ts[l] < t) { lo = l; break; }
    hi = l;
  }
  return lower_bound(ts, lo + 1, hi, t);
}

DEV int64_t wave_incl_max(int64_t x) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(x, d);
    if (LANE >= d) x = x > y ? x : y;
  }
  return x;
}

// ------------------------------------------------------------------------
// k_prep: SpanGroup.add filter (SpanGroup.java:321-338), the Downsampler
// seek (ValuesInInterval.seekInterval rounds up, Downsampler.java:431) or
// the "all" bounds (Downsampler.java:354-379), and the first bucket past the
// window (the point AggregationIterator keeps in its "next" slot, used to
// interpolate up to end_time, AggregationIterator.java:760-775).
// One thread per series.
// ------------------------------------------------------------------------
DEV void k_prep_store(const Params& P, const BatchDev& B, SeriesMeta SM,
                      int64_t s, bool keep, int64_t lo, int64_t hi,
                      uint8_t of_has, int64_t of_ts, double of_val) {
  SM.keep[s] = keep;
  SM.lo[s] = lo;
  SM.hi[s] = hi;
  const bool any = keep && lo < hi;
  SM.kf[s] = any ? (int32_t)bucket_of(P, B.ts[lo]) : 0;
  SM.kl[s] = any ? (int32_t)bucket_of(P, B.ts[hi - 1]) : -1;
  SM.of_has[s] = of_has;
  SM.of_ts[s] = of_ts;
  SM.of_val[s] = of_val;
}

// RateSpan's rate between two bucket points (RateSpan.java:121-180); kept =
// false for a counter reset RateSpan drops (dropResets)
DEV double rate_between(const Params& P, int64_t t0, double v0, int64_t t1,
                        double v1, bool* kept) {
  const double dt = (double)(t1 - t0) / 1000.0;
  double diff = v1 - v0;
  *kept = true;
  if (P.counter && diff < 0) {
    if (P.drop_resets) {
      *kept = false;
      return 0.0;
    }
    diff = (double)P.counter_max - v0 + v1;
    const double r = diff / dt;
    return (P.reset_value > 0 && r > (double)P.reset_value) ? 0.0 : r;
  }
  return diff / dt;
}

// Rate queries: the kept rates AFTER the first bucket past the window.  The
// reference's rate mode pre-consumes each span's first (junk) rate and keeps
// the span contributing while it has a second one (AggregationIterator.java:
// 448-459) — those rates may all lie past the window (a series whose
// outage covers the whole window), so the bucket past it is not enough.
// next(): fills (t, v) with the next bucket point after the previous one,
// false when the span has no more.  Returns the count (capped at 2) and the
// first rate in *r1.
template <class Next>
DEV int rates_beyond(const Params& P, int64_t t, double v, Next&& next,
                     double* r1) {
  int n = 0;
  int64_t tn;
  double vn;
  for (int guard = 0; n < 2 && guard < (1 << 20) && next(&tn, &vn); ++guard) {
    bool kept;
    const double r = rate_between(P, t, v, tn, vn, &kept);
    if (kept && n++ == 0) *r1 = r;
    t = tn;
    v = vn;  // RateSpan continues from a dropped reset's point too
  }
  return n;
}

// one series' k_prep: keep / lo / hi always; with `full` also the point
// past the window and the stores (k_prep_fold's other threads of the series
// need only the bounds)
template <class M>
DEV void prep_series(const Params& P, const BatchDev& B, SeriesMeta SM,
                     int* err_word, int64_t s, bool full, bool* keep_o,
                     int64_t* lo_o, int64_t* hi_o) {
  const int64_t p0 = B.offsets[s], p1 = B.offsets[s + 1];
  const bool keep = p1 > p0 && B.ts[p0] <= P.end_ms && B.ts[p1 - 1] >= P.start_ms;
  int64_t lo = p1, hi = p1;
  if (keep) {
    lo = lower_bound_interp(B.ts, p0, p1, P.seek_ts);
    hi = lower_bound_interp(B.ts, lo, p1, P.stop_ts);
  }
  *keep_o = keep;
  *lo_o = lo;
  *hi_o = hi;
  if (!full) return;
  SM.keep[s] = keep;
  uint8_t of_has = 0;
  int64_t of_ts = 0;
  double of_val = 0.0;
  if (keep) {
    if (!P.run_all && P.fill == 0 && hi < p1) {
      const int sf = B.series_float ? (int)B.series_float[s] : 1;
      const int64_t t = B.ts[hi];
      int64_t e;
      if (P.cal) {  // the calendar bucket holding t (Downsampler.java:383-397)
        const int64_t k = cal_bucket(P, t);
        if (k < P.cal_lo || k + 1 >= P.cal_n) {
          atomicOr(err_word, ERR_CAL_RANGE);
          k_prep_store(P, B, SM, s, keep, lo, hi, 0, 0, 0.0);
          return;
        }
        of_ts = P.cal[k];
        e = P.cal[k + 1];
      } else {
        of_ts = align_ts(t, P.interval);
        e = of_ts + P.interval;
      }
      M st = M::init();
      int64_t i = hi;
      for (; i < p1 && B.ts[i] < e; ++i)
        st.push(point_value(B, i, B.val[i], sf));
      int err = 0;
      of_val = st.finish(&err);
      of_has = 1;
      // (percentile downsampling: the bucket values here are counts —
      // k_ds_select fills of_val, of_rate and the rate bits later)
      if (P.rate && !P.ds_sel) {
        // the next bucket points: fixed-interval buckets (the row path takes
        // rate queries; calendar grids step their table)
        auto next = [&](int64_t* tn, double* vn) -> bool {
          if (i >= p1) return false;
          int64_t bt, be;
          if (P.cal) {
            const int64_t k = cal_bucket(P, B.ts[i]);
            if (k < P.cal_lo || k + 1 >= P.cal_n) return false;
            bt = P.cal[k];
            be = P.cal[k + 1];
          } else {
            bt = align_ts(B.ts[i], P.interval);
            be = bt + P.interval;
          }
          M b = M::init();
          for (; i < p1 && B.ts[i] < be; ++i)
            b.push(point_value(B, i, B.val[i], sf));
          int e2 = 0;
          *tn = bt;
          *vn = b.finish(&e2);
          return true;
        };
        double r1 = 0.0;
        const int kb = rates_beyond(P, of_ts, of_val, next, &r1);
        of_has |= (uint8_t)(kb << 1);
        SM.of_rate[s] = r1;
      }
    }
  }
  k_prep_store(P, B, SM, s, keep, lo, hi, of_has, of_ts, of_val);
}

template <class M>
__global__ void k_prep(Params P, BatchDev B, SeriesMeta SM, int* err_word) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= B.S) return;
  bool keep;
  int64_t lo, hi;
  prep_series<M>(P, B, SM, err_word, s, true, &keep, &lo, &hi);
}

// ------------------------------------------------------------------------
// k_bucketize_k: the same reduction with K consecutive points per lane
// (K/2 16-byte loads per column per lane; a step covers 64*K points).  Each
// lane folds its points sequentially (Java order inside the lane), closes
// the buckets that start and end inside it, and hands its first ("head")
// and last ("tail") runs to a segmented wave scan over the tails — so the
// cross-lane scan is paid once per 64*K points instead of once per 128.
// ------------------------------------------------------------------------
typedef long long ll2_t __attribute__((ext_vector_type(2)));

// Bucket index when the grid spans < 2^32 ms (P.narrow): a 32-bit relative
// time, a double-reciprocal estimate and one exact correction — branch free.
DEV int bucket_narrow(const Params& P, int64_t ts) {
  if (P.run_all) return 0;
  const uint32_t rel = (uint32_t)(ts - P.gbase);
  const uint32_t iv = (uint32_t)P.interval;
  uint32_t q = (uint32_t)((double)rel * P.inv_interval);
  const uint32_t r = rel - q * iv;
  q = ((int32_t)r < 0) ? q - 1 : (r >= iv ? q + 1 : q);
  return (int)q;
}

// Point times on the bucket grid: absolute ms (int64_t), or on narrow grids
// ms since the grid base (uint32_t: the cells fold, whose 32-bit times save
// the 64-bit adds, compares and registers of the absolute ones).
DEV int bucket_rel(const Params& P, uint32_t rel) {
  if (P.run_all) return 0;
  const uint32_t iv = (uint32_t)P.interval;
  uint32_t q = (uint32_t)((double)rel * P.inv_interval);
  const uint32_t r = rel - q * iv;
  q = ((int32_t)r < 0) ? q - 1 : (r >= iv ? q + 1 : q);
  return (int)q;
}
DEV int tbucket_narrow(const Params& P, int64_t t) { return bucket_narrow(P, t); }
DEV int tbucket_narrow(const Params& P, uint32_t t) { return bucket_rel(P, t); }
DEV int64_t tbucket(const Params& P, int64_t t) { return bucket_of(P, t); }
DEV int64_t tbucket(const Params& P, uint32_t t) { return bucket_rel(P, t); }
// the start of bucket k on a fixed grid / its end for fold_lane
DEV int64_t tstart_fixed(const Params& P, int64_t k, int64_t) {
  return P.gbase + k * P.interval;
}
DEV uint32_t tstart_fixed(const Params& P, int64_t k, uint32_t) {
  return (uint32_t)(k * P.interval);
}
DEV int64_t tbound(const Params& P, int64_t k, int64_t) {
  return P.run_all ? INT64_MAX : bucket_ts(P, k);
}
DEV uint32_t tbound(const Params& P, int64_t k, uint32_t) {
  return P.run_all ? 0xFFFFFFFFu : (uint32_t)(k * P.interval);
}
template <class TT> DEV TT tmin();
template <> DEV int64_t tmin<int64_t>() { return INT64_MIN; }
template <> DEV uint32_t tmin<uint32_t>() { return 0u; }

DEV void wait_vmcnt(int n) {
  // s_waitcnt vmcnt(n) (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14,
  // expcnt and lgkmcnt at their no-wait maxima)
  switch (n) {
#define OTSDB_W(N) case N: __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (0x7 << 4) | (0xF << 8) | (((N) >> 4) << 14)); break;
    OTSDB_W(0) OTSDB_W(1) OTSDB_W(2) OTSDB_W(3) OTSDB_W(4) OTSDB_W(5)
    OTSDB_W(6) OTSDB_W(7) OTSDB_W(8) OTSDB_W(9) OTSDB_W(10) OTSDB_W(11)
    OTSDB_W(12) OTSDB_W(13) OTSDB_W(14) OTSDB_W(15) OTSDB_W(16) OTSDB_W(17)
    OTSDB_W(18) OTSDB_W(19) OTSDB_W(20) OTSDB_W(21) OTSDB_W(22) OTSDB_W(23)
    OTSDB_W(24) OTSDB_W(25) OTSDB_W(26) OTSDB_W(27) OTSDB_W(28) OTSDB_W(29)
    OTSDB_W(30) OTSDB_W(31) OTSDB_W(32)
#undef OTSDB_W
    default: __builtin_amdgcn_s_waitcnt(0x7F << 4); break;  // vmcnt(0)
  }
}

// L2 prefetch of a stream's bytes some steps ahead: each lane loads one
// dword of every 64-byte stretch (a step's lines, one load per lane) into a
// register the stream only retires at its next step, after that step's own
// loads are issued.  The point streams are bound by the bytes a wavefront
// keeps in flight at their occupancy; this adds the lines of a later step
// for one VGPR and one load per array.  Distances are build knobs
// (OTSDB_PF_FOLD / _CELLS / _BUCK, steps ahead, 0 = off).
#ifndef OTSDB_PF_FOLD
#define OTSDB_PF_FOLD 0
#endif
#ifndef OTSDB_PF_CELLS
#define OTSDB_PF_CELLS 0
#endif
#ifndef OTSDB_PF_BUCK
#define OTSDB_PF_BUCK 0
#endif
struct L2Touch {
  uint32_t v = 0;
  DEV void touch(const void* p) { v = *reinterpret_cast<const uint32_t*>(p); }
  // the data is never used: an empty asm only makes the register live, so
  // the wait for it lands here (a step later), not at the touch
  DEV void retire() { asm volatile("" ::"v"(v)); }
};

DEV double readlane_d(double x, int l) {
  const int64_t b = __builtin_bit_cast(int64_t, x);
  const int32_t lo = __builtin_amdgcn_readlane((int32_t)(uint32_t)b, l);
  const int32_t hi = __builtin_amdgcn_readlane((int32_t)(b >> 32), l);
  return __builtin_bit_cast(double, (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
DEV int64_t readlane_l(int64_t b, int l) {
  const int32_t lo = __builtin_amdgcn_readlane((int32_t)(uint32_t)b, l);
  const int32_t hi = __builtin_amdgcn_readlane((int32_t)(b >> 32), l);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Where closed buckets go.  Directly (one scattered 8-B value store and one
// 1-B state store per closing lane), or through a per-wavefront LDS ring of
// WIN bucket values that sink_flush drains in runs of 64 consecutive buckets,
// absent ones included (kAbsentBits): the row leaves the CU as contiguous
// 512-B stores and no state byte is written (k_transform derives the states,
// Params.sentinel) — the scattered stores cost 2 of k_bucketize's 17 ms on
// C2.
struct RowSink {
  double* rowv;
  uint8_t* rows;
  double* rv;      // LDS ring values, or null
  int mask;        // WIN - 1
  int direct;      // wave-uniform: write straight to HBM this step
  int states;      // direct writes also store the state byte (no ring)
  int nostore;     // tuning ablation (ABL == 2): the flush stores nothing
  int nt;          // flush with non-temporal stores
  DEV void put(int k, double v) {
    if (states) {
      rowv[k] = v;
      rows[k] = ST_REAL;
      return;
    }
    v = is_nan(v) ? qnan() : v;  // never the absent pattern
    if (direct) rowv[k] = v;
    else rv[k & mask] = v;
  }
};

DEV double absent_value() { return __longlong_as_double(kAbsentBits); }

// RateSpan over a series' bucket points, carried across ring flushes
// (k_transform's two passes, transform_rate, folded into the flush of each
// run of 64 final buckets): the previous point of pass 1, the first kept
// rate (the junk one), and the latest kept rate pass 2 holds.
struct RateState {
  int64_t carry_pts;   // last real bucket (pass 1's previous point)
  double carry_pv;
  int64_t r0_idx;      // first kept rate
  double r0_val;
  int64_t last_kept;
  int64_t carry_k;     // latest kept rate
  double carry_kv;
  int kept_count;      // capped at 2
  int bad;             // non-increasing timestamps (fallback reports it)
};

// One run of final buckets [f, min(f + 64, limit)) of the ring through
// RateSpan (RateSpan.java:103-180) and the rate-mode contribution rule
// (AggregationIterator.java:448-459, :744-753): each bucket gets its rate
// (ST_REAL) or the latest kept rate at or before it (ST_INTERP), exactly as
// transform_rate's passes; what depends on the whole series (buckets before
// the first kept rate, after the last one, fewer than two rates) is fixed
// by rate_finish.
DEV void rate_flush(const Params& P, RowSink& S, RateState& R, int64_t f,
                    int64_t limit) {
  const int lane = LANE;
  const int64_t b = f + lane;
  const bool inb = b < limit;
  double v = 0.0;
  if (inb) {
    const int i = (int)(b & S.mask);
    v = S.rv[i];
    S.rv[i] = absent_value();
  }
  const bool p = inb && __double_as_longlong(v) != kAbsentBits;
  const int64_t t = inb ? bucket_ts(P, b) : 0;
  const uint64_t pm = __ballot(p);
  const uint64_t im = __ballot(inb);
  const uint64_t below = pm & ((1ULL << lane) - 1);
  const int pl = below ? 63 - __builtin_clzll(below) : -1;
  // every bucket of the run present (dense series): the previous point is
  // the lane before (a DPP shift, not a lane shuffle)
  double vp;
#ifndef OTSDB_RATE_SHFL  // tuning builds: lane shuffles only
  if (pm == im) vp = dppd<0x138, 0xF>(v);
  else
#endif
    vp = __shfl(v, pl >= 0 ? pl : 0);
  const int64_t tprev = pl >= 0 ? bucket_ts(P, f + pl) : R.carry_pts;
  const double vprev = pl >= 0 ? vp : R.carry_pv;
  bool kept = false;
  double rate = 0.0;
  if (p) {
    if (t <= tprev) R.bad = 1;
    const double dt = (double)(t - tprev) / 1000.0;
    double diff = v - vprev;
    if (P.counter && diff < 0) {
      if (!P.drop_resets) {
        kept = true;
        diff = (double)P.counter_max - vprev + v;
        const double r = diff / dt;
        rate = (P.reset_value > 0 && r > (double)P.reset_value) ? 0.0 : r;
      }
    } else {
      kept = true;
      rate = diff / dt;
    }
  }
  const bool k = p && kept;
  const uint64_t km = __ballot(k);
  if (km) {
    const int f0 = __builtin_ctzll(km);
    const double rf = readlane_d(rate, f0);
    if (R.r0_idx < 0) {
      R.r0_idx = f + f0;
      R.r0_val = rf;
    }
    R.kept_count += __popcll(km);
    if (R.kept_count > 2) R.kept_count = 2;
    R.last_kept = f + 63 - __builtin_clzll(km);
  }
  if (pm) {
    const int l = 63 - __builtin_clzll(pm);
    R.carry_pts = bucket_ts(P, f + l);
    R.carry_pv = readlane_d(v, l);
  }
  // pass 2: latest kept rate at or before each bucket
  const double kv = k ? rate : 0.0;
  const uint64_t upto = km & ((2ULL << lane) - 1);
  const int il = upto ? 63 - __builtin_clzll(upto) : -1;
  // every bucket of the run kept: its own rate
  double lv;
#ifndef OTSDB_RATE_SHFL
  if (km == im) lv = kv;
  else
#endif
    lv = __shfl(kv, il >= 0 ? il : 0);
  const double held = il >= 0 ? lv : (R.carry_k >= 0 ? R.carry_kv : R.r0_val);
  if (inb) {
    const bool real = k && b != R.r0_idx;
    if (S.nt) {
      __builtin_nontemporal_store(real ? kv : held, &S.rowv[b]);
      __builtin_nontemporal_store((uint8_t)(real ? ST_REAL : ST_INTERP), &S.rows[b]);
    } else {
      S.rowv[b] = real ? kv : held;
      S.rows[b] = real ? ST_REAL : ST_INTERP;
    }
  }
  if (km) {
    const int l = 63 - __builtin_clzll(km);
    R.carry_k = f + l;
    R.carry_kv = readlane_d(kv, l);
  }
}

// drains the ring's buckets [flushed, limit) (all final) to the row
template <int RATE = 0>
DEV void sink_flush(RowSink& S, int64_t& flushed, int64_t limit,
                    const Params* P = nullptr, RateState* R = nullptr) {
  const int lane = LANE;
  if (RATE) {
    for (int64_t f = flushed; f < limit; f += 64) rate_flush(*P, S, *R, f, limit);
    if (limit > flushed) flushed = limit;
    return;
  }
  for (int64_t f = flushed; f < limit; f += 64) {
    const int64_t b = f + lane;
    if (b < limit) {
      const int i = (int)(b & S.mask);
      const double v = S.rv[i];
      if (S.nt) __builtin_nontemporal_store(v, &S.rowv[b]);
      else if (!S.nostore || v == 1234.5678) S.rowv[b] = v;  // ablation
      S.rv[i] = absent_value();
    }
  }
  if (limit > flushed) flushed = limit;
}

// Fast lane fold for lanes whose K points fall into at most three adjacent
// buckets (the common case when buckets hold more than K/2 points; a 1 m
// bucket of 10 s points puts a lane's 8 points in 2 or 3 buckets).  Points
// are sorted by time, so only the first and last point need a bucket index:
// the lane spans buckets k0..k1 (k1 <= k0 + 2), every point before the start
// of bucket k0+1 belongs to k0 (the head run), every point from the start of
// k1 on to k1 (the tail run) and the rest to k0+1, a bucket wholly inside
// the lane that closes here.  All runs accumulate branch free with masked
// pushes, in point order.  Returns false (nothing changed) when the lane
// spans four or more buckets.
// nv < K: only the first nv points are in range (the step reaches past the
// end of the series / window); nv == 0 leaves the lane empty (nseg = 0).
template <class M, int K, bool FLOATONLY, class TT = int64_t>
DEV bool fold_fast(const Params& P, const BatchDev& B, int sf, int64_t i0,
                   const TT* t, const int64_t* v, RowSink& S, int& err,
                   int& nseg, int& cur_key, int& head_key, M& cur, M& head,
                   int nv = K) {
  if (nv <= 0) {
    nseg = 0;
    return true;
  }
  TT tl = t[K - 1];
  if (nv < K) {
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (j == nv - 1) tl = t[j];
  }
  const int k0 = tbucket_narrow(P, t[0]), k1 = tbucket_narrow(P, tl);
  if (k1 - k0 > 2) return false;
  // starts of the tail bucket k1 and of the middle bucket k0+1 (the lowest
  // time sends every point to the tail run)
  const TT b_tail = (k1 == k0) ? tmin<TT>() : tstart_fixed(P, k1, TT{});
  const TT b_mid =
      (k1 == k0 + 2) ? tstart_fixed(P, (int64_t)k0 + 1, TT{}) : b_tail;
  M h = M::init(), m = M::init(), c = M::init();
  bool any_mid = false;
  if (__ballot(k1 == k0 + 2) == 0) {
    // no lane of the wave spans three buckets (buckets of more than K
    // points): two runs, head and tail
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const double x =
          FLOATONLY ? bits_to_double(v[j]) : point_value(B, i0 + j, v[j], sf);
      const bool vj = j < nv;
      const bool inh = vj && t[j] < b_tail;
      h.push_if(inh, x);
      c.push_if(vj && !inh, x);
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const double x =
          FLOATONLY ? bits_to_double(v[j]) : point_value(B, i0 + j, v[j], sf);
      const bool vj = j < nv;
      const bool inh = vj && t[j] < b_mid;
      const bool inc = vj && t[j] >= b_tail;
      const bool inm = vj && !inh && !inc;
      h.push_if(inh, x);
      m.push_if(inm, x);
      c.push_if(inc, x);
      any_mid |= inm;
    }
  }
  head_key = k0;
  cur_key = k1;
  cur = c;
  if (k0 == k1) {
    nseg = 1;
  } else {
    nseg = any_mid ? 3 : 2;
    head = h;
    if (any_mid) S.put(k0 + 1, m.finish(&err));
  }
  return true;
}

// Folds the K points of one lane in order: the first run (which may continue
// from the previous lane) goes to `head`, the last run (which may continue
// into the next lane) stays in `cur`, runs in between close here.
template <class M, int K, bool FLOATONLY, bool CHECKED, class TT = int64_t>
DEV void fold_lane(const Params& P, const BatchDev& B, int sf, int64_t i0,
                   int64_t lo, int64_t hi, const TT* t, const int64_t* v,
                   RowSink& S, int& err, int& nseg,
                   int& cur_key, int& head_key, M& cur, M& head) {
  TT bnd = tmin<TT>();  // first timestamp past cur_key's bucket
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int64_t i = i0 + j;
    if (CHECKED && (i < lo || i >= hi)) continue;
    int k = cur_key;
    if (nseg == 0 || t[j] >= bnd) {
      k = (int)tbucket(P, t[j]);
      bnd = tbound(P, (int64_t)k + 1, TT{});
    }
    const double x = FLOATONLY ? bits_to_double(v[j]) : point_value(B, i, v[j], sf);
    if (nseg == 0) {
      cur_key = k;
      cur = M::from(x);
      nseg = 1;
    } else if (k == cur_key) {
      cur.push(x);
    } else {
      if (nseg == 1) {
        head_key = cur_key;
        head = cur;
      } else {  // a bucket wholly inside this lane
        S.put(cur_key, cur.finish(&err));
      }
      cur_key = k;
      cur = M::from(x);
      ++nseg;
    }
  }
}

// Segmented inclusive scan step over DPP: lanes combine the state DPP brings
// from an earlier lane when it belongs to the same bucket (keys are
// non-decreasing over the lanes, so equal keys mean one contiguous run).
template <int CTRL, int RM, class M>
DEV void seg_step_dpp(int key, M& st) {
  const int k2 = dpp32<CTRL, RM>(INT32_MIN, key);
  M o = st;
  o.template dpp<CTRL, RM>();
  if (k2 == key) st = M::combine(o, st);
}
template <class M>
DEV void seg_scan_dpp(int key, M& st) {
  seg_step_dpp<0x111, 0xF>(key, st);  // row_shr:1
  seg_step_dpp<0x112, 0xF>(key, st);  // row_shr:2
  seg_step_dpp<0x114, 0xF>(key, st);  // row_shr:4
  seg_step_dpp<0x118, 0xF>(key, st);  // row_shr:8
  seg_step_dpp<0x142, 0xA>(key, st);  // row_bcast:15 -> rows 1, 3
  seg_step_dpp<0x143, 0xC>(key, st);  // row_bcast:31 -> rows 2, 3
}
// ---- kOrdered monoids (dev): a bucket's points in the reference's order.
// Downsampler.ValuesInInterval feeds one bucket's values to runDouble in
// time order (Downsampler.java:461-479) and StdDev folds them in one
// sequential Welford pass (Aggregators.java:547-568).  The lane-local fold
// already leaves every run that STARTS inside a lane exact: buckets closed
// inside a lane, and each lane's tail run.  What the tree would merge is
// replayed instead: a lane whose points all continue its predecessor's
// bucket re-pushes them onto the predecessor's state (wave_shr:1), one round
// per lane of the longest such chain; then every head run is pushed onto its
// predecessor's final state.  Lane 0's predecessor is the previous step's
// open bucket (the carry).  Cost: (longest chain + 1) x K pushes per step
// (a 5 m bucket of 10 s points spans <= 3 whole lanes).
template <class M, int K>
DEV M push_run(M st, const BatchDev& B, int sf, int64_t i0, const int64_t* v,
               uint32_t mask) {
#pragma unroll
  for (int j = 0; j < K; ++j)
    if ((mask >> j) & 1u) st.push(point_value(B, i0 + j, v[j], sf));
  return st;
}
template <class M>
DEV M shr1_state(M st, const M& lane0) {
  st.template dpp<0x138, 0xF>();  // wave_shr:1
  return LANE == 0 ? lane0 : st;
}
template <class M, int K, class TT>
DEV void ordered_step(const Params& P, const BatchDev& B, int sf, int64_t lo,
                      int64_t hi, int64_t i0, const TT* t, const int64_t* v,
                      RowSink& S, int& err, int nseg, int key, int head_key,
                      const M& cur, M head, int& carry_key, M& carry) {
  const int lane = LANE;
  // the lane's points in [lo, hi), and those of its head run
  uint32_t vm = 0, hm = 0;
  if (nseg >= 1) {
    const TT hb = tbound(P, (int64_t)head_key + 1, TT{});
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t i = i0 + j;
      const bool ok = i >= lo && i < hi;
      vm |= (ok ? 1u : 0u) << j;
      hm |= (ok && t[j] < hb ? 1u : 0u) << j;
    }
  }
  const bool carry_in = carry_key >= 0 && carry_key < P.nb;
  const M in0 = carry_in ? carry : M::init();
  // the predecessor's tail key (lane 0: the carry's)
  const int pkey = dpp32<0x138, 0xF>(carry_in ? carry_key : INT32_MIN, key);
  // lanes wholly inside their predecessor's bucket (nseg == 0: lanes past
  // hi that keep_open points at the open bucket, pushing nothing)
  const bool pass = nseg <= 1 && pkey == key;
  M out = cur;
  int rounds = 0;
  for (uint64_t x = __ballot(pass); x; x &= x << 1) ++rounds;
  for (int r = 0; r < rounds; ++r) {
    const M in = shr1_state(out, in0);
    if (pass) out = push_run<M, K>(in, B, sf, i0, v, vm);
  }
  const M fin = shr1_state(out, in0);
  if (nseg >= 2) {  // head run closes inside this lane
    if (pkey == head_key) head = push_run<M, K>(fin, B, sf, i0, v, hm);
    S.put(head_key, head.finish(&err));
  }
  if (lane == 0 && carry_in && !(nseg >= 1 && carry_key == head_key))
    S.put(carry_key, carry.finish(&err));
  const int next_head = dpp32<0x130, 0xF>(INT32_MIN, head_key);  // wave_shl:1
  if (nseg >= 1 && lane < 63 && next_head != key) S.put(key, out.finish(&err));
  Packed p = out.pack();
  carry_key = __builtin_amdgcn_readlane(key, 63);
  p.x = readlane_d(p.x, 63);
  p.y = readlane_d(p.y, 63);
  p.z = readlane_d(p.z, 63);
  p.w = readlane_l(p.w, 63);
  carry = M::unpack(p);
}

// One step of the bucket reduction over the K consecutive points t[], v[]
// of every lane (points i0 .. i0+K-1 of the series, step base `base`):
// lane-local fold, the previous step's open bucket, the segmented wave scan
// over the lanes' tail runs, the row writes and the new carry.
// FO = 1: the caller guarantees doubles only (the cells fold decodes every
// value to its double bits): the per-point type tests and their registers
// are not compiled in
template <class M, int K, int DPP, class TT = int64_t, int FO = 0>
DEV void reduce_step(const Params& P, const BatchDev& B, int sf, int64_t lo,
                     int64_t hi, int64_t base, int64_t i0, const TT* t,
                     const int64_t* v, RowSink& S, int& err,
                     int& carry_key, M& carry, bool keep_open = false) {
  constexpr int PTS = 64 * K;
  const int lane = LANE;
  // ---- lane-local sequential fold (range checks only on the first and
  // last step; no per-point type test for all-double series)
  int nseg = 0, cur_key = 0, head_key = 0;
  M cur = M::init(), head = M::init();
  const bool full = base >= lo && base + PTS <= hi;
  // a step that only runs past hi (the last one): the fast fold still
  // applies, each lane to its in-range prefix
  const bool tail = !full && base >= lo && P.narrow;
  if (full || tail) {
    const bool fonly = FO || (!B.is_float && sf);
    bool done = false;
    const int64_t nr = hi - i0;
    const int nv = full ? K : (int)(nr < 0 ? 0 : (nr > K ? K : nr));
    if (P.narrow) {
      done = fonly
                 ? fold_fast<M, K, true, TT>(P, B, sf, i0, t, v, S, err, nseg,
                                             cur_key, head_key, cur, head, nv)
                 : fold_fast<M, K, false, TT>(P, B, sf, i0, t, v, S, err,
                                              nseg, cur_key, head_key, cur,
                                              head, nv);
    }
    if (!done) {
      if (full && fonly)
        fold_lane<M, K, true, false, TT>(P, B, sf, i0, lo, hi, t, v, S,
                                         err, nseg, cur_key, head_key, cur,
                                         head);
      else if (full)
        fold_lane<M, K, false, false, TT>(P, B, sf, i0, lo, hi, t, v, S,
                                          err, nseg, cur_key, head_key, cur,
                                          head);
      else
        fold_lane<M, K, FO != 0, true, TT>(P, B, sf, i0, lo, hi, t, v, S,
                                           err, nseg, cur_key, head_key, cur,
                                           head);
    }
  } else {
    fold_lane<M, K, FO != 0, true, TT>(P, B, sf, i0, lo, hi, t, v, S,
                                       err, nseg, cur_key, head_key, cur, head);
  }
#if defined(OTSDB_REDUCE_ABL) && OTSDB_REDUCE_ABL == 1  // timing: lane fold only
  {
    const double x = cur.finish(&err) + head.finish(&err);
    if (x == 1234.5678) S.put(cur_key, x);
    carry_key = __builtin_amdgcn_readlane(cur_key, 63);
    return;
  }
#endif
  if (nseg == 0) {  // lane wholly before lo (first step) or past hi
    cur_key = (i0 < lo) ? -1 : INT32_MAX;
    head_key = cur_key;
  } else if (nseg == 1) {
    head_key = cur_key;
  }
  if (keep_open) {
    // more points may follow in a later call (the next storage row of the
    // series): lanes past hi continue the last lane with points, so its
    // bucket stays open and becomes the carry instead of being written.
    // Lanes holding points are contiguous; the ones after the last of them
    // are exactly the lanes past hi.
    const uint64_t real = __ballot(nseg > 0);
    if (real) {
      const int L = 63 - __builtin_clzll(real);
      const int k = __builtin_amdgcn_readlane(cur_key, L);
      if (lane > L) {
        cur_key = k;
        head_key = k;
      }
    }
  }
  if constexpr (M::kOrdered) {
    ordered_step<M, K, TT>(P, B, sf, lo, hi, i0, t, v, S, err, nseg, cur_key,
                           head_key, cur, head, carry_key, carry);
    return;
  }
  // ---- previous step's open bucket
  if (lane == 0) {
    if (nseg >= 1 && carry_key == head_key) {
      if (nseg == 1) cur = M::combine(carry, cur);
      else head = M::combine(carry, head);
    } else if (carry_key >= 0 && carry_key < P.nb) {
      S.put(carry_key, carry.finish(&err));
    }
  }
  // ---- segmented inclusive scan over the lanes' tail runs
  int key = cur_key;
  M st = cur;
  int pkey, next_head;
  M pst;
  if (DPP) {
    // A tail run spans its own lane and the following lanes that hold no
    // bucket boundary (nseg <= 1), so the scan needs only the row steps
    // reaching the longest such stretch (the row broadcasts carry it across
    // rows): 1 m buckets of 10 s points (a boundary in every lane) skip it
    int L = 0;
    for (uint64_t y = __ballot(nseg <= 1); y; y &= y << 1) ++L;
    if (L > 0) {
      seg_step_dpp<0x111, 0xF>(key, st);               // row_shr:1
      if (L > 1) seg_step_dpp<0x112, 0xF>(key, st);    // row_shr:2
      if (L > 3) seg_step_dpp<0x114, 0xF>(key, st);    // row_shr:4
      if (L > 7) seg_step_dpp<0x118, 0xF>(key, st);    // row_shr:8
      seg_step_dpp<0x142, 0xA>(key, st);  // row_bcast:15 -> rows 1, 3
      seg_step_dpp<0x143, 0xC>(key, st);  // row_bcast:31 -> rows 2, 3
    }
    pkey = dpp32<0x138, 0xF>(INT32_MIN, key);  // wave_shr:1
    pst = st;
    pst.template dpp<0x138, 0xF>();
    next_head = dpp32<0x130, 0xF>(INT32_MIN, head_key);  // wave_shl:1
  } else {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int k2 = __shfl_up(key, d);
      M o = st;
      o.shfl_up(d);
      if (lane >= d && k2 == key) st = M::combine(o, st);
    }
    pkey = __shfl_up(key, 1);
    pst = st;
    pst.shfl_up(1);
    next_head = __shfl_down(head_key, 1);
  }
  const bool put_head = nseg >= 2;  // head run closes inside this lane
  const bool put_tail = nseg >= 1 && lane < 63 && next_head != key;
  M hfull = head;
  if (put_head && lane > 0 && pkey == head_key) hfull = M::combine(pst, head);
  if constexpr (M::kCostlyFinish) {
    // (a division / square root each: one finish a lane when no lane
    // closes both its head and its tail run, as with buckets of > K points)
    if (__ballot(put_head && put_tail) == 0) {
      if (put_head || put_tail) {
        const M& r = put_head ? hfull : st;
        S.put(put_head ? head_key : key, r.finish(&err));
      }
    } else {
      if (put_head) S.put(head_key, hfull.finish(&err));
      if (put_tail) S.put(key, st.finish(&err));
    }
  } else {
    if (put_head) S.put(head_key, hfull.finish(&err));
    if (put_tail) S.put(key, st.finish(&err));
  }
  Packed p = st.pack();
  if (DPP) {
    carry_key = __builtin_amdgcn_readlane(key, 63);
    p.x = readlane_d(p.x, 63);
    p.y = readlane_d(p.y, 63);
    p.z = readlane_d(p.z, 63);
    p.w = readlane_l(p.w, 63);
  } else {
    carry_key = __shfl(key, 63);
    p.x = __shfl(p.x, 63);
    p.y = __shfl(p.y, 63);
    p.z = __shfl(p.z, 63);
    p.w = __shfl(p.w, 63);
  }
  carry = M::unpack(p);
}

// Ring bookkeeping around one step (WIN > 0).  Before the step: every
// bucket the step can write lies in [k_open, k_hi]; if that range does not
// fit the ring behind the flushed mark, drain what is final and, failing
// that (a gap of more than WIN buckets inside one step), write this step
// straight to HBM.  After it: drain the final buckets in runs of 64.
DEV int64_t step_last_key(const Params& P, const BatchDev& B, int64_t base,
                          int64_t hi, int64_t pts) {
  const int64_t e = (base + pts < hi ? base + pts : hi) - 1;
  return bucket_of(P, B.ts[e]);
}

// returns true (RATE: nothing written) when the step spans more buckets
// than the ring holds
template <int WIN, int K, int RATE = 0>
DEV bool ring_before(const Params& P, const BatchDev& B, RowSink& S,
                     int64_t& flushed, int64_t lo, int64_t hi, int64_t base,
                     const int64_t* t, int carry_key, RateState* R = nullptr) {
  if (WIN == 0) return false;
  constexpr int64_t pts = 64 * K;
  // last key of the step: from lane 63's last point when the step is full
  // (already in registers; a scalar reload would wait on HBM every step)
  const int64_t k_hi =
      (base + pts <= hi)
          ? bucket_of(P, readlane_l(t[K - 1], 63))
          : step_last_key(P, B, base, hi, pts);
  if (k_hi >= flushed + WIN) {
    const int64_t k_open = (carry_key >= 0 && carry_key < P.nb)
                               ? carry_key
                               : bucket_of(P, B.ts[base > lo ? base : lo]);
    sink_flush<RATE>(S, flushed, k_open, &P, R);
    if (k_hi >= flushed + WIN) {
      if (RATE) return true;
      // a gap of more than WIN buckets inside this step: mark the span
      // absent, then let the step store straight to HBM behind it
      const int lane = LANE;
      for (int64_t f = flushed; f <= k_hi; f += 64)
        if (f + lane <= k_hi) S.rowv[f + lane] = absent_value();
      wait_vmcnt(0);
      S.direct = 1;
    }
  }
  return false;
}

template <int WIN, int FL, int RATE = 0>
DEV void ring_after(const Params& P, const BatchDev& B, RowSink& S,
                    int64_t& flushed, int64_t hi, int64_t base, int64_t pts,
                    int carry_key, RateState* R = nullptr) {
  if (WIN == 0) return;
  // buckets below the open one (or the whole step, past the end) are final
  const int64_t limit = (carry_key >= 0 && carry_key < P.nb)
                            ? carry_key
                            : step_last_key(P, B, base, hi, pts) + 1;
  if (S.direct) {
    if (limit > flushed) flushed = limit;
    S.direct = 0;
    return;
  }
  const int64_t full = flushed + ((limit - flushed) / FL) * FL;
  if (full > flushed) sink_flush<RATE>(S, flushed, full, &P, R);
}

// The rate row's buckets that depend on the whole series (transform_rate
// pass 2): fewer than two rates (or none kept) -> absent everywhere; before
// the first kept rate -> the junk rate, held; past the last kept rate ->
// absent, or the latest rate held toward a point past the window
// (AggregationIterator.java:448-459, :744-753).  kl: the last flushed bucket.
// The rates past the window (rates_beyond): is the rate at the bucket past
// it kept, its value, and whether any kept rate lies past the window.
struct PastRates {
  bool of_kept, any;
  int n;          // kept rates past the window, capped at 2
  double first;   // the first of them
};
DEV PastRates past_rates(const Params& P, const SeriesMeta& SM, int64_t s,
                         int64_t carry_pts, double carry_pv) {
  PastRates q{false, false, 0, 0.0};
  const int h = SM.of_has[s];
  if (!(h & 1)) return q;
  const double r = rate_between(P, carry_pts, carry_pv, SM.of_ts[s],
                                SM.of_val[s], &q.of_kept);
  const int kb = (h >> 1) & 3;
  q.n = (q.of_kept ? 1 : 0) + kb;
  if (q.n > 2) q.n = 2;
  q.first = q.of_kept ? r : SM.of_rate[s];
  q.any = q.n > 0;
  return q;
}

DEV void rate_finish(const Params& P, const SeriesMeta& SM, int64_t s,
                     RowSink& S, const RateState& R, int64_t kl) {
  const int lane = LANE;
  const int64_t nb = P.nb;
  const PastRates q = past_rates(P, SM, s, R.carry_pts, R.carry_pv);
  const int total = R.kept_count + q.n;
  if (total < 2) {
    for (int64_t b = lane; b < nb; b += 64) S.rows[b] = ST_ABSENT;
    return;
  }
  if (R.kept_count == 0) {
    // every kept rate lies past the window: the first one (the junk rate)
    // is held over the whole grid
    for (int64_t b = lane; b < nb; b += 64) {
      S.rowv[b] = q.first;
      S.rows[b] = ST_INTERP;
    }
    return;
  }
  for (int64_t b = lane; b < R.r0_idx; b += 64) {
    S.rowv[b] = R.r0_val;
    S.rows[b] = ST_INTERP;
  }
  if (!q.any) {
    for (int64_t b = R.last_kept + 1 + lane; b < nb; b += 64)
      S.rows[b] = ST_ABSENT;
  } else {
    for (int64_t b = kl + 1 + lane; b < nb; b += 64) {
      S.rowv[b] = R.carry_kv;
      S.rows[b] = ST_INTERP;
    }
  }
}

// RATE: RateSpan fused into the ring flush (rate_flush / rate_finish): the
// row leaves as rates + states, no k_transform pass; a step spanning more
// buckets than the ring hands the series back (P.redo).
// One series (wavefront) of k_bucketize_k: S says where its closed buckets
// go (row, LDS ring, or k_bucketize_group's group row).
template <class M, int K, int PF, int NT, int ABL, int DPP, int WIN, int FL,
          int RATE>
DEV void bucketize_series(const Params& P, const BatchDev& B,
                          const SeriesMeta& SM, RowSink& S, double* ring,
                          int64_t s) {
  static_assert(K % 2 == 0, "K must be even (16-byte loads)");
  static_assert((WIN & (WIN - 1)) == 0, "WIN: power of two");
  static_assert(!RATE || WIN > 0, "RATE needs the ring");
  const int lane = LANE;
  const int64_t lo = SM.keep[s] ? SM.lo[s] : 0;
  const int64_t hi = SM.keep[s] ? SM.hi[s] : 0;
  RateState RS{P.rate_origin_ts, P.rate_origin_val, -1, 0.0, -1, -1, 0.0, 0, 0};
  if (lo >= hi) {
    if (RATE) {  // absent, or its rates past the window held (rate_finish)
      rate_finish(P, SM, s, S, RS, -1);
      if (lane == 0) P.redo[s] = 0;
    }
    return;
  }
  const int sf = B.series_float ? (int)B.series_float[s] : 1;
  int64_t flushed = 0;
  if (WIN) {
    for (int i = lane; i < WIN; i += 64) ring[i] = absent_value();
    flushed = bucket_of(P, B.ts[lo]);
  }
  int err = 0;

  int carry_key = INT32_MIN;
  M carry = M::init();
  constexpr int PTS = 64 * K;
  // K consecutive points of this lane: K/2 16-byte loads per column
  auto load_step = [&](int64_t i0, int64_t* t, int64_t* v) {
    if (i0 + K <= hi) {
#pragma unroll
      for (int j = 0; j < K; j += 2) {
        const ll2_t* pt = reinterpret_cast<const ll2_t*>(B.ts + i0 + j);
        const ll2_t* pv = reinterpret_cast<const ll2_t*>(B.val + i0 + j);
        ll2_t tt, vv;
        if (NT == 1) {
          tt = __builtin_nontemporal_load(pt);
          vv = __builtin_nontemporal_load(pv);
        } else {
          tt = *pt;
          vv = *pv;
        }
        t[j] = tt.x; t[j + 1] = tt.y;
        v[j] = vv.x; v[j + 1] = vv.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        t[j] = (i0 + j < hi) ? B.ts[i0 + j] : 0;
        v[j] = (i0 + j < hi) ? B.val[i0 + j] : 0;
      }
    }
  };
  int64_t tn[K], vn[K];
  const int64_t base0 = lo & ~(int64_t)1;
  if (PF) load_step(base0 + (int64_t)K * lane, tn, vn);
  L2Touch pt_, pv_;
  for (int64_t base = base0; base < hi; base += PTS) {
    const int64_t i0 = base + (int64_t)K * lane;
    int64_t t[K], v[K];
    if (PF) {
#pragma unroll
      for (int j = 0; j < K; ++j) { t[j] = tn[j]; v[j] = vn[j]; }
      if (base + PTS < hi) load_step(i0 + PTS, tn, vn);
    } else {
      load_step(i0, t, v);
    }
    if (OTSDB_PF_BUCK) {
      pt_.retire();
      pv_.retire();
      if (base + (OTSDB_PF_BUCK + 1) * PTS <= hi) {
        pt_.touch(B.ts + i0 + OTSDB_PF_BUCK * PTS);
        pv_.touch(B.val + i0 + OTSDB_PF_BUCK * PTS);
      }
    }
    if (ABL == 1) {  // tuning ablation: stream only
      int64_t x = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) x ^= t[j] + v[j];
      if (x == 42) S.rows[0] = 1;
      continue;
    }
    // drain the buckets the previous step finished only now, after this
    // step's loads are issued: vmcnt retires loads and stores in issue
    // order, so stores issued before a load would hold up its data
    if (base != base0)
      ring_after<WIN, FL, RATE>(P, B, S, flushed, hi, base - PTS, PTS,
                                carry_key, &RS);
    if (ring_before<WIN, K, RATE>(P, B, S, flushed, lo, hi, base, t,
                                  carry_key, &RS)) {
      RS.bad = 1;  // RATE only: hand the series to the fallback kernels
      break;
    }
    reduce_step<M, K, DPP>(P, B, sf, lo, hi, base, i0, t, v, S, err,
                           carry_key, carry);
  }
  if (RATE && RS.bad) {
    if (lane == 0) P.redo[s] = 1;
    return;
  }
  if (carry_key >= 0 && carry_key < P.nb && lane == 0)
    S.put(carry_key, carry.finish(&err));
  // every bucket from the first point's to the last point's is written; a
  // last step that went direct already stored its buckets behind `flushed`
  // (the ring only holds absent slots there)
  const int64_t k_last = bucket_of(P, B.ts[hi - 1]);
  if (WIN && !S.direct) sink_flush<RATE>(S, flushed, k_last + 1, &P, &RS);
  if (RATE) {
    if (RS.bad) {
      if (lane == 0) P.redo[s] = 1;
      return;
    }
    rate_finish(P, SM, s, S, RS, k_last);
    if (lane == 0) P.redo[s] = 0;
  }
}

template <class M, int K, int PF = 0, int NT = 0, int WAVES = 1, int ABL = 0,
          int DPP = 0, int WIN = 0, int FL = 64, int RATE = 0>
__global__ __launch_bounds__(256, WAVES) void k_bucketize_k(Params P,
                                                            BatchDev B,
                                                            SeriesMeta SM,
                                                            Rows R) {
  constexpr int WS = WIN > 0 ? WIN : 1;
  __shared__ double ring_v[4][WS];
  const int w = threadIdx.x >> 6;
  const int64_t s = (int64_t)blockIdx.x * 4 + w;
  if (s >= B.S) return;
  if (P.only_redo && !P.redo[s]) return;
  RowSink S{R.val + s * P.nb, R.state + s * P.nb, ring_v[w], WS - 1,
            WIN == 0, WIN == 0, ABL == 2, NT == 2};
  bucketize_series<M, K, PF, NT, ABL, DPP, WIN, FL, RATE>(P, B, SM, S,
                                                          ring_v[w], s);
}

// ------------------------------------------------------------------------
// interpolation of a series between two of its points, exactly as
// AggregationIterator.nextDoubleValue (AggregationIterator.java:772-793)
// ------------------------------------------------------------------------
DEV double interp_value(int method, int64_t x, int64_t x0, double y0,
                        int64_t x1, double y1) {
  switch (method) {
    case 0: return y0 + (double)(x - x0) * (y1 - y0) / (double)(x1 - x0);
    case 1: return 0.0;
    case 2: return kDoubleMax;
    case 3: return -kDoubleMax;
    default: return y0;
  }
}

// ------------------------------------------------------------------------
// k_transform: per-series bucket row -> what the series contributes at each
// union timestamp of AggregationIterator (one wavefront per series):
//  * FillingDownsampler (FillingDownsampler.java:172-298): every grid bucket
//    is a point; missing ones take the fill value;
//  * RateSpan (RateSpan.java:121-180) over the bucket points, incl. the junk
//    first rate vs (0, 0) and the hold-previous-rate rule of
//    AggregationIterator (:448-459, :744-753);
//  * otherwise interpolation between the series' own points (:754-793),
//    contributing iff first <= x <= last (or a point exists past the window).
// ------------------------------------------------------------------------
template <int NCH>
__global__ __launch_bounds__(256) void k_transform(Params P, BatchDev B,
                                                   SeriesMeta SM, Rows R,
                                                   int* err_word);
template <int NCH>
DEV void transform_rate(const Params& P, const SeriesMeta& SM, int64_t s,
                        double* rowv, uint8_t* rows, bool sent, bool fill,
                        int64_t kf, int64_t kl, int* err_word);

template <int NCH>
__global__ __launch_bounds__(256) void k_transform(Params P, BatchDev B,
                                                   SeriesMeta SM, Rows R,
                                                   int* err_word) {
  const int lane = LANE;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= B.S) return;
  if (P.only_redo && !P.redo[s]) return;
  const int64_t nb = P.nb;
  double* rowv = R.val + s * nb;
  uint8_t* rows = R.state + s * nb;
  const bool sent = P.sentinel != 0;
  if (!SM.keep[s]) {
    if (sent)  // no memset before a sentinel-row query: clear the states
      for (int64_t b = lane; b < nb; b += 64) rows[b] = ST_ABSENT;
    return;
  }
  const bool fill = P.fill != 0 && !P.run_all;
  // sentinel rows: buckets [kf, kl] (first / last point's bucket) hold a
  // value or kAbsentBits, the others are absent
  const int64_t kf = sent ? SM.kf[s] : 0, kl = sent ? SM.kl[s] : -1;
  auto real_at = [&](int64_t b, double v) {
    return sent ? (b >= kf && b <= kl && __double_as_longlong(v) != kAbsentBits)
                : rows[b] == ST_REAL;
  };

  if (!P.rate) {
    if (fill) {
      for (int64_t c0 = 0; c0 < nb; c0 += 64) {
        const int64_t b = c0 + lane;
        if (b < nb) {
          if (!real_at(b, rowv[b])) {
            rowv[b] = P.fill_value;
            rows[b] = ST_REAL;
          } else if (sent) {
            rows[b] = ST_REAL;
          }
        }
      }
      return;
    }
    // NONE fill: interpolate inside gaps, and toward the point past the
    // window when there is one.
    const bool of = SM.of_has[s] != 0;
    int64_t carry_idx = -1;
    double carry_val = 0.0;
    // row values two chunks ahead: the chunk loop is a dependent chain, an
    // unprefetched load per chunk costs a full HBM latency
    double va = lane < nb ? rowv[lane] : 0.0;
    double vn = lane + 64 < nb ? rowv[lane + 64] : 0.0;
    for (int64_t c0 = 0; c0 < nb; c0 += 64) {
      const int64_t b = c0 + lane;
      const double vb = va;
      va = vn;
      vn = b + 128 < nb ? rowv[b + 128] : 0.0;
      const bool p = b < nb && real_at(b, vb);
      const double v = p ? vb : 0.0;
      if (sent && b < nb)  // every state of the row, written once
        rows[b] = p ? ST_REAL
                    : (((b > kf && b < kl) || (of && kf <= kl && b > kl))
                           ? ST_INTERP
                           : ST_ABSENT);
      // the real buckets of the chunk as a wave-uniform mask: each lane's
      // previous real bucket is the highest set bit below it (else the
      // carry), no cross-lane scan
      const uint64_t rm = __ballot(p);
      const uint64_t below = rm & ((1ULL << lane) - 1);
      const int pl = below ? 63 - __builtin_clzll(below) : -1;
      const int64_t prev = pl >= 0 ? c0 + pl : carry_idx;
      uint64_t gaps = __ballot(p && prev >= 0 && prev < b - 1);
      if (gaps) {
        const double yp = __shfl(v, pl >= 0 ? pl : 0);
        const double yprev = pl >= 0 ? yp : carry_val;
        while (gaps) {
          const int g = __builtin_ctzll(gaps);
          gaps &= gaps - 1;
          const int64_t k0 = __shfl(prev, g), k1 = c0 + g;
          const double y0 = __shfl(yprev, g), y1 = __shfl(v, g);
          const int64_t x0 = bucket_ts(P, k0), x1 = bucket_ts(P, k1);
          for (int64_t j = k0 + 1 + lane; j < k1; j += 64) {
            rowv[j] = interp_value(P.interp, bucket_ts(P, j), x0, y0, x1, y1);
            rows[j] = ST_INTERP;
          }
        }
      }
      if (rm) {
        const int l = 63 - __builtin_clzll(rm);
        carry_val = readlane_d(v, l);
        carry_idx = c0 + l;
      }
    }
    if (SM.of_has[s] && carry_idx >= 0) {
      const int64_t x0 = bucket_ts(P, carry_idx), x1 = SM.of_ts[s];
      const double y1 = SM.of_val[s];
      for (int64_t j = carry_idx + 1 + lane; j < nb; j += 64) {
        rowv[j] = interp_value(P.interp, bucket_ts(P, j), x0, carry_val, x1, y1);
        rows[j] = ST_INTERP;
      }
    }
    return;
  }

  transform_rate<NCH>(P, SM, s, rowv, rows, sent, fill, kf, kl, err_word);
}

// RateSpan over the bucket points of one series and the contribution rule
// of rate mode (AggregationIterator.java:448-459, :744-753).  Pass 1 computes
// the rate points (the first one against (0, 0) or the FillingDownsampler
// bucket before the grid), pass 2 writes each bucket's contribution: the
// series' latest rate at or before it, from its first real rate on the junk
// one.  NCH > 0: the row (<= 64*NCH buckets) stays in registers between the
// passes and is written once; NCH == 0: pass 1 stores the rates and a
// transient state in the row and pass 2 re-reads them.
template <int NCH>
DEV void transform_rate(const Params& P, const SeriesMeta& SM, int64_t s,
                        double* rowv, uint8_t* rows, bool sent, bool fill,
                        int64_t kf, int64_t kl, int* err_word) {
  const int lane = LANE;
  const int64_t nb = P.nb;
  auto real_at = [&](int64_t b, double v) {
    return sent ? (b >= kf && b <= kl && __double_as_longlong(v) != kAbsentBits)
                : rows[b] == ST_REAL;
  };
  constexpr int NR = NCH > 0 ? NCH : 1;
  double rreg[NR];
  uint32_t kmask = 0;  // bit c: this lane's bucket of chunk c is a kept rate
  const double cmax_d = (double)P.counter_max;
  int64_t carry_pts = P.rate_origin_ts;
  double carry_pv = P.rate_origin_val;
  int64_t r0_idx = -1, last_kept = -1;
  double r0_val = 0.0;
  int kept_count = 0;
  int bad_ts = 0;
  auto pass1 = [&](int64_t c0, int c, double vb) {
    const int64_t b = c0 + lane;
    const bool inb = b < nb;
    const uint8_t st = (inb && real_at(b, vb)) ? ST_REAL : 0;
    const bool pt = inb && (fill || st == ST_REAL);
    const double pv = (st == ST_REAL) ? vb : P.fill_value;
    const int64_t t = bucket_ts(P, b);
    // previous source point of each lane: highest set bit below it in the
    // chunk's point mask, else the carry
    const uint64_t pm = __ballot(pt);
    const uint64_t below = pm & ((1ULL << lane) - 1);
    const int pl = below ? 63 - __builtin_clzll(below) : -1;
    const double vp = __shfl(pv, pl >= 0 ? pl : 0);
    int64_t tprev;
    double vprev;
    if (pl >= 0) {
      tprev = bucket_ts(P, c0 + pl);
      vprev = vp;
    } else {
      tprev = carry_pts;
      vprev = carry_pv;
    }
    bool kept = false;
    double rate = 0.0;
    if (pt) {
      if (t <= tprev) bad_ts = 1;
      const double dt = (double)(t - tprev) / 1000.0;
      double diff = pv - vprev;
      if (P.counter && diff < 0) {
        if (!P.drop_resets) {
          kept = true;
          diff = cmax_d - vprev + pv;
          const double r = diff / dt;
          rate = (P.reset_value > 0 && r > (double)P.reset_value) ? 0.0 : r;
        }
      } else {
        kept = true;
        rate = diff / dt;
      }
    }
    if (NCH > 0) {
      rreg[c] = rate;
      if (pt && kept) kmask |= 1u << c;
    } else if (inb) {
      if (pt && kept) {
        rowv[b] = rate;
        rows[b] = ST_KEPT;
      } else {
        rows[b] = ST_ABSENT;
      }
    }
    const uint64_t km = __ballot(pt && kept);
    if (km) {
      const int f = __builtin_ctzll(km);
      if (r0_idx < 0) {
        r0_idx = c0 + f;
        r0_val = __shfl(rate, f);
      }
      kept_count += __popcll(km);
      if (kept_count > 2) kept_count = 2;
      last_kept = c0 + 63 - __builtin_clzll(km);
    }
    if (pm) {
      const int l = 63 - __builtin_clzll(pm);
      carry_pts = bucket_ts(P, c0 + l);
      carry_pv = readlane_d(pv, l);
    }
  };
  if (NCH > 0) {
    // the whole row first (every load in flight at once), then the chain
#pragma unroll
    for (int c = 0; c < NR; ++c) {
      const int64_t b = (int64_t)c * 64 + lane;
      rreg[c] = b < nb ? rowv[b] : 0.0;
    }
#pragma unroll
    for (int c = 0; c < NR; ++c)
      if ((int64_t)c * 64 < nb) pass1((int64_t)c * 64, c, rreg[c]);
  } else {
    double va = lane < nb ? rowv[lane] : 0.0;
    double vn = lane + 64 < nb ? rowv[lane + 64] : 0.0;
    for (int64_t c0 = 0; c0 < nb; c0 += 64) {
      const double vb = va;
      va = vn;
      vn = c0 + 128 + lane < nb ? rowv[c0 + 128 + lane] : 0.0;
      pass1(c0, 0, vb);
    }
  }
  if (__ballot(bad_ts) && lane == 0) atomicOr(err_word, ERR_RATE_TS);
  // kept rates past the window keep the series contributing to the end (and
  // when every kept rate lies past it, the first one is held everywhere)
  PastRates q{false, false, 0, 0.0};
  if (!fill) q = past_rates(P, SM, s, carry_pts, carry_pv);
  const bool of_kept = q.any;
  const int total = kept_count + q.n;
  if (kept_count == 0) r0_val = q.first;

  int64_t carry_k = -1;
  double carry_kv = 0.0;
  auto pass2 = [&](int64_t c0, int c, uint8_t st_in, double v_in) {
    const int64_t b = c0 + lane;
    const bool inb = b < nb;
    bool k;
    double kv;
    if (NCH > 0) {
      k = inb && ((kmask >> c) & 1u);
      kv = k ? rreg[c] : 0.0;
    } else {
      k = inb && st_in == ST_KEPT;
      kv = k ? v_in : 0.0;
    }
    // latest kept rate at or before each lane: highest set bit up to it
    const uint64_t km = __ballot(k);
    const uint64_t upto = km & ((2ULL << lane) - 1);
    const int il = upto ? 63 - __builtin_clzll(upto) : -1;
    const double lv = __shfl(kv, il >= 0 ? il : 0);
    const double held = il >= 0 ? lv : (carry_k >= 0 ? carry_kv : r0_val);
    if (inb) {
      if (total < 2 || (b > last_kept && !of_kept)) {
        rows[b] = ST_ABSENT;
      } else if (k && b != r0_idx) {
        if (NCH > 0) rowv[b] = kv;
        rows[b] = ST_REAL;
      } else {
        rowv[b] = held;
        rows[b] = ST_INTERP;
      }
    }
    if (km) {
      const int l = 63 - __builtin_clzll(km);
      carry_k = c0 + l;
      carry_kv = readlane_d(kv, l);
    }
  };
  if (NCH > 0) {
#pragma unroll
    for (int c = 0; c < NR; ++c)
      if ((int64_t)c * 64 < nb) pass2((int64_t)c * 64, c, 0, 0.0);
  } else {
    // pass 2 re-reads what pass 1 stored (KEPT flags and rates), two chunks
    // ahead like pass 1
    auto ld = [&](int64_t b, uint8_t& st, double& v) {
      st = b < nb ? rows[b] : (uint8_t)0;
      v = b < nb ? rowv[b] : 0.0;
    };
    uint8_t sa, sn;
    double va, vn;
    ld(lane, sa, va);
    ld(lane + 64, sn, vn);
    for (int64_t c0 = 0; c0 < nb; c0 += 64) {
      const uint8_t sc = sa;
      const double vc = va;
      sa = sn;
      va = vn;
      ld(c0 + 128 + lane, sn, vn);
      pass2(c0, 0, sc, vc);
    }
  }
}

// ------------------------------------------------------------------------
// k_group: cross-series aggregation (AggregationIterator.next + the
// aggregator's runDouble over the contributing spans in span order,
// AggregationIterator.java:514-567, :635-647, :735-797).  One thread per
// (chunk of a group's members, bucket); the members of a chunk are pushed in
// SpanCmp order, so a group of <= CHUNK series reproduces the Java sum
// bit for bit.  Single-chunk groups finish here; others leave partials.
// init (chained partials, otsdb_agg_partials_chained_device): the state of
// the group's members on earlier ranks; a group's first chunk continues it,
// so a dev chain runs on across ranks exactly as StdDev.runDouble's one
// loop (Aggregators.java:547-568).
// ------------------------------------------------------------------------
template <class M>
__global__ __launch_bounds__(256) void k_group(
    int64_t nb, int64_t n_tiles, const int64_t* __restrict__ tile_g,
    const int64_t* __restrict__ tile_m0, const int64_t* __restrict__ tile_m1,
    const uint8_t* __restrict__ tile_single, const int64_t* __restrict__ members,
    Rows R, Packed* __restrict__ partial, uint8_t* __restrict__ tile_emit,
    double* __restrict__ out_val, uint8_t* __restrict__ out_emit,
    int* err_word, int always_partial, const Packed* __restrict__ init = nullptr,
    const uint8_t* __restrict__ init_emit = nullptr) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t t = idx / nb;
  if (t >= n_tiles) return;
  const int64_t b = idx - t * nb;
  const int64_t m0 = tile_m0[t], m1 = tile_m1[t];
  M st = M::init();
  int emit = 0;
  if (init && (t == 0 || tile_g[t - 1] != tile_g[t])) {
    const int64_t o = tile_g[t] * nb + b;
    st = M::unpack(init[o]);
    emit = init_emit[o];
  }
  int64_t m = m0;
  // (the chain is latency-bound on the gathers: 8 members' loads in flight;
  // chunks of dev groups run up to kOrderedChunk members)
  for (; m + 8 <= m1; m += 8) {
    int64_t off[8];
    uint8_t sv[8];
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) off[u] = members[m + u] * nb + b;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      sv[u] = R.state[off[u]];
      v[u] = R.val[off[u]];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (sv[u]) {
        st.push(v[u]);
        emit |= sv[u] == ST_REAL;
      }
    }
  }
  for (; m < m1; ++m) {
    const int64_t off = members[m] * nb + b;
    const uint8_t sv = R.state[off];
    if (sv) {
      st.push(R.val[off]);
      emit |= sv == ST_REAL;
    }
  }
  if (tile_single[t] && !always_partial) {
    const int64_t o = tile_g[t] * nb + b;
    double r = 0.0;
    if (emit) {
      int e = 0;
      r = st.finish(&e);
      if (is_inf(r)) e |= ERR_INFINITY;
      if (e) atomicOr(err_word, e);
    }
    out_val[o] = r;
    out_emit[o] = (uint8_t)emit;
  } else {
    partial[t * nb + b] = st.pack();
    tile_emit[t * nb + b] = (uint8_t)emit;
  }
}

// ordered fold of the chunk partials [t0, t1) of bucket b; loads issued in
// batches of 8 ahead of the dependent combines (the chain is latency-bound)
template <class M>
DEV void fold_chunks(const Packed* __restrict__ partial,
                     const uint8_t* __restrict__ tile_emit, int64_t nb,
                     int64_t b, int64_t t0, int64_t t1, M& st, int& emit) {
  int64_t t = t0;
  for (; t + 8 <= t1; t += 8) {
    Packed q[8];
    uint8_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      q[j] = partial[(t + j) * nb + b];
      e[j] = tile_emit[(t + j) * nb + b];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      st = M::combine(st, M::unpack(q[j]));
      emit |= e[j];
    }
  }
  for (; t < t1; ++t) {
    st = M::combine(st, M::unpack(partial[t * nb + b]));
    emit |= tile_emit[t * nb + b];
  }
}

// first level of the ordered combine of groups with many chunks: slice s of
// group i (chunks [t0 + s*L, t0 + (s+1)*L)) -> scratch row i*ns + s
template <class M>
__global__ __launch_bounds__(256) void k_combine_l1(
    int64_t nb, int64_t n_groups, int64_t ns,
    const int64_t* __restrict__ grp_t0, const int64_t* __restrict__ grp_t1,
    const Packed* __restrict__ partial, const uint8_t* __restrict__ tile_emit,
    Packed* __restrict__ scratch, uint8_t* __restrict__ scratch_emit) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = idx / nb;  // i * ns + s
  if (row >= n_groups * ns) return;
  const int64_t b = idx - row * nb;
  const int64_t i = row / ns, sl = row - i * ns;
  const int64_t t0 = grp_t0[i], t1 = grp_t1[i];
  const int64_t L = (t1 - t0 + ns - 1) / ns;
  const int64_t a = t0 + sl * L;
  const int64_t e = a + L < t1 ? a + L : t1;
  M st = M::init();
  int emit = 0;
  if (a < e) fold_chunks<M>(partial, tile_emit, nb, b, a, e, st, emit);
  scratch[row * nb + b] = st.pack();
  scratch_emit[row * nb + b] = (uint8_t)emit;
}

// merge the chunk partials of multi-chunk groups in chunk order (ns > 0:
// the ns first-level slices of k_combine_l1, rows [i*ns, (i+1)*ns))
template <class M>
__global__ __launch_bounds__(256) void k_combine(
    int64_t nb, int64_t n_groups, const int64_t* __restrict__ grp_g,
    const int64_t* __restrict__ grp_t0, const int64_t* __restrict__ grp_t1,
    const Packed* __restrict__ partial, const uint8_t* __restrict__ tile_emit,
    double* __restrict__ out_val, uint8_t* __restrict__ out_emit,
    Packed* __restrict__ out_partial, int* err_word, int64_t ns,
    int keep_empty = 0) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = idx / nb;
  if (i >= n_groups) return;
  const int64_t b = idx - i * nb;
  const int64_t g = grp_g[i];
  // chained partials: a group with no local member keeps the state it came
  // with (copied to out_partial before the pipeline)
  if (keep_empty && grp_t0[i] == grp_t1[i]) return;
  M st = M::init();
  int emit = 0;
  if (ns > 0)
    fold_chunks<M>(partial, tile_emit, nb, b, i * ns, (i + 1) * ns, st, emit);
  else
    fold_chunks<M>(partial, tile_emit, nb, b, grp_t0[i], grp_t1[i], st, emit);
  const int64_t o = g * nb + b;
  if (out_partial) {
    out_partial[o] = st.pack();
    out_emit[o] = (uint8_t)emit;
    return;
  }
  double r = 0.0;
  if (emit) {
    int e = 0;
    r = st.finish(&e);
    if (is_inf(r)) e |= ERR_INFINITY;
    if (e) atomicOr(err_word, e);
  }
  out_val[o] = r;
  out_emit[o] = (uint8_t)emit;
}

// multi-GPU: merge per-rank partials in rank (= series) order, finalise
template <class M>
__global__ __launch_bounds__(256) void k_finalize_ranks(
    int64_t GB, int n_ranks, const Packed* __restrict__ partials,
    const uint8_t* __restrict__ emits, double* __restrict__ out_val,
    uint8_t* __restrict__ out_emit, int* err_word) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= GB) return;
  M st = M::init();
  int emit = 0;
  for (int r = 0; r < n_ranks; ++r) {
    st = M::combine(st, M::unpack(partials[(int64_t)r * GB + o]));
    emit |= emits[(int64_t)r * GB + o];
  }
  double v = 0.0;
  if (emit) {
    int e = 0;
    v = st.finish(&e);
    if (is_inf(v)) e |= ERR_INFINITY;
    if (e) atomicOr(err_word, e);
  }
  out_val[o] = v;
  out_emit[o] = (uint8_t)emit;
}

#ifndef OTSDB_DS_TU
// ------------------------------------------------------------------------
// Percentile / median across series (PercentileAgg.runDouble,
// Aggregators.java:687-706 — LEGACY estimation whatever the name says; and
// Median.runDouble, :412-431).  One thread per (group, bucket) for groups of
// up to SEL_K series: non-NaN contributions sorted in LDS, then selected.
// ------------------------------------------------------------------------
constexpr int SEL_K = 32;
constexpr int SEL_THREADS = 128;

DEV uint64_t order_key(double v) {  // total order, -0.0 < 0.0 (compareTo)
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}

__global__ __launch_bounds__(SEL_THREADS) void k_group_select(
    int64_t nb, int64_t n_tiles, const int64_t* __restrict__ tile_g,
    const int64_t* __restrict__ tile_m0, const int64_t* __restrict__ tile_m1,
    const uint8_t* __restrict__ tile_single,
    const int64_t* __restrict__ members, Rows R, double* __restrict__ out_val,
    uint8_t* __restrict__ out_emit, int* err_word, int median, double p) {
  __shared__ uint64_t buf[SEL_K * SEL_THREADS];
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t t = idx / nb;
  if (t >= n_tiles) return;
  const int64_t b = idx - t * nb;
  // groups above SEL_K series go through the radix-select path (select.hip)
  if (!tile_single[t]) return;
  const int64_t m0 = tile_m0[t], m1 = tile_m1[t];
  if (m1 - m0 > SEL_K) return;
  int n = 0, emit = 0;
  for (int64_t m = m0; m < m1; ++m) {
    const int64_t off = members[m] * nb + b;
    const uint8_t sv = R.state[off];
    if (!sv) continue;
    emit |= sv == ST_REAL;
    const double v = R.val[off];
    if (is_nan(v)) continue;
    // insertion sort by total order
    const uint64_t k = order_key(v);
    int j = n++;
    while (j > 0 && buf[(j - 1) * SEL_THREADS + threadIdx.x] > k) {
      buf[j * SEL_THREADS + threadIdx.x] = buf[(j - 1) * SEL_THREADS + threadIdx.x];
      --j;
    }
    buf[j * SEL_THREADS + threadIdx.x] = k;
  }
  auto val_at = [&](int i) {
    const uint64_t k = buf[i * SEL_THREADS + threadIdx.x];
    const uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k;
    return __longlong_as_double((long long)u);
  };
  double r = 0.0;
  if (emit) {
    if (n == 0) {
      r = qnan();
    } else if (median) {
      r = val_at(n / 2);
    } else if (n == 1) {
      r = val_at(0);
    } else {
      const double pos = p * (double)(n + 1);
      const double fpos = __builtin_floor(pos);
      const int ip = (int)fpos;
      const double dif = pos - fpos;
      if (pos < 1) r = val_at(0);
      else if (pos >= (double)n) r = val_at(n - 1);
      else {
        const double lower = val_at(ip - 1), upper = val_at(ip);
        r = lower + dif * (upper - lower);
      }
    }
    if (is_inf(r)) atomicOr(err_word, ERR_INFINITY);
  }
  const int64_t o = tile_g[t] * nb + b;
  out_val[o] = r;
  out_emit[o] = (uint8_t)emit;
}

// exclusive scan of counts[G] -> offsets[G+1] (single workgroup; G is the
// number of output groups, small next to the point stream)
__global__ __launch_bounds__(1024) void k_scan(int64_t G,
                                               const int64_t* __restrict__ in,
                                               int64_t* __restrict__ out) {
  __shared__ int64_t part[1024];
  const int tid = threadIdx.x;
  const int64_t per = (G + 1023) / 1024;
  const int64_t a = tid * per, e = (a + per < G) ? a + per : G;
  int64_t sum = 0;
  for (int64_t i = a; i < e; ++i) sum += in[i];
  part[tid] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int64_t x = tid >= d ? part[tid - d] : 0;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  int64_t run = part[tid] - sum;
  for (int64_t i = a; i < e; ++i) {
    out[i] = run;
    run += in[i];
  }
  if (tid == 1023) out[G] = part[1023];
}

// bounds of the data inside [seek_ts, stop_ts) (grid trimming for very wide
// windows)
__global__ void k_bounds(Params P, BatchDev B, unsigned long long* mm) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= B.S) return;
  const int64_t p0 = B.offsets[s], p1 = B.offsets[s + 1];
  if (p1 <= p0) return;
  const int64_t lo = lower_bound(B.ts, p0, p1, P.seek_ts);
  const int64_t hi = lower_bound(B.ts, lo, p1, P.stop_ts);
  if (lo >= hi) return;
  atomicMin(&mm[0], (unsigned long long)B.ts[lo]);
  atomicMax(&mm[1], (unsigned long long)B.ts[hi - 1]);
}

// ------------------------------------------------------------------------
// Synthetic workload generator (bit-identical to
// or_gen_fill in oracle/otsdb_oracle.c).  One wavefront per series.
// ------------------------------------------------------------------------
constexpr uint64_t GOLDEN = 0x9E3779B97F4A7C15ULL;
DEV uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

struct GenSeries {
  uint64_t key;
  int64_t n, first, last, phase;
  int n_out;
  int64_t out_lo[2], out_hi[2];
  int64_t counter0;
};

struct GenP {
  uint64_t seed;
  int64_t t0_ms, duration_ms, cadence_ms;
  int kind;
  int flags;  // otsdb_gen_spec.flags: 1 = whole-second phases
};

DEV GenSeries gen_params(const GenP& g, int64_t s) {
  GenSeries p;
  const uint64_t key = mix64((g.seed ^ (uint64_t)s) + GOLDEN);
  uint64_t r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = mix64(key + GOLDEN * (uint64_t)(j + 1));
  p.key = key;
  p.n = g.duration_ms / g.cadence_ms;
  p.phase = (int64_t)(r[0] % (uint64_t)g.cadence_ms);
  if (g.flags & 1) p.phase -= p.phase % 1000;
  p.first = 0;
  p.last = p.n;
  if (p.n > 1 && (r[1] % 100) < 5) {
    const int64_t cut = (int64_t)(r[3] % (uint64_t)(p.n / 2));
    if (r[2] & 1) p.first = cut;
    else p.last = p.n - cut;
  }
  p.n_out = (int)(r[4] % 3);
  const int64_t pph = 3600000 / g.cadence_ms;
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const uint64_t x = r[5 + o];
    const int64_t lo = (int64_t)(x % (uint64_t)(p.n > 0 ? p.n : 1));
    p.out_lo[o] = lo;
    p.out_hi[o] = lo + (int64_t)(1 + ((x >> 32) % 6)) * pph;
  }
  p.counter0 = (int64_t)(r[7] & 0xFFFFFFFFULL);
  return p;
}

DEV bool gen_present(const GenSeries& p, int64_t i) {
  if (i < p.first || i >= p.last) return false;
  for (int o = 0; o < p.n_out; ++o)
    if (i >= p.out_lo[o] && i < p.out_hi[o]) return false;
  const uint64_t h = mix64(p.key ^ ((uint64_t)(i + 1) * 0xD1B54A32D192ED03ULL));
  return (h >> 11) >= 180143985094819ULL;
}

__global__ __launch_bounds__(256) void k_gen_counts(GenP g, int64_t series0,
                                                    int64_t n_series,
                                                    int64_t* counts) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= n_series) return;
  const GenSeries p = gen_params(g, series0 + w);
  int64_t c = 0;
  for (int64_t c0 = 0; c0 < p.n; c0 += 64) {
    const int64_t i = c0 + LANE;
    c += __popcll(__ballot(i < p.n && gen_present(p, i)));
  }
  if (LANE == 0) counts[w] = c;
}

__global__ __launch_bounds__(256) void k_gen_fill(GenP g, int64_t series0,
                                                  int64_t n_series,
                                                  const int64_t* offsets,
                                                  int64_t* ts, int64_t* val) {
  const int lane = LANE;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= n_series) return;
  const GenSeries p = gen_params(g, series0 + w);
  int64_t pos = offsets[w];
  int64_t counter = p.counter0;
  for (int64_t c0 = 0; c0 < p.n; c0 += 64) {
    const int64_t i = c0 + lane;
    const bool inr = i < p.n;
    const uint64_t hv = mix64(p.key + (uint64_t)(i + 1) * 0x8CB92BA72F3D8DD7ULL);
    int64_t v = 0;
    if (g.kind == 2) {
      // counter: running sum of increments, reset to 0 (segmented scan)
      int rst = inr && ((hv >> 40) % 10000) == 0;
      int64_t x = (!inr || rst) ? 0 : (int64_t)(500 + (hv % 1001));
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int r2 = __shfl_up(rst, d);
        const int64_t x2 = __shfl_up(x, d);
        if (lane >= d && !rst) {
          x += x2;
          rst |= r2;
        }
      }
      v = rst ? x : counter + x;
      counter = __shfl(v, 63);
    } else if (g.kind == 0) {
      v = __double_as_longlong((double)(hv >> 11) * 0x1p-53 * 100.0);
    } else {
      v = (int64_t)((hv >> 11) % 100);
    }
    const bool pr = inr && gen_present(p, i);
    const uint64_t m = __ballot(pr);
    if (pr) {
      const int64_t q = pos + __popcll(m & ((1ULL << lane) - 1));
      ts[q] = g.t0_ms + p.phase + i * g.cadence_ms;
      val[q] = v;
    }
    pos += __popcll(m);
  }
}

#endif  // OTSDB_DS_TU

}  // namespace otsdb
