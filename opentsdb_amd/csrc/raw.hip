// raw.hip — raw (non-downsampled) group-by: AggregationIterator over the
// spans' own points (src/core/AggregationIterator.java:395-797), every
// Aggregators entry on both the long (runLong) and the double (runDouble)
// path.
//
// Pipeline (one query, every group at once):
//   k_raw_prep        per series: SpanGroup.add filter (SpanGroup.java:321-338)
//                     and the iterator's seek(start) (first point >= start,
//                     AggregationIterator.java:414-441)
//   k_raw_rate        (rate queries) one wavefront per series: RateSpan over
//                     the points from the seek on (RateSpan.java:121-180), the
//                     first rate taken against (0, 0); dropped resets
//                     compacted out with a ballot
//   k_raw_cand_*      per member: the points the member feeds to the emission
//                     loop (its "next" slot values with ts <= end), gathered
//                     per group, then sorted per group (rocPRIM segmented
//                     radix sort) — the emitted timestamps are their union
//   k_raw_unique      per group: distinct timestamps -> result ts arrays
//   k_raw_eval        one thread per emitted point: walks the group's spans
//                     in SpanCmp order exactly like the Java iterator
//                     (contribution rule, isInteger over current+next slots,
//                     LERP/ZIM/MAX/MIN/PREV, rate hold) and feeds the
//                     aggregator sequentially — bit-identical to the Java loop
//   k_raw_select      median / percentiles: one wavefront per emitted point,
//                     radix select over the contributions' order keys
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace otsdb {

// ---------------------------------------------------------- Java long math
DEV int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
DEV int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
DEV int64_t jmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
DEV int64_t jdiv(int64_t a, int64_t b) {  // truncating; MIN / -1 wraps
  return b == -1 ? jsub(0, a) : a / b;
}
DEV int64_t d2l(double d) {  // Java (long) cast: NaN -> 0, saturating
  if (d != d) return 0;
  if (d >= 9.2233720368547758e18) return INT64_MAX;
  if (d <= -9.2233720368547758e18) return INT64_MIN;
  return (int64_t)d;
}

constexpr int64_t kMsMask = (int64_t)0xFFFFF00000000000ULL;  // Const.java:92

// The per-series point streams the iterator walks: the batch's own points
// (non-rate) or the rate points k_raw_rate wrote (all doubles).
struct RawView {
  const int64_t* ts;
  const int64_t* val;
  const uint8_t* is_float;      // per point, or null
  const uint8_t* series_float;  // per series, or null
  int all_double;               // every point is a double
  int64_t* lo;                  // [S] first point (first point >= start)
  int64_t* hi;                  // [S] one past the last point
};

DEV int view_float(const RawView& V, int64_t s, int64_t i) {
  if (V.all_double) return 1;
  if (V.is_float) return V.is_float[i];
  return V.series_float ? V.series_float[s] : 1;
}

DEV double view_double(const RawView& V, int64_t s, int64_t i) {
  const int64_t b = V.val[i];
  return view_float(V, s, i) ? __longlong_as_double(b) : (double)b;
}

// last index in [a, b) with ts <= x, or a - 1
DEV int64_t last_le(const int64_t* ts, int64_t a, int64_t b, int64_t x) {
  int64_t lo = a, hi = b;
  while (lo < hi) {
    const int64_t m = lo + ((hi - lo) >> 1);
    if (ts[m] <= x) lo = m + 1;
    else hi = m;
  }
  return lo - 1;
}

// ------------------------------------------------------------------------
// k_raw_prep: one thread per series.
// ------------------------------------------------------------------------
__global__ void k_raw_prep(Params P, BatchDev B, int64_t* __restrict__ lo,
                           int64_t* __restrict__ hi) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= B.S) return;
  const int64_t p0 = B.offsets[s], p1 = B.offsets[s + 1];
  const bool keep = p1 > p0 && B.ts[p0] <= P.end_ms && B.ts[p1 - 1] >= P.start_ms;
  lo[s] = keep ? lower_bound(B.ts, p0, p1, P.start_ms) : p1;
  hi[s] = p1;
}

// ------------------------------------------------------------------------
// k_raw_rate: RateSpan.populateNextRate over the points [lo, hi) of a series
// (one wavefront per series).  Rate i uses source points i-1 and i; the
// first against (0, 0 long).  Kept rates are written compactly from the
// series' own offset (rates never outnumber points).
// ------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_raw_rate(Params P, BatchDev B,
                                                  int64_t* __restrict__ lo,
                                                  int64_t* __restrict__ hi,
                                                  int64_t* __restrict__ rts,
                                                  int64_t* __restrict__ rval,
                                                  int* err_word) {
  const int lane = LANE;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= B.S) return;
  const int64_t a = lo[s], b = hi[s];
  const int64_t base = B.offsets[s];
  const int sf = B.series_float ? (int)B.series_float[s] : 1;
  auto flt = [&](int64_t i) { return B.is_float ? (int)B.is_float[i] : sf; };
  int64_t pos = base;
  int bad = 0;
  for (int64_t c0 = a; c0 < b; c0 += 64) {
    const int64_t i = c0 + lane;
    bool kept = false;
    double rate = 0.0;
    int64_t t1 = 0;
    if (i < b) {
      int64_t t0 = 0, v0 = 0;
      int f0 = 0;
      if (i > a) {
        t0 = B.ts[i - 1];
        v0 = B.val[i - 1];
        f0 = flt(i - 1);
      }
      t1 = B.ts[i];
      const int64_t v1 = B.val[i];
      const int f1 = flt(i);
      if (t1 <= t0) bad = 1;
      const double dt = (double)jsub(t1, t0) / 1000.0;
      const bool both_int = !f0 && !f1;
      const double d0 = f0 ? __longlong_as_double(v0) : (double)v0;
      const double d1 = f1 ? __longlong_as_double(v1) : (double)v1;
      double diff = both_int ? (double)jsub(v1, v0) : d1 - d0;
      if (P.counter && diff < 0) {
        if (!P.drop_resets) {
          kept = true;
          diff = both_int ? (double)jadd(jsub(P.counter_max, v0), v1)
                          : (double)P.counter_max - d0 + d1;
          const double r = diff / dt;
          rate = (P.reset_value > 0 && r > (double)P.reset_value) ? 0.0 : r;
        }
      } else {
        kept = true;
        rate = diff / dt;
      }
    }
    const uint64_t m = __ballot(kept);
    if (kept) {
      const int64_t q = pos + __popcll(m & ((1ULL << lane) - 1));
      rts[q] = t1;
      rval[q] = __double_as_longlong(rate);
    }
    pos += __popcll(m);
  }
  if (__ballot(bad) && lane == 0) atomicOr(err_word, ERR_RATE_TS);
  if (lane == 0) {
    lo[s] = base;
    hi[s] = pos;
  }
}

// ------------------------------------------------------------------------
// Emission candidates.  A member's points enter the emission loop through
// its "next" slot: from its first point on (from its second with rate, whose
// first rate is pre-consumed into the current slot,
// AggregationIterator.java:448-459), while ts <= end (hasNext, :500-512).
// ------------------------------------------------------------------------
DEV void cand_range(const Params& P, const RawView& V, int64_t s, int64_t* a,
                    int64_t* b) {
  int64_t x = V.lo[s], y = V.hi[s];
  if (P.rate) {
    // a single rate point ends the span in the constructor (endReached)
    if (y - x < 2) {
      *a = *b = x;
      return;
    }
    ++x;
  }
  *a = x;
  *b = (x < y) ? last_le(V.ts, x, y, P.end_ms) + 1 : x;
}

__global__ void k_raw_cand_count(Params P, RawView V, int64_t M,
                                 const int64_t* __restrict__ members,
                                 int64_t* __restrict__ count) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  int64_t a, b;
  cand_range(P, V, members[m], &a, &b);
  count[m] = b - a;
}

// Repeated timestamps inside a span.  The iterator's next() moves every
// span whose "next" slot holds the minimum timestamp, one point each
// (AggregationIterator.java:514-588): a timestamp held k times by one span
// is emitted k times, the m-th emission moving that span's m-th copy into
// its current slot while the other spans keep theirs.  An emission is the
// pair (x, m) — m the occurrence of x inside the span that holds it — and
// the candidates carry it as the key (x << 16) | m: the group's distinct
// keys, in order, are its emissions.
constexpr int kOccBits = 16;
constexpr int64_t kOccMax = (int64_t)1 << kOccBits;
constexpr int64_t kRawTsMax = (int64_t)1 << (63 - kOccBits);

// one wavefront per member: the candidate keys; a timestamp that decreases
// inside a span, a run of more than 2^16 copies or a timestamp past 2^47 ms
// flags ERR_RAW_DUP (E_UNSUPPORTED)
__global__ __launch_bounds__(256) void k_raw_cand_fill(
    Params P, RawView V, int64_t M, const int64_t* __restrict__ members,
    const int64_t* __restrict__ cand_off, uint64_t* __restrict__ keys,
    int* err_word) {
  const int lane = LANE;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  int64_t a, b;
  cand_range(P, V, members[m], &a, &b);
  const int64_t o = cand_off[m] - a;
  int bad = 0;
  for (int64_t i = a + lane; i < b; i += 64) {
    const int64_t t = V.ts[i];
    // occurrence of t: the copies before it in the span (from its seek:
    // copies before the first candidate were never in the next slot); the
    // run's first copy by a gallop back from i, O(log occ) loads, not a
    // walk (a run of k copies cost O(k^2) walking; on a decreasing span the
    // value is moot: the query is flagged below)
    const int64_t occ = i - lower_bound_back(V.ts, a, i + 1, t);
    keys[o + i] = ((uint64_t)t << kOccBits) | (uint64_t)occ;
    if ((i > a && V.ts[i - 1] > t) || occ >= kOccMax || t >= kRawTsMax) bad = 1;
  }
  if (__ballot(bad) && lane == 0) atomicOr(err_word, ERR_RAW_DUP);
}

// per group segment bounds of the candidate array (for the segmented sort)
__global__ void k_raw_segments(int64_t G, const int64_t* __restrict__ goff,
                               const int64_t* __restrict__ cand_off,
                               int64_t* __restrict__ seg_b,
                               int64_t* __restrict__ seg_e) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  seg_b[g] = cand_off[goff[g]];
  seg_e[g] = cand_off[goff[g + 1]];
}

// one wavefront per group: distinct sorted candidate keys.  mode 0 counts,
// mode 1 writes the emitted timestamps, their occurrence and their group.
__global__ __launch_bounds__(256) void k_raw_unique(
    int64_t G, const int64_t* __restrict__ seg_b,
    const int64_t* __restrict__ seg_e, const uint64_t* __restrict__ sorted,
    int64_t* __restrict__ counts, const int64_t* __restrict__ out_off,
    int64_t cap, int64_t* __restrict__ out_ts, int32_t* __restrict__ ugrp,
    int32_t* __restrict__ uocc, int mode) {
  const int lane = LANE;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= G) return;
  const int64_t a = seg_b[g], b = seg_e[g];
  int64_t pos = mode ? out_off[g] : 0;
  for (int64_t c0 = a; c0 < b; c0 += 64) {
    const int64_t i = c0 + lane;
    const bool d = i < b && (i == a || sorted[i] != sorted[i - 1]);
    const uint64_t m = __ballot(d);
    if (mode && d) {
      const int64_t p = pos + __popcll(m & ((1ULL << lane) - 1));
      if (p < cap) {
        out_ts[p] = (int64_t)(sorted[i] >> kOccBits);
        uocc[p] = (int32_t)(sorted[i] & (kOccMax - 1));
        ugrp[p] = (int32_t)g;
      }
    }
    pos += __popcll(m);
  }
  if (!mode && lane == 0) counts[g] = pos;
}

// ------------------------------------------------------------------------
// One span's slots at emission (x, occ) (AggregationIterator.next/
// moveToNext):
//   state 0: not started (x < first point): current slot empty, next slot
//            holds the first point
//   state 1: contributing (first <= x <= last, or any x with a rate span
//            whose junk first rate sits in the current slot): current = the
//            latest point <= x (the junk rate before the second rate point),
//            next = the one after it, if any.  With k copies of x in the
//            span, emission (x, occ) holds copy min(occ, k - 1).
//   state 2: ended / empty: both slots empty (zeroed / TIME_MASK).  A span
//            expires at the next() after its last point entered the current
//            slot (:519-526): after emission (last, k - 1).
// ------------------------------------------------------------------------
struct Slots {
  int state;
  int64_t cur, nxt;  // point indices; nxt = -1 when the slot is TIME_MASK
};

DEV Slots span_slots(const Params& P, const RawView& V, int64_t s, int64_t x,
                     int occ) {
  Slots r{2, -1, -1};
  const int64_t a = V.lo[s], b = V.hi[s];
  if (P.rate) {
    if (b - a < 2 || x > V.ts[b - 1]) return r;
    r.state = 1;
    r.cur = last_le(V.ts, a, b, x);
    if (r.cur < a) r.cur = a;
    r.nxt = r.cur + 1 < b ? r.cur + 1 : -1;
    return r;
  }
  if (a >= b || x > V.ts[b - 1]) return r;
  if (V.ts[a] > x) {
    r.state = 0;
    r.nxt = a;
    return r;
  }
  r.state = 1;
  r.cur = last_le(V.ts, a, b, x);
  if (V.ts[r.cur] == x && (occ > 0 || (r.cur > a && V.ts[r.cur - 1] == x))) {
    // copies of x: [f, r.cur]; emission occ holds copy occ (f by a gallop
    // back: O(log k) loads per (emission, member))
    const int64_t f = lower_bound_back(V.ts, a, r.cur + 1, x);
    if (r.cur - f >= occ) {
      r.cur = f + occ;
    } else if (r.cur == b - 1) {  // fewer copies: the last point expired
      r.state = 2;
      r.cur = r.nxt = -1;
      return r;
    }
  }
  r.nxt = r.cur + 1 < b ? r.cur + 1 : -1;
  return r;
}

// AggregationIterator.isInteger (:612-625): no float in any slot
DEV int slots_float(const RawView& V, int64_t s, const Slots& q) {
  int f = 0;
  if (q.state == 1) f |= view_float(V, s, q.cur);
  if (q.nxt >= 0) f |= view_float(V, s, q.nxt);
  return f;
}

// nextDoubleValue (:735-797) for a contributing span
DEV double span_double(const Params& P, const RawView& V, int64_t s,
                       const Slots& q, int64_t x, int* err) {
  const double y0 = view_double(V, s, q.cur);
  if (P.rate) return y0;
  const int64_t x0 = V.ts[q.cur];
  if (x == x0) return y0;
  const double y1 = view_double(V, s, q.nxt);
  const int64_t x1 = V.ts[q.nxt];
  if (x == x1) return y1;
  if (x1 & kMsMask) *err |= ERR_X1_MASK;
  switch (P.interp) {
    case 0: return y0 + (double)jsub(x, x0) * (y1 - y0) / (double)jsub(x1, x0);
    case 1: return 0.0;
    case 2: return kDoubleMax;
    case 3: return -kDoubleMax;
    default: return y0;
  }
}

// nextLongValue (:682-729) for a contributing span (long slots only)
DEV int64_t span_long(const Params& P, const RawView& V, const Slots& q,
                      int64_t x, int* err) {
  const int64_t y0 = V.val[q.cur];
  const int64_t x0 = V.ts[q.cur];
  if (x == x0) return y0;
  const int64_t y1 = V.val[q.nxt];
  const int64_t x1 = V.ts[q.nxt];
  if (x == x1) return y1;
  if (x1 & kMsMask) *err |= ERR_X1_MASK;
  switch (P.interp) {
    case 0: return jadd(y0, jdiv(jmul(jsub(x, x0), jsub(y1, y0)), jsub(x1, x0)));
    case 1: return 0;
    case 2: return INT64_MAX;
    case 3: return INT64_MIN;
    default: return y0;
  }
}

// Aggregator.runLong of every non-selection aggregator (Aggregators.java),
// fed sequentially in span order.
struct LongAcc {
  int agg;
  int64_t a, b, n;
  double mean, m2;
  DEV explicit LongAcc(int g) : agg(g), a(0), b(0), n(0), mean(0.0), m2(0.0) {}
  DEV void push(int64_t v) {
    switch (agg) {
      case OTSDB_AGG_SUM: case OTSDB_AGG_PFSUM: case OTSDB_AGG_ZIMSUM:
      case OTSDB_AGG_AVG:
        a = n ? jadd(a, v) : v; break;
      case OTSDB_AGG_SQUARESUM: a = n ? jadd(a, jmul(v, v)) : jmul(v, v); break;
      case OTSDB_AGG_MIN: case OTSDB_AGG_MIMMIN: a = (n && a <= v) ? a : v; break;
      case OTSDB_AGG_MAX: case OTSDB_AGG_MIMMAX: a = (n && a >= v) ? a : v; break;
      case OTSDB_AGG_MULT: a = n ? jmul(a, v) : v; break;
      case OTSDB_AGG_DEV:  // StdDev.runLong (:498-531): Welford from n = 2
        if (n == 0) {
          mean = (double)v;
        } else {
          const double x = (double)v;
          const double nm = mean + (x - mean) / (double)(n + 1);
          m2 += (x - mean) * (x - nm);
          mean = nm;
        }
        break;
      case OTSDB_AGG_DIFF: if (n == 0) a = v; else b = v; break;
      case OTSDB_AGG_FIRST: case OTSDB_AGG_NONE: if (n == 0) a = v; break;
      case OTSDB_AGG_LAST: a = v; break;
      default: break;  // count
    }
    ++n;
  }
  DEV int64_t finish(int* err) const {
    switch (agg) {
      case OTSDB_AGG_AVG: return jdiv(a, (int64_t)(int32_t)n);
      case OTSDB_AGG_COUNT: return n;
      case OTSDB_AGG_NONE: if (n > 1) *err |= ERR_NONE_MULTI; return a;
      case OTSDB_AGG_DEV: return n == 1 ? 0 : d2l(__builtin_sqrt(m2 / (double)n));
      case OTSDB_AGG_DIFF: return n == 1 ? 0 : jsub(b, a);
      default: return a;
    }
  }
};

// ------------------------------------------------------------------------
// k_raw_eval: one thread per emitted point (threads of a wavefront take
// consecutive points of one group, so the spans' binary searches share
// cache lines).  M is the double-path monoid of the aggregator.
// ------------------------------------------------------------------------
template <class M>
__global__ __launch_bounds__(256) void k_raw_eval(
    Params P, RawView V, int agg, int mixed, int64_t n_out,
    const int64_t* __restrict__ goff, const int64_t* __restrict__ members,
    const int32_t* __restrict__ ugrp, const int32_t* __restrict__ uocc,
    const int64_t* __restrict__ out_ts, int64_t* __restrict__ out_val,
    uint8_t* __restrict__ out_isint, int* err_word) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n_out) return;
  const int32_t g = ugrp[u];
  const int64_t x = out_ts[u];
  const int occ = uocc[u];
  const int64_t m0 = goff[g], m1 = goff[g + 1];
  int err = 0;
  // isInteger: decided over every span's slots before any value is read
  bool is_int = !P.rate && !V.all_double;
  if (is_int && mixed) {
    for (int64_t m = m0; m < m1 && is_int; ++m) {
      const int64_t s = members[m];
      is_int = !slots_float(V, s, span_slots(P, V, s, x, occ));
    }
  }
  int64_t bits;
  if (is_int) {
    LongAcc acc(agg);
    for (int64_t m = m0; m < m1; ++m) {
      const int64_t s = members[m];
      const Slots q = span_slots(P, V, s, x, occ);
      if (q.state == 1) acc.push(span_long(P, V, q, x, &err));
    }
    bits = acc.finish(&err);
  } else {
    M st = M::init();
    for (int64_t m = m0; m < m1; ++m) {
      const int64_t s = members[m];
      const Slots q = span_slots(P, V, s, x, occ);
      if (q.state == 1) st.push(span_double(P, V, s, q, x, &err));
    }
    const double r = st.finish(&err);
    if (is_inf(r)) err |= ERR_INFINITY;
    bits = __double_as_longlong(r);
  }
  out_val[u] = bits;
  out_isint[u] = is_int ? 1 : 0;
  if (err) atomicOr(err_word, err);
}

// ------------------------------------------------------------------------
// Selection (median / percentiles) on the raw path.
// ------------------------------------------------------------------------
DEV uint64_t raw_dkey(double v) {  // total order, -0.0 < 0.0
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
DEV double raw_key_double(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k;
  return __longlong_as_double((long long)u);
}
DEV uint64_t raw_lkey(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ULL; }

// commons-math3 3.4.1 Percentile position for estimation `est`
// (0 LEGACY, 3 R_3, 7 R_7), SURVEY §8a a11
DEV double pct_position(double p, int64_t n, int est) {
  if (est == 3) return (p <= 0.5 / (double)n) ? 0.0 : __builtin_rint((double)n * p);
  if (est == 7) return (p == 0.0) ? 0.0 : (p == 1.0 ? (double)n : 1.0 + (double)(n - 1) * p);
  return (p == 0.0) ? 0.0 : (p == 1.0 ? (double)n : p * (double)(n + 1));
}

// one wavefront (block of 64) per emitted point u0 + blockIdx.x; `slab`
// holds kmax keys per block
__global__ __launch_bounds__(64) void k_raw_select(
    Params P, RawView V, int median, int64_t u0, int64_t n_out,
    const int64_t* __restrict__ goff, const int64_t* __restrict__ members,
    const int32_t* __restrict__ ugrp, const int32_t* __restrict__ uocc,
    const int64_t* __restrict__ out_ts, int64_t* __restrict__ out_val,
    uint8_t* __restrict__ out_isint, uint64_t* __restrict__ slab,
    int64_t kmax, int* err_word) {
  __shared__ uint32_t hist[256];
  const int lane = LANE;
  const int64_t u = u0 + blockIdx.x;
  if (u >= n_out) return;
  const int32_t g = ugrp[u];
  const int64_t x = out_ts[u];
  const int occ = uocc[u];
  const int64_t m0 = goff[g], m1 = goff[g + 1];
  int err = 0;
  int fl = 0;
  const bool typed = !P.rate && !V.all_double;
  if (typed)
    for (int64_t m = m0 + lane; m < m1; m += 64) {
      const int64_t s = members[m];
      fl |= slots_float(V, s, span_slots(P, V, s, x, occ));
    }
  const bool is_int = typed && __ballot(fl) == 0;
  uint64_t* keys = slab + (int64_t)blockIdx.x * kmax;
  int64_t n = 0;
  for (int64_t mb = m0; mb < m1; mb += 64) {
    const int64_t m = mb + lane;
    bool has = false;
    uint64_t key = 0;
    if (m < m1) {
      const int64_t s = members[m];
      const Slots q = span_slots(P, V, s, x, occ);
      if (q.state == 1) {
        if (is_int) {
          const int64_t v = span_long(P, V, q, x, &err);
          key = median ? raw_lkey(v) : raw_dkey((double)v);
          has = true;
        } else {
          const double v = span_double(P, V, s, q, x, &err);
          has = !is_nan(v);  // NaNs are filtered (Median/PercentileAgg)
          key = raw_dkey(v);
        }
      }
    }
    const uint64_t bm = __ballot(has);
    if (has) keys[n + __popcll(bm & ((1ULL << lane) - 1))] = key;
    n += __popcll(bm);
  }
  __syncthreads();
  // the ranks the estimator reads
  const int est = is_int ? P.pct_est : 0;  // runDouble ignores it (:690)
  int64_t r0 = 0, r1 = 0;
  double pos = 0.0;
  bool empty = n == 0;
  if (!empty) {
    if (median) {
      r0 = r1 = n / 2;
    } else if (n > 1) {
      pos = pct_position(P.pct, n, est);
      if (pos < 1) {
        r0 = r1 = 0;
      } else if (pos >= (double)n) {
        r0 = r1 = n - 1;
      } else {
        const int64_t ip = (int64_t)__builtin_floor(pos);
        r0 = ip - 1;
        r1 = ip;
      }
    }
  }
  uint64_t k0 = 0, k1 = 0;
  if (!empty) {
    auto key_at = [&](int64_t i) { return keys[i]; };
    k0 = wave_select(n, r0, hist, key_at);
    k1 = (r1 == r0) ? k0 : wave_select(n, r1, hist, key_at);
  }
  if (lane != 0) return;
  int64_t bits;
  if (is_int) {
    // Median.runLong (:397-411): a[n/2]; PercentileAgg.runLong: (long) of
    // the estimate over the values as doubles (:676-685)
    if (median) {
      bits = (int64_t)(k0 ^ 0x8000000000000000ULL);
    } else {
      const double lo = raw_key_double(k0), hi = raw_key_double(k1);
      double r = lo;
      if (n > 1 && pos >= 1 && pos < (double)n)
        r = lo + (pos - __builtin_floor(pos)) * (hi - lo);
      bits = d2l(r);
    }
  } else {
    double r;
    if (empty) {
      r = qnan();
    } else if (median || n == 1) {
      r = raw_key_double(k0);
    } else {
      const double lo = raw_key_double(k0), hi = raw_key_double(k1);
      r = lo;
      if (pos >= 1 && pos < (double)n)
        r = lo + (pos - __builtin_floor(pos)) * (hi - lo);
    }
    if (is_inf(r)) err |= ERR_INFINITY;
    bits = __double_as_longlong(r);
  }
  out_val[u] = bits;
  out_isint[u] = is_int ? 1 : 0;
  if (err) atomicOr(err_word, err);
}

}  // namespace otsdb
