// monoids.h — per-aggregator reduction states for the GPU engine.
//
// Every Aggregators entry (src/core/Aggregators.java:231-852) is expressed as
//   push(state, v)      sequential step, bit-identical to the Java loop body
//   combine(a, b)       merge of two adjacent runs (a before b)
//   finish(state)       runDouble's return value
// push() is used wherever the engine can keep Java's order (cross-series
// reduction inside a chunk: bit-exact vs the reference for groups of up to
// CHUNK series); combine() where it reduces in a tree (downsample buckets in
// a wavefront, chunk and rank merges) — exact for min/max/count/first/last/
// diff, within 1e-12 relative for sum/avg/mult/squareSum (north star).
// kOrdered monoids (dev) never take the tree inside a downsample bucket:
// Welford over offset data (counters near 2^32 with a spread of 10^4) is
// ill-conditioned, and the reference's own sequential result lies ~1e-11
// from the exact one, so any other order — Chan's merge included, even in
// exact arithmetic — lands ~1e-11 from the reference's.  reduce_step hands
// the running state from lane to lane in point order instead (bit-exact).
//
// The 32-byte otsdb_partial {x, y, z, w} is the exchange format between
// chunks and between ranks (RCCL); pack/unpack map each state onto it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

namespace otsdb {

constexpr double kDoubleMax = 1.7976931348623157e308;

DEV bool is_nan(double v) { return v != v; }
DEV bool is_inf(double v) { return v == __builtin_inf() || v == -__builtin_inf(); }
DEV double qnan() { return __builtin_nan(""); }

// DPP lane movers (VALU, no LDS round trip).  CTRL is a DPP control word
// (row_shr:n = 0x110+n, row_bcast:15 = 0x142, row_bcast:31 = 0x143,
// wave_shr:1 = 0x138, wave_shl:1 = 0x130); lanes whose source is invalid or
// whose row is masked off keep their own value.
template <int CTRL, int RM>
DEV int32_t dpp32(int32_t x) {
  return __builtin_amdgcn_update_dpp(x, x, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM>
DEV int32_t dpp32(int32_t old, int32_t x) {
  return __builtin_amdgcn_update_dpp(old, x, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM>
DEV int64_t dpp64(int64_t x) {
  const int32_t lo = dpp32<CTRL, RM>((int32_t)(uint32_t)x);
  const int32_t hi = dpp32<CTRL, RM>((int32_t)(x >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int CTRL, int RM>
DEV double dppd(double x) {
  return __builtin_bit_cast(double, dpp64<CTRL, RM>(__builtin_bit_cast(int64_t, x)));
}

template <int CTRL, int RM> DEV double dppv(double x) { return dppd<CTRL, RM>(x); }
template <int CTRL, int RM> DEV int64_t dppv(int64_t x) { return dpp64<CTRL, RM>(x); }
template <int CTRL, int RM> DEV int32_t dppv(int32_t x) { return dpp32<CTRL, RM>(x); }

struct Packed {
  double x, y, z;
  int64_t w;
};

// ---------------------------------------------------------------- sum-like
// Sum/ZimSum/PfSum (Aggregators.java:231-262), Avg (:362-392),
// SquareSum (:264-295), Count (:620-647): (s, n) with NaN skipping.
template <int KIND>  // 0 sum, 1 avg, 2 squareSum, 3 count
struct MSum {
  static constexpr bool kOrdered = false;
  static constexpr bool kCostlyFinish = KIND == 1;  // s / n
  double s;
  int32_t n;
  DEV static MSum init() { return {0.0, 0}; }
  DEV static MSum from(double v) {
    if (is_nan(v)) return {0.0, 0};
    return {0.0 + (KIND == 2 ? v * v : v), 1};
  }
  DEV void push(double v) {
    if (!is_nan(v)) {
      s += (KIND == 2 ? v * v : v);
      ++n;
    }
  }
  DEV void push_if(bool mk, double v) {  // branch free; s is never -0.0
    const bool ok = mk & !is_nan(v);
    s += ok ? (KIND == 2 ? v * v : v) : 0.0;
    n += ok ? 1 : 0;
  }
  DEV static MSum combine(const MSum& a, const MSum& b) {
    return {a.s + b.s, a.n + b.n};
  }
  DEV double finish(int* err) const {
    if (KIND == 3) return (double)n;
    if (n == 0) return qnan();
    return KIND == 1 ? s / (double)(int32_t)n : s;
  }
  DEV Packed pack() const { return {s, 0.0, 0.0, n}; }
  DEV static MSum unpack(const Packed& p) { return {p.x, (int32_t)p.w}; }
  DEV void shfl_up(int d) {
    s = __shfl_up(s, d);
    n = __shfl_up(n, d);
  }
  template <int CTRL, int RM>
  DEV void dpp() {
    s = dppv<CTRL, RM>(s);
    n = dppv<CTRL, RM>(n);
  }
};

// ---------------------------------------------------------------- min/max
// Min/MimMin (:297-328), Max/MimMax (:330-360).
template <bool MAX>
struct MMinMax {
  static constexpr bool kOrdered = false;
  static constexpr bool kCostlyFinish = false;
  double m;
  DEV static MMinMax init() { return {MAX ? -__builtin_inf() : __builtin_inf()}; }
  DEV static MMinMax from(double v) {
    return {is_nan(v) ? (MAX ? -__builtin_inf() : __builtin_inf()) : v};
  }
  DEV void push(double v) {
    if (!is_nan(v) && (MAX ? v > m : v < m)) m = v;
  }
  DEV void push_if(bool mk, double v) {
    m = (mk & (MAX ? v > m : v < m)) ? v : m;  // NaN compares false
  }
  DEV static MMinMax combine(const MMinMax& a, const MMinMax& b) {
    return (MAX ? b.m > a.m : b.m < a.m) ? b : a;  // keeps the earliest
  }
  DEV double finish(int* err) const {
    return (m == (MAX ? -__builtin_inf() : __builtin_inf())) ? qnan() : m;
  }
  DEV Packed pack() const { return {m, 0.0, 0.0, 0}; }
  DEV static MMinMax unpack(const Packed& p) { return {p.x}; }
  DEV void shfl_up(int d) { m = __shfl_up(m, d); }
  template <int CTRL, int RM>
  DEV void dpp() { m = dppv<CTRL, RM>(m); }
};

// ---------------------------------------------------------------- dev
// StdDev.runDouble (:498-571): Welford from the first non-NaN value,
// population sigma; Chan et al. merge for runs.
struct MDev {
  static constexpr bool kOrdered = true;
  static constexpr bool kCostlyFinish = false;
  double mean, m2;
  int32_t n;
  DEV static MDev init() { return {0.0, 0.0, 0}; }
  DEV static MDev from(double v) {
    if (is_nan(v)) return {0.0, 0.0, 0};
    return {v, 0.0, 1};
  }
  DEV void push(double x) {
    if (is_nan(x)) return;
    if (n == 0) {
      mean = x;
      n = 1;
      return;
    }
    ++n;
    const double new_mean = mean + (x - mean) / (double)n;
    m2 += (x - mean) * (x - new_mean);
    mean = new_mean;
  }
  DEV void push_if(bool mk, double x) {
    if (mk) push(x);
  }
  DEV static MDev combine(const MDev& a, const MDev& b) {
    if (a.n == 0) return b;
    if (b.n == 0) return a;
    const int64_t n = a.n + b.n;
    const double delta = b.mean - a.mean;
    const double dn = (double)n;
    MDev r;
    r.n = n;
    r.mean = a.mean + delta * ((double)b.n / dn);
    r.m2 = a.m2 + b.m2 + delta * delta * ((double)a.n * (double)b.n / dn);
    return r;
  }
  DEV double finish(int* err) const {
    if (n == 0) return qnan();
    if (n == 1) return 0.0;
    return __builtin_sqrt(m2 / (double)n);
  }
  DEV Packed pack() const { return {mean, m2, 0.0, n}; }
  DEV static MDev unpack(const Packed& p) { return {p.x, p.y, (int32_t)p.w}; }
  DEV void shfl_up(int d) {
    mean = __shfl_up(mean, d);
    m2 = __shfl_up(m2, d);
    n = __shfl_up(n, d);
  }
  template <int CTRL, int RM>
  DEV void dpp() {
    mean = dppv<CTRL, RM>(mean);
    m2 = dppv<CTRL, RM>(m2);
    n = dppv<CTRL, RM>(n);
  }
};

// ---------------------------------------------------------------- first/last
// First (:810-829), Last (:831-852): NaN is NOT skipped.
template <bool LAST>
struct MFirstLast {
  static constexpr bool kOrdered = false;
  static constexpr bool kCostlyFinish = false;
  double v;
  int64_t has;
  DEV static MFirstLast init() { return {0.0, 0}; }
  DEV static MFirstLast from(double x) { return {x, 1}; }
  DEV void push(double x) {
    if (LAST || !has) v = x;
    has = 1;
  }
  DEV void push_if(bool mk, double x) {
    if (mk) push(x);
  }
  DEV static MFirstLast combine(const MFirstLast& a, const MFirstLast& b) {
    if (LAST) return b.has ? b : a;
    return a.has ? a : b;
  }
  DEV double finish(int* err) const { return v; }
  DEV Packed pack() const { return {v, 0.0, 0.0, has}; }
  DEV static MFirstLast unpack(const Packed& p) { return {p.x, p.w}; }
  DEV void shfl_up(int d) {
    v = __shfl_up(v, d);
    has = __shfl_up(has, d);
  }
  template <int CTRL, int RM>
  DEV void dpp() {
    v = dppv<CTRL, RM>(v);
    has = dppv<CTRL, RM>(has);
  }
};

// ---------------------------------------------------------------- mult
// Multiply.runDouble (:476-484): product of every value, NaN included.
struct MMult {
  static constexpr bool kOrdered = false;
  static constexpr bool kCostlyFinish = false;
  double p;
  int64_t has;
  DEV static MMult init() { return {1.0, 0}; }
  DEV static MMult from(double x) { return {x, 1}; }
  DEV void push(double x) {
    p = has ? p * x : x;
    has = 1;
  }
  DEV void push_if(bool mk, double x) {
    if (mk) push(x);
  }
  DEV static MMult combine(const MMult& a, const MMult& b) {
    if (!a.has) return b;
    if (!b.has) return a;
    return {a.p * b.p, 1};
  }
  DEV double finish(int* err) const { return p; }
  DEV Packed pack() const { return {p, 0.0, 0.0, has}; }
  DEV static MMult unpack(const Packed& p) { return {p.x, p.w}; }
  DEV void shfl_up(int d) {
    p = __shfl_up(p, d);
    has = __shfl_up(has, d);
  }
  template <int CTRL, int RM>
  DEV void dpp() {
    p = dppv<CTRL, RM>(p);
    has = dppv<CTRL, RM>(has);
  }
};

// ---------------------------------------------------------------- diff
// Diff.runDouble (:598-618): last value minus the first non-NaN value;
// 0 when the first non-NaN value is the last value.
struct MDiff {
  static constexpr bool kOrdered = false;
  static constexpr bool kCostlyFinish = false;
  double fnn, last;
  int64_t flags;  // bit0 has_any, bit1 has_fnn, bit2 has_after_fnn
  DEV static MDiff init() { return {0.0, 0.0, 0}; }
  DEV static MDiff from(double x) {
    MDiff r{0.0, x, 1};
    if (!is_nan(x)) {
      r.fnn = x;
      r.flags |= 2;
    }
    return r;
  }
  DEV void push(double x) { *this = combine(*this, from(x)); }
  DEV void push_if(bool mk, double x) {
    if (mk) push(x);
  }
  DEV static MDiff combine(const MDiff& a, const MDiff& b) {
    if (!(a.flags & 1)) return b;
    if (!(b.flags & 1)) return a;
    MDiff r;
    r.last = b.last;
    if (a.flags & 2) {
      r.fnn = a.fnn;
      r.flags = 1 | 2 | 4;
    } else {
      r.fnn = b.fnn;
      r.flags = 1 | (b.flags & 6);
    }
    return r;
  }
  DEV double finish(int* err) const {
    if (!(flags & 2)) return qnan();
    if (!(flags & 4)) return 0.0;
    return last - fnn;
  }
  DEV Packed pack() const { return {fnn, last, 0.0, flags}; }
  DEV static MDiff unpack(const Packed& p) { return {p.x, p.y, p.w}; }
  DEV void shfl_up(int d) {
    fnn = __shfl_up(fnn, d);
    last = __shfl_up(last, d);
    flags = __shfl_up(flags, d);
  }
  template <int CTRL, int RM>
  DEV void dpp() {
    fnn = dppv<CTRL, RM>(fnn);
    last = dppv<CTRL, RM>(last);
    flags = dppv<CTRL, RM>(flags);
  }
};

// ---------------------------------------------------------------- none
// None.runDouble (:439-461): exactly one value, else IllegalDataException.
struct MNone {
  static constexpr bool kOrdered = false;
  static constexpr bool kCostlyFinish = false;
  double v;
  int32_t n;
  DEV static MNone init() { return {0.0, 0}; }
  DEV static MNone from(double x) { return {x, 1}; }
  DEV void push(double x) {
    if (n == 0) v = x;
    ++n;
  }
  DEV void push_if(bool mk, double x) {
    if (mk) push(x);
  }
  DEV static MNone combine(const MNone& a, const MNone& b) {
    return {a.n ? a.v : b.v, a.n + b.n};
  }
  DEV double finish(int* err) const {
    if (n > 1) *err |= 1;  // E_ILLEGAL_DATA
    return v;
  }
  DEV Packed pack() const { return {v, 0.0, 0.0, n}; }
  DEV static MNone unpack(const Packed& p) { return {p.x, (int32_t)p.w}; }
  DEV void shfl_up(int d) {
    v = __shfl_up(v, d);
    n = __shfl_up(n, d);
  }
  template <int CTRL, int RM>
  DEV void dpp() {
    v = dppv<CTRL, RM>(v);
    n = dppv<CTRL, RM>(n);
  }
};

}  // namespace otsdb
