// decode.hip — compacted RowSeq columns -> columnar (ts, value, is_float).
//
// RowSeq.Iterator (RowSeq.java:552-643) walks a compacted column qualifier by
// qualifier: a qualifier whose first byte has the 0xF0 flag nibble is a
// 4-byte millisecond qualifier (Internal.inMilliseconds, Internal.java:621),
// otherwise a 2-byte seconds qualifier; the low 4 bits are the flags
// (0x8 float, 0x7 value length - 1) and the value cursor advances by the
// value length.  Because qualifier widths can mix inside a row
// (Const.MS_MIXED_COMPACT), where each qualifier starts is a sequential
// property; on the GPU it is a wave scan over 2-byte units of the boolean
// recurrence  start(u+1) = !(start(u) && ms(u))  (composition of maps
// {0,1} -> {0,1}), followed by a scan of value lengths.  One wavefront per
// row.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"
#include "launch.h"

namespace otsdb {


enum : int { ERR_CORRUPT_CELL = 1 << 21 };  // (16 is ERR_X1_MASK)

// map {0,1}->{0,1} as 2 bits: bit0 = f(0), bit1 = f(1)
DEV int fmap_apply(int f, int s) { return (f >> s) & 1; }
DEV int fmap_compose(int g, int f) {  // g o f
  return fmap_apply(g, f & 1) | (fmap_apply(g, (f >> 1) & 1) << 1);
}

// The first vl (1..8) bytes at a, big-endian, from two aligned 8-byte loads
// (values sit at any byte offset: one meta byte per multi-value column);
// byte loads within 16 bytes of the end of the value buffer.
DEV uint64_t load_be(const uint8_t* base, int64_t a, int vl, int64_t vend) {
  const int64_t al = a & ~(int64_t)7;
  uint64_t w;
  if (((uintptr_t)base & 7) == 0 && al + 16 <= vend) {
    const uint64_t lo = *reinterpret_cast<const uint64_t*>(base + al);
    const uint64_t hi = *reinterpret_cast<const uint64_t*>(base + al + 8);
    const int sh = (int)(a - al) * 8;
    w = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;  // bytes a.. a+7, LE
  } else {
    w = 0;
    for (int i = 0; i < vl; ++i) w |= (uint64_t)base[a + i] << (8 * i);
  }
  return __builtin_bswap64(w) >> (64 - 8 * vl);
}

// RowSeq value bits of a point: big-endian signed 1/2/4/8-byte longs
// (RowSeq.java:233-245), 4-byte floats widened, 8-byte doubles (:256-266)
DEV int64_t value_bits(uint64_t x, int vl, int fl) {
  if (fl) return vl == 4 ? __double_as_longlong((double)__uint_as_float((uint32_t)x))
                         : (int64_t)x;
  switch (vl) {
    case 1: return (int8_t)x;
    case 2: return (int16_t)x;
    case 4: return (int32_t)x;
    default: return (int64_t)x;
  }
}

// exclusive wave prefix sum of x; total = the wave's sum.  DPP row shifts
// and row broadcasts (VALU only, no LDS round trips); lanes without a
// source add 0
DEV int wave_excl_scan(int x, int& total) {
  int incl = x;
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xF, 0xF, false);  // row_shr:1
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xF, 0xF, false);  // row_shr:2
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xF, 0xF, false);  // row_shr:4
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xF, 0xF, false);  // row_shr:8
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xA, 0xF, false);  // row_bcast:15
  incl += __builtin_amdgcn_update_dpp(0, incl, 0x143, 0xC, 0xF, false);  // row_bcast:31
  total = __builtin_amdgcn_readlane(incl, 63);
  return incl - x;
}

// Fast path of one column whose qualifiers all have the width of the first
// (the common case: no MS_MIXED_COMPACT) — point i's qualifier is at
// qw * i, no start-recurrence scan — and, for the write, whose values all
// have one length (point i's value at vl * i).  Same checks and results as
// the generic walk below; returns false (nothing done) when the column is
// not uniform.  mode 0: count + validate, records uniformity in fast[r];
// mode 1: writes.
DEV bool decode_uniform(const CellsDev& C, int64_t r, int mode,
                        const uint8_t* q, int64_t qlen, int64_t vbase,
                        int64_t vlen, int64_t base_ms, int64_t* row_count,
                        const int64_t* row_out, uint8_t* fast, int64_t cap,
                        int64_t* ts, int64_t* val, uint8_t* isf, int& bad) {
  const int lane = LANE;
  if (mode == 1 && fast[r] != 1) return false;
  const int qw = ((q[0] & 0xF0) == 0xF0) ? 4 : 2;
  if (qlen % qw || ((uintptr_t)q & 1)) return false;
  const int64_t n = qlen / qw;
  auto qual_at = [&](int64_t i) -> uint32_t {
    const uint16_t* h = reinterpret_cast<const uint16_t*>(q + qw * i);
    const uint32_t a = __builtin_bswap16(h[0]);
    return qw == 2 ? a : (a << 16) | __builtin_bswap16(h[1]);
  };
  if (mode == 0) {
    const int v0 = (int)(qual_at(0) & 0x7) + 1;  // same address: broadcast
    int consistent = 1, diff = 0;
    int64_t vsum = 0;
    for (int64_t i0 = 0; i0 < n; i0 += 64) {
      const int64_t i = i0 + lane;
      if (i < n) {
        const uint32_t qv = qual_at(i);
        const int mk = (((qv >> (qw == 2 ? 8 : 24)) & 0xF0) == 0xF0);
        consistent &= (qw == 4) == (mk != 0);
        const int vl = (int)(qv & 0x7) + 1;
        if (qv & 0x8) bad |= !(vl == 4 || vl == 8);
        else bad |= !(vl == 1 || vl == 2 || vl == 4 || vl == 8);
        diff |= vl != v0;
        vsum += vl;
      }
    }
    if (__ballot(!consistent)) return false;
    for (int d = 32; d >= 1; d >>= 1) vsum += __shfl_xor(vsum, d);
    const int64_t meta = n > 1 ? 1 : 0;
    if (vsum + meta != vlen) bad = 1;
    const bool one_len = __ballot(diff) == 0;  // every lane votes
    if (lane == 0) {
      row_count[r] = n;
      fast[r] = one_len ? 1 : 0;
    }
    return true;
  }
  // mode 1, one value length
  const int vl = (int)(qual_at(0) & 0x7) + 1;
  const int64_t vend = C.val_off[C.R];
  const int64_t out0 = row_out[r];
  for (int64_t i0 = 0; i0 < n; i0 += 64) {
    const int64_t i = i0 + lane;
    if (i >= n) break;
    const uint32_t qv = qual_at(i);
    const int64_t o = out0 + i;
    if (o >= cap) continue;
    const int fl = (qv & 0x8) != 0;
    const uint64_t x = load_be(C.val, vbase + vl * i, vl, vend);
    ts[o] = qw == 4 ? base_ms + (int64_t)((qv & 0x0FFFFFC0u) >> 6)
                    : base_ms + (int64_t)((qv & 0xFFFFu) >> 4) * 1000;
    val[o] = value_bits(x, vl, fl);
    isf[o] = (uint8_t)fl;
  }
  return true;
}

// one wavefront per row; mode 0 counts (and validates), mode 1 writes
#ifndef OTSDB_DS_TU
// fast[r]: 1 = one qualifier width and one value length (k_decode writes
// by direct indexing); 0 = one width, lengths mixed (counted by k_decode,
// written by k_decode_generic); 2 = widths mixed (k_decode_generic counts
// and writes).  flags[0] / flags[1]: some row is 2 / some data row is not 1
// (plain stores of 1: the engine launches k_decode_generic only then, so the
// common batch keeps k_decode's small register footprint).
__global__ __launch_bounds__(256) void k_decode(
    CellsDev C, int mode, int64_t* __restrict__ row_count,
    const int64_t* __restrict__ row_out, uint8_t* __restrict__ fast,
    int64_t cap, int64_t* __restrict__ ts, int64_t* __restrict__ val,
    uint8_t* __restrict__ isf, int* err_word, int* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= C.R) return;
  const uint8_t* q = C.qual + C.qual_off[r];
  const int64_t qlen = C.qual_off[r + 1] - C.qual_off[r];
  const uint8_t* v = C.val + C.val_off[r];
  const int64_t vlen = C.val_off[r + 1] - C.val_off[r];
  const int64_t base_ms = C.row_base_s[r] * 1000;
  if (qlen & 1) {  // not a data-point column (Internal.java:262-264)
    if (mode == 0 && lane == 0) {
      row_count[r] = 0;
      fast[r] = 1;  // nothing to write
    }
    return;
  }
  // a multi-value column whose meta byte says seconds and ms are mixed
  // (RowSeq.java:338-356) goes straight to the generic walk (the flag only
  // steers; the walk validates either way)
  if (qlen > 0 && !(qlen > 4 && vlen > 0 && (v[vlen - 1] & 1))) {
    int fbad = 0;
    if (decode_uniform(C, r, mode, q, qlen, C.val_off[r], vlen, base_ms,
                       row_count, row_out, fast, cap, ts, val, isf, fbad)) {
      if (__ballot(fbad) && lane == 0) atomicOr(err_word, ERR_CORRUPT_CELL);
      if (mode == 0 && lane == 0 && !fast[r]) flags[1] = 1;
      return;
    }
  }
  if (mode == 0 && lane == 0) {
    fast[r] = 2;
    flags[0] = 1;
    flags[1] = 1;
  }
}

// The generic walk (rows k_decode left to it, see fast[] above): mode 0
// counts and validates the rows of mixed qualifier widths, mode 1 writes
// every row not written by k_decode.  One wavefront per row.
__global__ __launch_bounds__(256) void k_decode_generic(
    CellsDev C, int mode, int64_t* __restrict__ row_count,
    const int64_t* __restrict__ row_out, const uint8_t* __restrict__ fast,
    int64_t cap, int64_t* __restrict__ ts, int64_t* __restrict__ val,
    uint8_t* __restrict__ isf, int* err_word) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= C.R) return;
  const uint8_t fr = fast[r];
  if (mode == 0 ? fr != 2 : fr == 1) return;
  const uint8_t* q = C.qual + C.qual_off[r];
  const int64_t qlen = C.qual_off[r + 1] - C.qual_off[r];
  const int64_t vlen = C.val_off[r + 1] - C.val_off[r];
  const int64_t base_ms = C.row_base_s[r] * 1000;
  // Generic column (qualifier widths mixed, MS_MIXED_COMPACT): 8 two-byte
  // units per lane, 512 per pass.  Each lane composes its units' maps
  // start(u+1) = !(start(u) && ms(u)) sequentially, one wave scan of the
  // lanes' maps gives every lane its entry state, the lane then walks its
  // units; point counts and value offsets are lane prefix sums + wave scans.
  const int64_t units = qlen >> 1;
  const int64_t vend = C.val_off[C.R];
  const int64_t vb0 = C.val_off[r];
  int carry_start = 1;
  int32_t carry_n = 0;
  int64_t carry_voff = 0;
  int bad = 0;
  const int64_t out0 = mode ? row_out[r] : 0;
  constexpr int GU = 8;  // two-byte units per lane, 512 a pass (16 — a
                        // 360-point mixed row in one pass — measured
                        // slower: 162 vs 140 ms for C2's mixed cells)
  for (int64_t u0 = 0; u0 < units; u0 += 64 * GU) {
    const int64_t ub = u0 + GU * lane;
    const int nu = ub >= units ? 0 : (int)(units - ub < GU ? units - ub : GU);
    // the lane's 2*GU bytes and the 4 after them (a 4-byte qualifier may
    // start at the lane's last unit)
    uint32_t w[GU / 2 + 1];
#pragma unroll
    for (int i = 0; i <= GU / 2; ++i) w[i] = 0;
    if (2 * ub + 2 * GU + 4 <= qlen) {
#pragma unroll
      for (int i = 0; i < GU / 8; ++i) {
        const uint4 x = *reinterpret_cast<const uint4*>(q + 2 * ub + 16 * i);
        w[4 * i] = x.x; w[4 * i + 1] = x.y; w[4 * i + 2] = x.z; w[4 * i + 3] = x.w;
      }
      w[GU / 2] = *reinterpret_cast<const uint32_t*>(q + 2 * ub + 2 * GU);
    } else if (nu > 0) {
      for (int i = 0; i < 2 * GU + 4; ++i)
        if (2 * ub + i < qlen) w[i >> 2] |= (uint32_t)q[2 * ub + i] << (8 * (i & 3));
    }
    auto byte_at = [&](int k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu; };
    int F = 0x2;  // identity
    uint32_t msb = 0;
#pragma unroll
    for (int i = 0; i < GU; ++i) {
      const int ms = i < nu && (byte_at(2 * i) & 0xF0) == 0xF0;
      msb |= (uint32_t)ms << i;
      if (i < nu) F = fmap_compose(ms ? 0x1 : 0x3, F);
    }
    int G = F;  // inclusive composition over the lanes
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int g = __shfl_up(G, d);
      if (lane >= d) G = fmap_compose(G, g);
    }
    int Gex = __shfl_up(G, 1);
    if (lane == 0) Gex = 0x2;
    int st = fmap_apply(Gex, carry_start);
    // the lane's points: starts, qualifiers, value lengths
    uint32_t startm = 0;
    int np = 0, vs = 0;
#pragma unroll
    for (int i = 0; i < GU; ++i) {
      if (i < nu && st) {
        startm |= 1u << i;
        const int ms = (msb >> i) & 1;
        if (ms && ub + i + 1 >= units) bad = 1;  // cut by the column end
        const uint32_t qv =
            ms ? (byte_at(2 * i) << 24) | (byte_at(2 * i + 1) << 16) |
                     (byte_at(2 * i + 2) << 8) | byte_at(2 * i + 3)
               : (byte_at(2 * i) << 8) | byte_at(2 * i + 1);
        const int vl = (int)(qv & 0x7) + 1;
        if (qv & 0x8) bad |= !(vl == 4 || vl == 8);
        else bad |= !(vl == 1 || vl == 2 || vl == 4 || vl == 8);
        ++np;
        vs += vl;
      }
      if (i < nu) st = !(st && ((msb >> i) & 1));
    }
    int tn, tv;
    const int np_ex = wave_excl_scan(np, tn);
    const int vs_ex = wave_excl_scan(vs, tv);
    if (mode == 1 || vs > 0) {
      int k = 0, vo = 0;
#pragma unroll
      for (int i = 0; i < GU; ++i) {
        if ((startm >> i) & 1) {
          const int ms = (msb >> i) & 1;
          const uint32_t qv =
              ms ? (byte_at(2 * i) << 24) | (byte_at(2 * i + 1) << 16) |
                       (byte_at(2 * i + 2) << 8) | byte_at(2 * i + 3)
                 : (byte_at(2 * i) << 8) | byte_at(2 * i + 1);
          const int vl = (int)(qv & 0x7) + 1;
          const int64_t voff = carry_voff + vs_ex + vo;
          if (voff + vl > vlen) bad = 1;
          if (mode == 1 && !bad) {
            const int64_t o = out0 + carry_n + np_ex + k;
            if (o < cap) {
              const int64_t a = vb0 + voff;
              uint64_t x;
              if (a + 8 <= vend) {
                x = __builtin_bswap64(*reinterpret_cast<const uint64_t*>(C.val + a));
              } else {
                x = 0;
                for (int b = 0; b < 8; ++b)
                  x = (x << 8) | (a + b < vend ? (uint64_t)C.val[a + b] : 0);
              }
              x >>= 64 - 8 * vl;
              const int fl = (qv & 0x8) != 0;
              ts[o] = ms ? base_ms + (int64_t)((qv & 0x0FFFFFC0u) >> 6)
                         : base_ms + (int64_t)((qv & 0xFFFFu) >> 4) * 1000;
              val[o] = value_bits(x, vl, fl);
              isf[o] = (uint8_t)fl;
            }
          }
          ++k;
          vo += vl;
        }
      }
    }
    carry_n += tn;
    carry_voff += tv;
    carry_start = fmap_apply(__shfl(G, 63), carry_start);
  }
  if (mode == 0) {
    // all value bytes consumed, the meta byte of multi-value columns aside
    // (Internal.java:316-321)
    const int64_t meta = carry_n > 1 ? 1 : 0;
    if (carry_voff + meta != vlen) bad = 1;
    if (lane == 0) row_count[r] = carry_n;
  }
  if (__ballot(bad) && lane == 0) atomicOr(err_word, ERR_CORRUPT_CELL);
}
#endif  // OTSDB_DS_TU

// ------------------------------------------------------------------------
// k_encode: the inverse — columnar series -> compacted RowSeq columns, the
// layout the write path + compaction produce (test/bench infrastructure, the
// device twin of tests/cells.py): one row per (series, hour), a 2-byte
// qualifier for whole-second offsets and a 4-byte ms qualifier otherwise
// (Internal.buildQualifier, Internal.java:848-863), doubles as 8 bytes, longs
// in the smallest of 1/2/4/8 bytes (TSDB.addPoint, TSDB.java:1051-1147), and
// the trailing meta byte (bit0 = mixed s/ms) on multi-value columns
// (CompactionQueue.buildCompactedColumn, CompactionQueue.java:594-616).
// One wavefront per series; rows are runs of consecutive points with the
// same hour, so every offset is a prefix sum inside the series (64-bit
// masks for the in-chunk parts, carries across chunks).  mode 0 counts
// rows / qualifier bytes / value bytes per series, mode 1 writes them at
// the per-series bases the caller scanned.
#ifndef OTSDB_DS_TU
// ------------------------------------------------------------------------
DEV int enc_long_len(int64_t v) {
  if (v >= -128 && v <= 127) return 1;
  if (v >= -32768 && v <= 32767) return 2;
  if (v >= INT32_MIN && v <= INT32_MAX) return 4;
  return 8;
}

// lanes [a, b] (a <= b) of a 64-bit mask
DEV uint64_t lane_range(int a, int b) {
  const uint64_t hi = b >= 63 ? ~0ULL : ((1ULL << (b + 1)) - 1);
  return hi & ~((1ULL << a) - 1);
}

__global__ __launch_bounds__(256) void k_encode(
    int64_t S, const int64_t* __restrict__ offsets,
    const int64_t* __restrict__ ts, const int64_t* __restrict__ val,
    const uint8_t* __restrict__ series_float, int mode,
    int64_t* __restrict__ s_rows, int64_t* __restrict__ s_qb,
    int64_t* __restrict__ s_vb, int64_t* __restrict__ row_series,
    int64_t* __restrict__ row_base_s, int64_t* __restrict__ qual_off,
    int64_t* __restrict__ val_off, uint8_t* __restrict__ qual,
    uint8_t* __restrict__ vbytes) {
  const int lane = LANE;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= S) return;
  const int64_t p0 = offsets[s], p1 = offsets[s + 1];
  const int fl = series_float ? (int)series_float[s] : 1;
  int64_t row = mode ? s_rows[s] : 0, qo = mode ? s_qb[s] : 0,
          vo = mode ? s_vb[s] : 0;
  const int64_t row0 = row, qo0 = qo, vo0 = vo;
  // the row open at the chunk start: its start is before the chunk
  int64_t prev_hour = INT64_MIN;
  int carry_ms = 0, carry_s = 0;  // the open row has 4- / 2-byte qualifiers
  for (int64_t c0 = p0; c0 < p1; c0 += 64) {
    const int64_t p = c0 + lane;
    const bool in = p < p1;
    const int64_t t = in ? ts[p] : 0;
    const int64_t v = in ? val[p] : 0;
    const int64_t sec = t / 1000;
    const int64_t hour = sec - sec % 3600;
    const int64_t off_ms = t - hour * 1000;
    const int ms = in && (off_ms % 1000 != 0);
    const int qlen = in ? (ms ? 4 : 2) : 0;
    const int vlen = in ? (fl ? 8 : enc_long_len(v)) : 0;
    int64_t ph = __shfl_up(hour, 1);
    if (lane == 0) ph = prev_hour;
    const bool rs = in && hour != ph;            // row starts here
    const int64_t nh = __shfl_down(hour, 1);
    const bool next_in = (p + 1 < p1);
    const bool re = in && (!next_in || (lane < 63 ? nh != hour
                                                  : ts[p + 1] / 1000 -
                                                        (ts[p + 1] / 1000) % 3600 !=
                                                        hour));
    const uint64_t rsm = __ballot(rs), msm = __ballot(ms), inm = __ballot(in);
    // this lane's row inside the chunk: from its start lane (or the chunk
    // start when the row began earlier) to here
    const uint64_t below = rsm & lane_range(0, lane);
    const int st_l = below ? 63 - __builtin_clzll(below) : -1;
    const int a = st_l >= 0 ? st_l : 0;
    const uint64_t span = lane_range(a, lane) & inm;
    const bool open_row = st_l < 0;  // continues the row of the last chunk
    const int any_ms = ((msm & span) != 0) || (open_row && carry_ms);
    const int any_s = ((~msm & span) != 0) || (open_row && carry_s);
    // a row has more than one point iff its end is not also its start, or
    // it continues from the previous chunk
    const bool single = rs && re;
    const int meta = (re && !single) ? 1 : 0;
    // prefix sums of qualifier and value bytes (meta bytes included)
    int qe = qlen, ve = vlen + meta;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(qe, d), z = __shfl_up(ve, d);
      if (lane >= d) {
        qe += y;
        ve += z;
      }
    }
    const int64_t q_at = qo + qe - qlen;
    const int64_t v_at = vo + ve - vlen - meta;
    const int64_t r_at = row + __popcll(rsm & ((1ULL << lane) - 1));
    if (mode == 1 && in) {
      const int flags = fl ? (0x8 | 7) : (vlen - 1);
      if (ms) {
        const uint32_t q = 0xF0000000u | ((uint32_t)off_ms << 6) | (uint32_t)flags;
        qual[q_at] = (uint8_t)(q >> 24);
        qual[q_at + 1] = (uint8_t)(q >> 16);
        qual[q_at + 2] = (uint8_t)(q >> 8);
        qual[q_at + 3] = (uint8_t)q;
      } else {
        const uint32_t q = ((uint32_t)(off_ms / 1000) << 4) | (uint32_t)flags;
        qual[q_at] = (uint8_t)(q >> 8);
        qual[q_at + 1] = (uint8_t)q;
      }
      const uint64_t x = (uint64_t)v;  // doubles: their bits; longs: two's
      for (int i = 0; i < vlen; ++i)
        vbytes[v_at + i] = (uint8_t)(x >> (8 * (vlen - 1 - i)));
      if (meta) vbytes[v_at + vlen] = (any_ms && any_s) ? 1 : 0;
      if (rs) {
        row_series[r_at] = s;
        row_base_s[r_at] = hour;
        qual_off[r_at] = q_at;
        val_off[r_at] = v_at;
      }
    }
    // carries: the row open at the chunk end
    const int last = 63 - __builtin_clzll(inm);
    const uint64_t lb = rsm & lane_range(0, last);
    const int ls = lb ? 63 - __builtin_clzll(lb) : -1;
    const uint64_t tail = lane_range(ls >= 0 ? ls : 0, last) & inm;
    const int tail_ms = (msm & tail) != 0, tail_s = (~msm & tail) != 0;
    if (ls >= 0) {
      carry_ms = tail_ms;
      carry_s = tail_s;
    } else {
      carry_ms |= tail_ms;
      carry_s |= tail_s;
    }
    prev_hour = __shfl(hour, last);
    row += __popcll(rsm);
    qo += __shfl(qe, last);
    vo += __shfl(ve, last);
  }
  if (mode == 0 && lane == 0) {
    s_rows[s] = row - row0;
    s_qb[s] = qo - qo0;
    s_vb[s] = vo - vo0;
  }
}
#endif  // OTSDB_DS_TU

// ------------------------------------------------------------------------
// k_bucketize_cells: decode fused into the downsample.
// One wavefront per series walks its compacted columns in row order and
// feeds the decoded points straight into k_bucketize_k's reduction
// (reduce_step): the compacted bytes (10 B / point for seconds + doubles)
// are read once and no columnar copy is written.  Each step of 64*K points
// stages the step's qualifier bytes, then its value bytes, through the
// wave's LDS with aligned 16-byte loads (the columns sit at any byte offset
// and a lane's values are 8 bytes apart: direct loads would touch eight
// times the cache lines); values may have any legal length per point (long
// counters are stored in 1/2/4/8 bytes) — their offsets are a wave prefix
// sum of the lengths.  What k_prep derives from columnar timestamps is
// derived from the cells: the SpanGroup.add filter from the series' first
// and last point, the seek / stop window per step, and the first bucket
// past the window (lane 0 walks its points in order, as k_prep does).
// Closed buckets go straight to the row with their state byte.  Columns
// must have one qualifier width (no MS_MIXED_COMPACT; the write path emits
// one per resolution): a series holding a mixed column raises
// ERR_CELLS_GENERIC and the host decodes instead.  Corrupt columns (illegal
// value lengths, value bytes that do not add up) raise ERR_CORRUPT_CELL
// (Internal.extractDataPoints, Internal.java:307-321).
// ------------------------------------------------------------------------
enum : int { ERR_CELLS_GENERIC = 1 << 20 };
// the uniform cells fold (fold_member_cells_u) met a qualifier whose flags
// are not its series' one: the engine runs the batch's fold again with the
// general kernel (which decodes mixed value lengths point by point)
enum : int { ERR_CELLS_NONUNI = 1 << 24 };

struct CellRow {
  const uint8_t* q;
  int64_t n, vbase, vlen, base_ms;
  int qw;
  bool ok;
};

DEV CellRow cell_row(const CellsDev& C, int64_t r) {
  CellRow w;
  const int64_t qo = C.qual_off[r], qlen = C.qual_off[r + 1] - qo;
  w.q = C.qual + qo;
  w.vbase = C.val_off[r];
  w.vlen = C.val_off[r + 1] - w.vbase;
  w.base_ms = C.row_base_s[r] * 1000;
  w.qw = (qlen > 0 && (w.q[0] & 0xF0) == 0xF0) ? 4 : 2;
  w.n = qlen / w.qw;
  w.ok = qlen > 0 && qlen % w.qw == 0 && !((uintptr_t)w.q & 1);
  return w;
}

DEV uint32_t cell_qual(const CellRow& w, int64_t i) {
  const uint16_t* h = reinterpret_cast<const uint16_t*>(w.q + w.qw * i);
  const uint32_t a = __builtin_bswap16(h[0]);
  return w.qw == 2 ? a : (a << 16) | __builtin_bswap16(h[1]);
}

DEV int64_t qual_ts(int64_t base_ms, int qw, uint32_t qv) {
  return qw == 4 ? base_ms + (int64_t)((qv & 0x0FFFFFC0u) >> 6)
                 : base_ms + (int64_t)((qv & 0xFFFFu) >> 4) * 1000;
}

// the folded double of a value (RowSeq longValue/doubleValue -> toDouble,
// RowSeq.java:552-643)
DEV int64_t dbits_of(uint64_t x, int vl, int fl) {
  const int64_t bits = value_bits(x, vl, fl);
  return fl ? bits : __double_as_longlong((double)bits);
}

DEV void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// copies bytes [src, src + n) into lds with aligned 16-byte loads (whole
// 16-byte blocks around the range: never past a page); returns where src's
// first byte landed
DEV int stage16(uint8_t* lds, const uint8_t* src, int64_t n) {
  const uintptr_t a = (uintptr_t)src, al = a & ~(uintptr_t)15;
  const int sh = (int)(a - al);
  const int nch = (int)((sh + n + 15) >> 4);
  for (int c = LANE; c < nch; c += 64)
    *reinterpret_cast<uint4*>(lds + 16 * c) =
        *reinterpret_cast<const uint4*>(al + 16 * (uintptr_t)c);
  wave_lds_fence();
  return sh;
}

DEV uint64_t lds_be(const uint8_t* lds, int o, int vl) {
  const int al = o & ~7;
  const uint64_t lo = *reinterpret_cast<const uint64_t*>(lds + al);
  const uint64_t hi = *reinterpret_cast<const uint64_t*>(lds + al + 8);
  const int sh = (o - al) * 8;
  const uint64_t w = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  return __builtin_bswap64(w) >> (64 - 8 * vl);
}

// Big-endian fields of W bytes each, N consecutive ones from LDS byte o on
// (o any byte offset; the lane's N*W bytes are read as whole dwords and the
// fields cut out with byte-align funnels)
template <int W, int N>
DEV void lds_be_run(const uint8_t* lds, int o, uint32_t* out) {
  constexpr int ND = (W * N + 3) / 4 + 1;
  const int a = o & ~3, sh = o & 3;
  uint32_t d[ND + 1];
#pragma unroll
  for (int i = 0; i < ND; ++i)
    d[i] = *reinterpret_cast<const uint32_t*>(lds + a + 4 * i);
  d[ND] = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int b = W * j;  // compile-time byte offset of field j
    // bytes sh + b .. : dword (b >> 2) + carry, shift ((b & 3) + sh) & 3
    const int r = (b & 3) + sh;
    const int i0 = b >> 2;
    const uint32_t lo = r >= 4 ? d[i0 + 1] : d[i0];
    const uint32_t hi = r >= 4 ? d[i0 + 2] : d[i0 + 1];
    const uint32_t x = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(r & 3));
    out[j] = W == 2 ? (((x & 0xFF) << 8) | ((x >> 8) & 0xFF))
                    : __builtin_bswap32(x);
  }
}

// N consecutive values of VL bytes (one length and type for all of them,
// fl: floating point) from LDS byte o on -> the folded double's bits
// (RowSeq extractIntegerValue / extractFloatingPointValue, toDouble)
template <int VL, int N, int FL>
DEV void lds_values(const uint8_t* lds, int o, int64_t* v) {
  constexpr int ND = (VL * N + 3) / 4 + 1;
  const int a = o & ~3;
  const uint32_t sh = (uint32_t)(o & 3);
  uint32_t d[ND + 1];
#pragma unroll
  for (int i = 0; i < ND; ++i)
    d[i] = *reinterpret_cast<const uint32_t*>(lds + a + 4 * i);
  d[ND] = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (VL == 8) {
      const uint32_t lo = __builtin_amdgcn_alignbyte(d[2 * j + 1], d[2 * j], sh);
      const uint32_t hi = __builtin_amdgcn_alignbyte(d[2 * j + 2], d[2 * j + 1], sh);
      const int64_t x = (int64_t)(((uint64_t)__builtin_bswap32(lo) << 32) |
                                  __builtin_bswap32(hi));
      v[j] = FL ? x : __double_as_longlong((double)x);
    } else if (VL == 4) {
      const uint32_t x = __builtin_bswap32(
          __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh));
      v[j] = __double_as_longlong(FL ? (double)__uint_as_float(x)
                                     : (double)(int32_t)x);
    } else {
      const int b = VL * j;
      const int r = (b & 3) + (int)sh;
      const int i0 = b >> 2;
      const uint32_t lo = r >= 4 ? d[i0 + 1] : d[i0];
      const uint32_t hi = r >= 4 ? d[i0 + 2] : d[i0 + 1];
      const uint32_t x = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(r & 3));
      const int32_t iv = VL == 2 ? (int32_t)(int16_t)(((x & 0xFF) << 8) | ((x >> 8) & 0xFF))
                                 : (int32_t)(int8_t)(x & 0xFF);
      v[j] = __double_as_longlong((double)iv);
    }
  }
}

#ifndef OTSDB_DS_TU
__global__ void k_series_rows(int64_t R, int64_t S,
                              const int64_t* __restrict__ row_series,
                              int64_t* __restrict__ series_row) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > R) return;
  const int64_t prev = r == 0 ? -1 : row_series[r - 1];
  const int64_t cur = r == R ? S : row_series[r];
  for (int64_t s = prev + 1; s <= cur && s <= S; ++s) series_row[s] = r;
}
#endif  // OTSDB_DS_TU

template <class M, int K, int WAVES = 1, int ABL = 0>
__global__ __launch_bounds__(256, WAVES) void k_bucketize_cells(
    Params P, CellsDev C, const int64_t* __restrict__ series_row, int64_t S,
    SeriesMeta SM, Rows R, int* err_word) {
  static_assert(K % 2 == 0, "K");
  constexpr int PTS = 64 * K;
  constexpr int QB = PTS * 4 + 32, VB = PTS * 8 + 64;
  // two buffers per wave: row r is read from one while row r + 1 lands in
  // the other (LDS-DMA, no VGPRs in flight)
  __shared__ __attribute__((aligned(16))) uint8_t lq_all[4][2][QB];
  __shared__ __attribute__((aligned(16))) uint8_t lv_all[4][2][VB];
  const int lane = LANE;
  const int wv = threadIdx.x >> 6;
  const int64_t s = (int64_t)blockIdx.x * 4 + wv;
  if (s >= S) return;
  const int64_t r0 = series_row[s], r1 = series_row[s + 1];
  auto meta = [&](bool keep, uint8_t of_has, int64_t of_ts, double of_val) {
    if (lane == 0) {
      SM.keep[s] = keep;
      SM.lo[s] = 0;
      SM.hi[s] = 0;
      SM.kf[s] = 0;
      SM.kl[s] = -1;
      SM.of_has[s] = of_has;
      SM.of_ts[s] = of_ts;
      SM.of_val[s] = of_val;
    }
  };
  // SpanGroup.add filter (SpanGroup.java:321-338) from the first and last
  // point of the series
  bool keep = r0 < r1;
  if (keep) {
    const CellRow a = cell_row(C, r0), z = cell_row(C, r1 - 1);
    if (!a.ok || !z.ok) {
      if (lane == 0) atomicOr(err_word, ERR_CELLS_GENERIC);
      meta(false, 0, 0, 0.0);
      return;
    }
    const int64_t t_first = qual_ts(a.base_ms, a.qw, cell_qual(a, 0));
    const int64_t t_last = qual_ts(z.base_ms, z.qw, cell_qual(z, z.n - 1));
    keep = t_first <= P.end_ms && t_last >= P.start_ms;
  }
  if (!keep) {
    meta(false, 0, 0, 0.0);
    return;
  }
  BatchDev Bd{0, nullptr, nullptr, nullptr, nullptr, nullptr};
  RowSink Sk{R.val + s * P.nb, R.state + s * P.nb, nullptr, 0, 1, 1, 0, 0};
  int err = 0, carry_key = INT32_MIN;
  M carry = M::init();
  int64_t stop_r = -1, stop_i = 0;  // first point at or past stop_ts
  int generic = 0, corrupt = 0;
  // a row fits the prefetch buffers when it has <= PTS points; its whole
  // qualifier and value byte ranges then go to LDS by DMA, issued while the
  // previous row is being reduced
  auto fits = [&](const CellRow& w) {
    return w.ok && w.n <= PTS && w.vlen + 16 <= VB && w.qw * w.n + 16 <= QB;
  };
  auto prefetch = [&](const CellRow& w, int buf) -> int {  // DMA instrs
    int k = 0;
    const uintptr_t qa = (uintptr_t)w.q, qal = qa & ~(uintptr_t)15;
    const int nq = (int)(((qa - qal) + w.qw * w.n + 15) >> 4);
    for (int c0 = 0; c0 < nq; c0 += 64, ++k)
      if (c0 + lane < nq)
        __builtin_amdgcn_global_load_lds(
            (const void*)(qal + 16 * (uintptr_t)(c0 + lane)),
            (void*)&lq_all[wv][buf][16 * c0], 16, 0, 0);
    const uintptr_t va = (uintptr_t)(C.val + w.vbase),
                    val_ = va & ~(uintptr_t)15;
    const int nvb = (int)(((va - val_) + w.vlen + 15) >> 4);
    for (int c0 = 0; c0 < nvb; c0 += 64, ++k)
      if (c0 + lane < nvb)
        __builtin_amdgcn_global_load_lds(
            (const void*)(val_ + 16 * (uintptr_t)(c0 + lane)),
            (void*)&lv_all[wv][buf][16 * c0], 16, 0, 0);
    return k;
  };
  // Row metadata (column offsets, base time, qualifier width) for 64 rows at
  // a time, one row per lane: one parallel load round trip per 64 rows
  // instead of two dependent ones (offsets, then the first qualifier byte)
  // in front of every row's prefetch.
  int64_t mb = INT64_MIN, m_qo = 0, m_vo = 0, m_bms = 0, m_ql = 0, m_vl = 0;
  int m_q0 = 0;
  auto row_at = [&](int64_t rr) -> CellRow {
    if (rr < mb || rr >= mb + 64) {  // wave-uniform
      mb = rr;
      const int64_t x = rr + lane;
      if (x < r1) {
        m_qo = C.qual_off[x];
        m_ql = C.qual_off[x + 1] - m_qo;
        m_vo = C.val_off[x];
        m_vl = C.val_off[x + 1] - m_vo;
        m_bms = C.row_base_s[x] * 1000;
        m_q0 = m_ql > 0 ? C.qual[m_qo] : 0;
      }
    }
    const int j = (int)(rr - mb);
    CellRow w;
    const int64_t qo = readlane_l(m_qo, j), qlen = readlane_l(m_ql, j);
    w.q = C.qual + qo;
    w.vbase = readlane_l(m_vo, j);
    w.vlen = readlane_l(m_vl, j);
    w.base_ms = readlane_l(m_bms, j);
    const int q0 = __builtin_amdgcn_readlane(m_q0, j);
    w.qw = (qlen > 0 && (q0 & 0xF0) == 0xF0) ? 4 : 2;
    w.n = qlen / w.qw;
    w.ok = qlen > 0 && qlen % w.qw == 0 && !((uintptr_t)w.q & 1);
    return w;
  };
  int64_t r = r0;
  while (r < r1 && row_at(r).base_ms + 3600000 <= P.seek_ts) ++r;
  int buf = 0;
  CellRow wn = r < r1 ? row_at(r) : CellRow{};
  if (r < r1 && fits(wn)) prefetch(wn, 0);
  for (; r < r1 && stop_r < 0; ++r, buf ^= 1) {
    const CellRow w = wn;
    if (!w.ok) {
      generic = 1;
      break;
    }
    const bool pre = fits(w);  // this row already sits in buffer buf
    int n_next = 0;
    if (r + 1 < r1) {
      wn = row_at(r + 1);
      if (fits(wn)) n_next = prefetch(wn, buf ^ 1);
    }
    uint8_t* lq = lq_all[wv][buf];
    uint8_t* lv = lv_all[wv][buf];
    if (pre) {
      wait_vmcnt(n_next);  // this row's DMA done, the next row's may fly
      wave_lds_fence();
    }
    int64_t vpos = 0;  // value bytes of the row consumed so far
    for (int64_t st0 = 0; st0 < w.n; st0 += PTS) {
      const int n_st = (int)(w.n - st0 < PTS ? w.n - st0 : PTS);
      // qualifiers of the step -> LDS -> K per lane
      const int sq = pre ? (int)((uintptr_t)w.q & 15)
                         : stage16(lq, w.q + w.qw * st0, (int64_t)w.qw * n_st);
      uint32_t qv[K];
      if (w.qw == 2) lds_be_run<2, K>(lq, sq + 2 * K * lane, qv);
      else lds_be_run<4, K>(lq, sq + 4 * K * lane, qv);
      // one flags nibble for every point of the step (what compaction of
      // one series' same-typed values writes) -> value length and type are
      // wave-uniform: no length scan, no per-point type dispatch
      const uint32_t f0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(qv[0] & 0xF));
      int vl[K], lsum = 0, odd = 0, bad = 0, mixed = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const int i = K * lane + j;
        vl[j] = 0;
        if (i < n_st) {
          const int mk = ((qv[j] >> (w.qw == 2 ? 8 : 24)) & 0xF0) == 0xF0;
          odd |= (w.qw == 4) != (mk != 0);
          mixed |= (qv[j] & 0xF) != f0;
          vl[j] = (int)(qv[j] & 0x7) + 1;
          lsum += vl[j];
        }
      }
      generic |= __ballot(odd) != 0;
      if (generic) break;
      const bool uni = __ballot(mixed) == 0;
      int64_t t[K], v[K];
      int step_bytes, sv;
      if (uni) {
        const int vlu = (int)(f0 & 0x7) + 1, flu = (f0 & 0x8) != 0;
        corrupt |= flu ? !(vlu == 4 || vlu == 8)
                       : !(vlu == 1 || vlu == 2 || vlu == 4 || vlu == 8);
        step_bytes = vlu * n_st;
        if (corrupt || vpos + step_bytes > w.vlen) {
          corrupt = 1;
          break;
        }
        sv = pre ? (int)((uintptr_t)(C.val + w.vbase) & 15)
                 : stage16(lv, C.val + w.vbase + vpos, step_bytes);
        const int o = sv + vlu * K * lane;
        switch (vlu + 16 * flu) {
          case 8 + 16: lds_values<8, K, 1>(lv, o, v); break;
          case 4 + 16: lds_values<4, K, 1>(lv, o, v); break;
          case 8: lds_values<8, K, 0>(lv, o, v); break;
          case 4: lds_values<4, K, 0>(lv, o, v); break;
          case 2: lds_values<2, K, 0>(lv, o, v); break;
          default: lds_values<1, K, 0>(lv, o, v); break;
        }
      } else {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          if (K * lane + j < n_st) {
            if (qv[j] & 0x8) bad |= !(vl[j] == 4 || vl[j] == 8);
            else bad |= !(vl[j] == 1 || vl[j] == 2 || vl[j] == 4 || vl[j] == 8);
          }
        }
        corrupt |= __ballot(bad) != 0;
        if (corrupt) break;
        // value offsets: exclusive wave scan of the lanes' byte counts
        int incl = lsum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int y = __shfl_up(incl, d);
          if (lane >= d) incl += y;
        }
        step_bytes = __shfl(incl, 63);
        if (vpos + step_bytes > w.vlen) {
          corrupt = 1;
          break;
        }
        sv = pre ? (int)((uintptr_t)(C.val + w.vbase) & 15)
                 : stage16(lv, C.val + w.vbase + vpos, step_bytes);
        int off = sv + incl - lsum;
#pragma unroll
        for (int j = 0; j < K; ++j) {
          v[j] = dbits_of(lds_be(lv, off, vl[j]), vl[j], (qv[j] & 0x8) != 0);
          off += vl[j];
        }
      }
      // the step's points are [lo, hi) in row indices (timestamps increase):
      // counted against the seek / stop bounds unless the whole row lies
      // inside them (offsets < 2^22 ms)
      const bool inside =
          w.base_ms >= P.seek_ts && w.base_ms + (1 << 22) <= P.stop_ts;
      // (points past n_st keep whatever the LDS held: reduce_step only
      // reads the step's [lo, hi))
      int lt_seek = 0, lt_stop = 0;
      if (w.qw == 2) {
#pragma unroll
        for (int j = 0; j < K; ++j)
          t[j] = w.base_ms + (int64_t)(((qv[j] & 0xFFFFu) >> 4) * 1000u);
      } else {
#pragma unroll
        for (int j = 0; j < K; ++j)
          t[j] = w.base_ms + (int64_t)((qv[j] & 0x0FFFFFC0u) >> 6);
      }
      if (!inside) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const bool in = K * lane + j < n_st;
          lt_seek += in && t[j] < P.seek_ts;
          lt_stop += in && t[j] < P.stop_ts;
        }
      }
      vpos += step_bytes;
      int sum_seek = 0, sum_stop = n_st;
      if (!inside) {
        sum_seek = lt_seek;
        sum_stop = lt_stop;
        for (int d = 32; d >= 1; d >>= 1) {
          sum_seek += __shfl_xor(sum_seek, d);
          sum_stop += __shfl_xor(sum_stop, d);
        }
      }
      const int64_t lo = st0 + sum_seek, hi = st0 + sum_stop;
      if (ABL == 1) {  // tuning ablation: decode only, no reduction
        int64_t x = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) x ^= t[j] + v[j];
        if (x == 42) Sk.rowv[0] = 1.0;
      } else if (hi > lo)
        reduce_step<M, K, 1>(P, Bd, 1, lo, hi, st0, st0 + (int64_t)K * lane,
                             t, v, Sk, err, carry_key, carry,
#ifdef OTSDB_CELLS_NOKEEP  // timing ablation (wrong across rows)
                             false);
#else
                             true);
#endif
      if (hi < st0 + n_st) {  // reached stop_ts inside this row
        stop_r = r;
        stop_i = hi;
        break;
      }
      // LDS reuse by the next step / row: every lane is done reading
      wave_lds_fence();
    }
    if (generic || corrupt) break;
    // every value byte of the column used, the meta byte aside
    if (stop_r < 0 && vpos + (w.n > 1 ? 1 : 0) != w.vlen) {
      corrupt = 1;
      break;
    }
  }
  // no LDS-DMA may still be landing when the wave (and its block's LDS)
  // goes away
  wait_vmcnt(0);
  if (generic || corrupt) {
    // a mixed column is parsed by the generic decode, which also judges
    // whether it is corrupt
    if (lane == 0)
      atomicOr(err_word, generic ? ERR_CELLS_GENERIC : ERR_CORRUPT_CELL);
    meta(false, 0, 0, 0.0);
    return;
  }
  if (carry_key >= 0 && carry_key < P.nb && lane == 0)
    Sk.put(carry_key, carry.finish(&err));
  // the first bucket past the window (k_prep's of_val): lane 0 folds its
  // points in order, across rows (NONE fill only, like k_prep)
  uint8_t of_has = 0;
  int64_t of_ts = 0;
  double of_val = 0.0;
  if (!P.run_all && P.fill == 0 && stop_r >= 0 && lane == 0) {
    CellRow w = cell_row(C, stop_r);
    // value offset of point stop_i: the lengths of the points before it
    int64_t voff = 0;
    for (int64_t i = 0; i < stop_i; ++i) voff += (cell_qual(w, i) & 0x7) + 1;
    const int64_t vend = C.val_off[C.R];
    const int64_t t = qual_ts(w.base_ms, w.qw, cell_qual(w, stop_i));
    int64_t e;
    bool ok = true;
    if (P.cal) {
      const int64_t k = cal_bucket(P, t);
      ok = k >= P.cal_lo && k + 1 < P.cal_n;
      of_ts = ok ? P.cal[k] : 0;
      e = ok ? P.cal[k + 1] : 0;
    } else {
      of_ts = align_ts(t, P.interval);
      e = of_ts + P.interval;
    }
    if (!ok) {
      atomicOr(err_word, ERR_CAL_RANGE);
    } else {
      int64_t r = stop_r, i = stop_i;
      // folds the points of [.., end) from (r, i) on, across rows; false
      // when the span has no point left
      auto fold_until = [&](int64_t end, double* out) -> bool {
        M st = M::init();
        bool any = false;
        while (r < r1) {
          if (i >= w.n) {
            if (++r >= r1) break;
            w = cell_row(C, r);
            if (!w.ok) {
              r = r1;
              break;
            }
            i = 0;
            voff = 0;
            continue;
          }
          const uint32_t q = cell_qual(w, i);
          if (qual_ts(w.base_ms, w.qw, q) >= end) break;
          const int l = (int)(q & 0x7) + 1;
          st.push(bits_to_double(dbits_of(
              load_be(C.val, w.vbase + voff, l, vend), l, (q & 0x8) != 0)));
          voff += l;
          ++i;
          any = true;
        }
        int e2 = 0;
        *out = st.finish(&e2);
        return any;
      };
      fold_until(e, &of_val);
      of_has = 1;
      if (P.rate) {  // kept rates past that bucket (k_prep's rates_beyond)
        auto next = [&](int64_t* tn, double* vn) -> bool {
          if (r >= r1 || i >= w.n) return false;
          const int64_t tt = qual_ts(w.base_ms, w.qw, cell_qual(w, i));
          int64_t bt, be;
          if (P.cal) {
            const int64_t k = cal_bucket(P, tt);
            if (k < P.cal_lo || k + 1 >= P.cal_n) return false;
            bt = P.cal[k];
            be = P.cal[k + 1];
          } else {
            bt = align_ts(tt, P.interval);
            be = bt + P.interval;
          }
          *tn = bt;
          return fold_until(be, vn);
        };
        double r1v = 0.0;
        const int kb = rates_beyond(P, of_ts, of_val, next, &r1v);
        of_has |= (uint8_t)(kb << 1);
        SM.of_rate[s] = r1v;
      }
    }
  }
  if (__ballot(err) && lane == 0) atomicOr(err_word, err);
  meta(true, of_has, of_ts, of_val);
}

// series point offsets from per-row output offsets (rows sorted by series)
#ifndef OTSDB_DS_TU
__global__ void k_series_offsets(int64_t R, int64_t S,
                                 const int64_t* __restrict__ row_series,
                                 const int64_t* __restrict__ row_out,
                                 int64_t* __restrict__ offsets) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > R) return;
  // series in (prev, cur] start at row r
  const int64_t prev = r == 0 ? -1 : row_series[r - 1];
  const int64_t cur = r == R ? S : row_series[r];
  for (int64_t s = prev + 1; s <= cur && s <= S; ++s) offsets[s] = row_out[r];
}

// ------------------------------------------------------------------------
// k_requal: columns whose qualifier widths mix (MS_MIXED_COMPACT rows, or
// second rows and millisecond rows in one series) rewritten with one width,
// so the cells fold streams them: every qualifier becomes the 4-byte
// millisecond qualifier of the same point (Internal.buildQualifier,
// Internal.java:848-863: 0xF << 28 | offset_ms << 6 | flags; a 2-byte
// qualifier's offset_s * 1000 < 2^22), the value pool stays as it is (same
// points, same value bytes, same meta byte).  One wavefront per row, 16
// two-byte units per lane (1,024 a pass: a 360-point row in one); MODE 0
// counts the row's points, MODE 1 writes its qualifiers at 4 * row_out[r]
// (qoff_out[r]), compacted through LDS into coalesced stores.
//
// Qualifier starts without a scan.  start(u+1) = !(start(u) && ms(u)): a
// unit that does not look like a millisecond qualifier's first (high nibble
// 0xF) makes the next unit a start, so inside a run of ms-looking units that
// begins on a start, starts and non-starts alternate; with the run's first
// unit at position a, the non-starts are a+1, a+3, ... (up to the unit just
// past the run).  Runs are labelled by the parity of a with one add (the
// carry of `m + even run starts` clears exactly the runs that begin on even
// positions).  Across a lane whose units all look like ms ones the start
// state flips 16 times (returns unchanged), so a lane's entry state is the
// exit state of the nearest lane below holding a non-ms unit (one ballot),
// or the pass's carry; the lane's starts for entry state 1 and 0 differ
// exactly on its units up to and including its first non-ms unit.  (Holding
// one unit per lane instead — ms-looking units as a 64-bit wave mask, the
// same logic on scalar registers — measured 2.5x slower for the count: a
// dependent chain of ~20 scalar ops per 64 units.)
DEV void requal_lane(uint32_t m, int nu, uint32_t& S1, uint32_t& flip, int& d,
                     int& fixed_out) {
  const uint32_t vm = nu >= 16 ? 0xFFFFu : ((1u << nu) - 1);
  const uint32_t edges = m & ~(m << 1);             // run starts
  const uint32_t x = m + (edges & 0x55555555u);      // even-start runs carry out
  const uint32_t ns = (((m & ~x) << 1) & 0xAAAAAAAAu) | (((m & x) << 1) & 0x55555555u);
  S1 = ~ns & vm;
  const uint32_t nz = ~m & vm;
  d = nz != 0;
  fixed_out = !((ns >> nu) & 1u);
  flip = d ? ((2u << __builtin_ctz(nz)) - 1) : vm;
}

// The lane's 32 bytes at a (units past the row are masked off later) and,
// for a 4-byte qualifier at its last unit, the 4 after them.
template <int MODE>
DEV void requal_words(const CellsDev& C, int64_t a, int64_t pool_end,
                      uint32_t* w) {
#pragma unroll
  for (int k = 0; k < 9; ++k) w[k] = 0;
  if (a + 36 <= pool_end) {
    const uint4 x0 = *reinterpret_cast<const uint4*>(C.qual + a);
    const uint4 x1 = *reinterpret_cast<const uint4*>(C.qual + a + 16);
    w[0] = x0.x; w[1] = x0.y; w[2] = x0.z; w[3] = x0.w;
    w[4] = x1.x; w[5] = x1.y; w[6] = x1.z; w[7] = x1.w;
    if (MODE == 1) w[8] = *reinterpret_cast<const uint32_t*>(C.qual + a + 32);
  } else if (a < pool_end) {  // the pool's last bytes
#pragma unroll
    for (int i = 0; i < 36; ++i)
      if (a + i < pool_end) w[i >> 2] |= (uint32_t)C.qual[a + i] << (8 * (i & 3));
  }
}

// rows per wavefront: the next row's first pass is loaded while this one
// is processed (rows are contiguous in the pool: it starts where this ends)
#ifndef OTSDB_RQ_RPW
#define OTSDB_RQ_RPW 8
#endif

template <int MODE>
__global__ __launch_bounds__(256) void k_requal(
    CellsDev C, int64_t* __restrict__ row_count,
    const int64_t* __restrict__ row_out, int64_t* __restrict__ qoff_out,
    uint8_t* __restrict__ qual_out, int* err_word) {
  constexpr int RPW = OTSDB_RQ_RPW;
  __shared__ uint32_t lds[MODE ? 4 : 1][MODE ? 1024 + 64 : 1];
  const int lane = LANE, wv = threadIdx.x >> 6;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wv) * RPW;
  if (r0 >= C.R) return;
  if (MODE == 1 && r0 == 0 && lane == 0) qoff_out[C.R] = 4 * row_out[C.R];
  const int64_t pool_end = C.qual_off[C.R];
  // the wave's row offsets (and output offsets), one per lane
  const int64_t off_l = (lane <= RPW && r0 + lane <= C.R) ? C.qual_off[r0 + lane] : 0;
  const int64_t out_l = (MODE == 1 && lane < RPW && r0 + lane < C.R) ? row_out[r0 + lane] : 0;
  const uint64_t below_me = (1ULL << lane) - 1;
  int bad = 0;
  uint32_t wn[9];
  requal_words<MODE>(C, readlane_l(off_l, 0) + 32 * lane, pool_end, wn);
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int64_t r = r0 + k;
    if (r >= C.R) break;
    const int64_t qa = readlane_l(off_l, k), qe = readlane_l(off_l, k + 1);
    uint32_t w[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) w[i] = wn[i];
    if (k + 1 < RPW && r + 1 < C.R) requal_words<MODE>(C, qe + 32 * lane, pool_end, wn);
    const int64_t qlen = qe - qa;
    const int64_t out0 = MODE ? readlane_l(out_l, k) : 0;
    if (MODE == 1 && lane == 0) qoff_out[r] = 4 * out0;
    if (qlen & 1) {  // not a data-point column (Internal.java:262-264)
      if (MODE == 0 && lane == 0) row_count[r] = 0;
      continue;
    }
    const int64_t units = qlen >> 1;
    int cs = 1;
    int64_t n_acc = 0;  // MODE 0: the lane's points; MODE 1: the row's so far
    for (int64_t u0 = 0; u0 < units; u0 += 1024) {
      if (u0 > 0) requal_words<MODE>(C, qa + 2 * u0 + 32 * lane, pool_end, w);
      const int64_t ub = u0 + 16 * lane;
      const int nu = ub >= units ? 0 : (int)(units - ub < 16 ? units - ub : 16);
      uint32_t m = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        m |= (uint32_t)((w[i] & 0xF0u) == 0xF0u) << (2 * i);
        m |= (uint32_t)((w[i] & 0xF00000u) == 0xF00000u) << (2 * i + 1);
      }
      m &= nu >= 16 ? 0xFFFFu : ((1u << nu) - 1);
      uint32_t S1, flip;
      int d, fixed_out;
      requal_lane(m, nu, S1, flip, d, fixed_out);
      const uint64_t below = __ballot(d) & below_me;
      const int fo_src = __shfl(fixed_out, below ? 63 - __builtin_clzll(below) : 0);
      const int cin = below ? fo_src : cs;
      const uint32_t S = cin ? S1 : (S1 ^ flip);
      // a 4-byte qualifier cut by the column end
      if (nu > 0 && ub + nu == units) bad |= (int)(((S & m) >> (nu - 1)) & 1u);
      cs = __builtin_amdgcn_readlane(d ? fixed_out : cin, 63);
      const int np = __builtin_popcount(S);
      if (MODE == 0) {
        n_acc += np;
        continue;
      }
      int tot;
      const int k0 = wave_excl_scan(np, tot);
      // branch free: every unit's 4-byte form goes to LDS, a non-start's to
      // the lane's scratch slot
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        // the unit's 4 bytes B0 B1 B2 B3 as stored (little-endian word)
        const uint32_t u = (i & 1) ? __builtin_amdgcn_alignbyte(w[(i >> 1) + 1], w[i >> 1], 2)
                                   : w[i >> 1];
        const uint32_t q2 = __builtin_amdgcn_perm(0u, u, 0x0c0c0001u);  // B0 B1
        const uint32_t ms4 = 0xF0000000u | ((q2 >> 4) * 64000u) | (q2 & 0xFu);
        // a 4-byte qualifier is kept byte for byte
        const uint32_t o = ((m >> i) & 1u) ? u : __builtin_amdgcn_perm(0u, ms4, 0x00010203u);
        const int slot = ((S >> i) & 1u) ? k0 + __builtin_popcount(S & ((1u << i) - 1))
                                         : 1024 + lane;
        lds[MODE ? wv : 0][slot] = o;
      }
      wave_lds_fence();
      uint32_t* dst = reinterpret_cast<uint32_t*>(qual_out) + out0 + n_acc;
      for (int j = lane; j < tot; j += 64) dst[j] = lds[MODE ? wv : 0][j];
      n_acc += tot;
      wave_lds_fence();
    }
    if (MODE == 0) {
      int tot;
      wave_excl_scan((int)n_acc, tot);
      if (lane == 0) row_count[r] = tot;
    }
  }
  if (__ballot(bad) && lane == 0) atomicOr(err_word, ERR_CORRUPT_CELL);
}
#endif  // OTSDB_DS_TU

}  // namespace otsdb
