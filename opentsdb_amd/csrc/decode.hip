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

namespace otsdb {

struct CellsDev {
  int64_t R;
  const int64_t* row_series;
  const int64_t* row_base_s;
  const int64_t* qual_off;
  const uint8_t* qual;
  const int64_t* val_off;
  const uint8_t* val;
};

enum : int { ERR_CORRUPT_CELL = 16 };

// map {0,1}->{0,1} as 2 bits: bit0 = f(0), bit1 = f(1)
DEV int fmap_apply(int f, int s) { return (f >> s) & 1; }
DEV int fmap_compose(int g, int f) {  // g o f
  return fmap_apply(g, f & 1) | (fmap_apply(g, (f >> 1) & 1) << 1);
}

// one wavefront per row; mode 0 counts (and validates), mode 1 writes
__global__ __launch_bounds__(256) void k_decode(
    CellsDev C, int mode, int64_t* __restrict__ row_count,
    const int64_t* __restrict__ row_out, int64_t cap, int64_t* __restrict__ ts,
    int64_t* __restrict__ val, uint8_t* __restrict__ isf, int* err_word) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= C.R) return;
  const uint8_t* q = C.qual + C.qual_off[r];
  const int64_t qlen = C.qual_off[r + 1] - C.qual_off[r];
  const uint8_t* v = C.val + C.val_off[r];
  const int64_t vlen = C.val_off[r + 1] - C.val_off[r];
  const int64_t base_ms = C.row_base_s[r] * 1000;
  if (qlen & 1) {  // not a data-point column (Internal.java:262-264)
    if (mode == 0 && lane == 0) row_count[r] = 0;
    return;
  }
  const int64_t units = qlen >> 1;
  int carry_start = 1;
  int64_t carry_n = 0, carry_voff = 0;
  int bad = 0;
  const int64_t out0 = mode ? row_out[r] : 0;
  for (int64_t u0 = 0; u0 < units; u0 += 64) {
    const int64_t u = u0 + lane;
    const bool in = u < units;
    const uint8_t b0 = in ? q[2 * u] : 0;
    const int ms = in && ((b0 & 0xF0) == 0xF0);
    // f_u(s) = !(s && ms_u)
    int f = in ? (ms ? 0x1 : 0x3) : 0x2;  // identity for lanes past the row
    int F = f;                               // inclusive composition
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int g = __shfl_up(F, d);
      if (lane >= d) F = fmap_compose(F, g);
    }
    int Fex = __shfl_up(F, 1);
    if (lane == 0) Fex = 0x2;  // identity
    const int start = in && fmap_apply(Fex, carry_start);
    // a 4-byte qualifier must fit in the row
    if (start && ms && u + 1 >= units) bad = 1;
    uint32_t qv = 0;
    int vl = 0;
    if (start) {
      if (ms) {
        if (u + 1 < units)
          qv = ((uint32_t)b0 << 24) | ((uint32_t)q[2 * u + 1] << 16) |
               ((uint32_t)q[2 * u + 2] << 8) | (uint32_t)q[2 * u + 3];
      } else {
        qv = ((uint32_t)b0 << 8) | (uint32_t)q[2 * u + 1];
      }
      vl = (int)(qv & 0x7) + 1;
      // RowSeq.extractIntegerValue / extractFloatingPointValue lengths
      if (qv & 0x8) bad |= !(vl == 4 || vl == 8);
      else bad |= !(vl == 1 || vl == 2 || vl == 4 || vl == 8);
    }
    // exclusive scans: point index and value offset
    const uint64_t sm = __ballot(start);
    const int64_t idx = carry_n + __popcll(sm & ((1ULL << lane) - 1));
    int64_t vo = vl;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t y = __shfl_up(vo, d);
      if (lane >= d) vo += y;
    }
    const int64_t voff = carry_voff + vo - vl;
    if (start && voff + vl > vlen) bad = 1;
    if (mode == 1 && start && !bad) {
      const int64_t o = out0 + idx;
      if (o < cap) {
        const uint8_t* p = v + voff;
        int64_t t;
        if (ms) t = base_ms + (int64_t)((qv & 0x0FFFFFC0u) >> 6);
        else t = base_ms + (int64_t)((qv & 0xFFFFu) >> 4) * 1000;
        int64_t bits = 0;
        const int fl = (qv & 0x8) != 0;
        uint64_t x = 0;
        for (int i = 0; i < vl; ++i) x = (x << 8) | p[i];
        if (!fl) {  // big-endian signed 1/2/4/8 bytes (RowSeq.java:233-245)
          switch (vl) {
            case 1: bits = (int8_t)x; break;
            case 2: bits = (int16_t)x; break;
            case 4: bits = (int32_t)x; break;
            case 8: bits = (int64_t)x; break;
            default: bad = 1;
          }
        } else {    // float widened / double (RowSeq.java:256-266)
          if (vl == 4) bits = __double_as_longlong((double)__uint_as_float((uint32_t)x));
          else if (vl == 8) bits = (int64_t)x;
          else bad = 1;
        }
        ts[o] = t;
        val[o] = bits;
        isf[o] = (uint8_t)fl;
      }
    }
    carry_n += __popcll(sm);
    carry_voff += __shfl(vo, 63);
    carry_start = fmap_apply(__shfl(F, 63), carry_start);
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

// series point offsets from per-row output offsets (rows sorted by series)
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

}  // namespace otsdb
