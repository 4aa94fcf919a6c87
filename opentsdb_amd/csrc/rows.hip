// rows.hip — storage rows -> compacted columns -> spans.
//
// Query-time compaction.  The scanner hands every storage row to
// CompactionQueue.compact (TSDB.compact, SaltScanner.java:849-881): the row's
// columns — single-point cells, compacted columns, append columns (0x05),
// annotations (0x01), histograms (0x06) — become ONE compacted column, the
// form RowSeq reads.  Rules restated (oracle/otsdb_oracle.c or_compact_row
// follows the same lines):
//   * buildHeapProcessAnnotations (CompactionQueue.java:435-489): odd-length
//     qualifiers are not data (append columns are parsed, the rest skipped);
//     every data column becomes a ColumnDatapointIterator whose 2-byte
//     single cells get the legacy fix-ups (ColumnDatapointIterator.java:73-87:
//     8-byte "float" values whose high half is zero become 4-byte floats,
//     Internal.fixFloatingPointValue :577-591; the qualifier's length bits are
//     rewritten to the value length, Internal.fixQualifierFlags :535-545);
//   * AppendDataPoints.parseKeyValue (AppendDataPoints.java:118-236): the
//     (qualifier, value) pairs of an append column, keyed by time offset in a
//     TreeMap — the later of equal offsets replaces the earlier — and emitted
//     in offset order; a value that does not break down is
//     IllegalDataException, a qualifier that is not exactly {0x05,0,0} is
//     IllegalArgumentException;
//   * noMergesOrFixups (:317-332): one heaped column holding one 2-byte cell
//     that needs no fix-up, or one 4-byte ms cell, is returned as stored;
//   * defaultMergeDataPoints (:549-584): the iterators pop from a
//     PriorityQueue ordered by (time offset, newer HBase cell first,
//     ColumnDatapointIterator.compareTo :192-199); the first cell of an offset
//     is kept, later ones are compared with it and, when their bytes differ,
//     raise IllegalDataException unless tsd.storage.fix_duplicates;
//   * buildCompactedColumn (:594-616): one meta byte after the values of a
//     multi-value column, bit 0 = seconds and ms cells mixed.
// When every column's cells are in offset order (what the write path and
// compaction produce) the heap order IS the stable sort by (offset, column
// rank, position), rank = (HBase timestamp desc, column index desc), so a
// wavefront sorts the row's cell keys in LDS (bitonic) and keeps the first of
// each offset.  A row holding a column whose cells go back in time takes an
// exact emulation of the heap (wave arg-min over the column heads per step).
//
// Kernels (one wavefront per storage row unless said otherwise):
//   k_rows_uniform  64 rows per wavefront: single compacted columns the
//                   merge rebuilds byte for byte (one qualifier width,
//                   strictly increasing offsets, lengths adding up, meta 0)
//                   are VERBATIM; the rest are left to k_rows_plan;
//   k_rows_plan     classifies the row: EMPTY (no data point: dropped, like
//                   the scanner drops a null compaction), VERBATIM (the
//                   noMergesOrFixups case), LONE (one data column: its cells
//                   in column order, consecutive equal offsets merged — a
//                   one-iterator heap), or GENERAL (several columns or an
//                   append column: cell count for the scratch records);
//                   LONE/VERBATIM output sizes; construction errors in
//                   column order;
//   k_rows_general  GENERAL rows: cell records -> sort (or heap emulation) ->
//                   merged column in a staging area;
//   k_rows_write    packs every kept row at its scanned output offsets.
//
// Span assembly (Span.addRow, Span.java:177-220; RowSeq.addRow,
// RowSeq.java:91-222; checkRowOrder :387-392): a series whose rows arrive
// with strictly increasing base times (what one scanner delivers) is its
// rows, unchanged.  Any other series (a row key seen twice, rows out of
// order) is replayed exactly by one lane: the merge into the first RowSeq of
// the same key when the row's first point is not after the last RowSeq's last
// point (two-pointer merge by offset, the incoming duplicate dropped, meta
// byte = OR of the two last bytes' bit 0), a new RowSeq otherwise, then the
// stable sort by base time.  RowSeq.size / timestamp(i) read the mixed bit
// from the last value byte exactly as the reference does (:338-420).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace otsdb {

#ifndef OTSDB_DS_TU

struct RawDev {
  int64_t R;
  const int64_t* row_col_off;  // [R+1]
  const int64_t* col_qoff;     // [C+1]
  const uint8_t* qual;
  const int64_t* col_voff;     // [C+1]
  const uint8_t* val;
  const int64_t* col_ts;       // [C] or null (= column index)
};

// row status codes (otsdb_status values)
enum : int { RS_ILLEGAL_DATA = 1, RS_ILLEGAL_ARGUMENT = 3, RS_UNSUPPORTED = 5 };
enum : uint8_t {
  RK_EMPTY = 0, RK_VERBATIM = 1, RK_LONE = 2, RK_GENERAL = 3, RK_LARGE = 4,
  RK_PENDING = 5  // k_rows_uniform left the row to k_rows_plan
};
// column types
enum : int { CT_SKIP = 0, CT_APPEND = 1, CT_ONE = 2, CT_MULTI = 3 };

constexpr int kRowCellCap = 8192;  // GENERAL rows: cells sorted in LDS
constexpr int kRowColCap = 4096;   // GENERAL rows: data columns ranked in LDS

// one cell of a GENERAL row (scratch), 32 bytes
struct CellRec {
  int64_t qpos;   // qualifier bytes: index into qual (or val, RF_QINVAL)
  int64_t vpos;   // value bytes: index into val
  int32_t off;    // time offset, ms
  int32_t col;    // column rank in the row
  uint8_t ql, vl; // qualifier / value length of the point
  uint8_t vav;    // value bytes present in the column (<= vl)
  uint8_t flags;  // RF_*
  uint8_t qfix;   // fixed second qualifier byte (RF_QFIX)
  uint8_t pad[7];
};
enum : uint8_t {
  RF_QFIX = 1, RF_QINVAL = 2, RF_MS = 4, RF_APPEND = 8, RF_OVERRUN = 16
};

// LARGE rows (past kRowCellCap cells or kRowColCap data columns): one slot
// each, claimed by k_rows_plan
struct LargeSlots {
  unsigned long long* ctr;  // [0] slots, [1] ranked columns
  int64_t* row;             // slot -> row
  int64_t* ncol;            // its data columns
  int64_t* cbase;           // its first ranked-column position
};

DEV void row_error(unsigned long long* first_err, int64_t r, int code) {
  atomicMin(first_err, ((unsigned long long)r << 8) | (unsigned)code);
}

DEV int32_t qual_off_ms(uint32_t qv, int ms) {
  return ms ? (int32_t)((qv & 0x0FFFFFC0u) >> 6)
            : (int32_t)((qv & 0xFFFFu) >> 4) * 1000;
}

DEV int lane_prev(uint64_t mask, int lane) {  // highest set bit below lane
  const uint64_t m = mask & ((1ULL << lane) - 1);
  return m ? 63 - __builtin_clzll(m) : -1;
}
DEV int lane_last_le(uint64_t mask, int lane) {  // highest set bit <= lane
  const uint64_t m = lane == 63 ? mask : mask & ((2ULL << lane) - 1);
  return m ? 63 - __builtin_clzll(m) : -1;
}

DEV int64_t wave_incl_scan(int64_t x) {
  const int lane = LANE;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

DEV int32_t wave_sum_i(int32_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
  return x;
}

DEV int64_t wave_sum_l(int64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
  return x;
}

DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// AppendDataPoints.parseKeyValue's first loop: the number of (qualifier,
// value) pairs, or -1 when the bytes do not break down
DEV int64_t append_count(const uint8_t* v, int64_t vl) {
  int64_t n = 0, i = 0;
  while (i < vl) {
    const int ql = (v[i] & 0xF0) == 0xF0 ? 4 : 2;
    if (i + ql > vl) return -1;
    i += ql + (v[i + ql - 1] & 0x7) + 1;
    if (i > vl) return -1;
    ++n;
  }
  return n;
}

// checkForFixup on a 2-byte cell: the fixed second qualifier byte and the
// value bytes after the float fix (vskip = 4 when the high half is dropped);
// bad = the high half is not zero
DEV uint8_t fixup2(uint8_t f, const uint8_t* v, int64_t vl, int& vskip,
                   int& bad) {
  vskip = 0;
  bad = 0;
  if ((f & 0x8) && (f & 0x7) == 0x3 && vl == 8) {
    if (v[0] | v[1] | v[2] | v[3]) bad = 1;
    vskip = 4;
  }
  return (uint8_t)((f & ~0x7) | ((vl - vskip - 1) & 0xFF));
}

struct ColInfo {
  int type;     // CT_*
  int err;      // construction error (RS_*), 0 if none
  int64_t cells;  // CT_ONE: 1, CT_APPEND: pairs, CT_MULTI: -1 (walk)
  int fixed;    // CT_ONE 2-byte: checkForFixup changes the cell
};

// One column as buildHeapProcessAnnotations + the iterator constructor see
// it (lane-level)
DEV ColInfo col_info(const RawDev& D, int64_t c) {
  ColInfo ci{CT_SKIP, 0, 0, 0};
  const int64_t qo = D.col_qoff[c], ql = D.col_qoff[c + 1] - qo;
  const int64_t vo = D.col_voff[c], vl = D.col_voff[c + 1] - vo;
  if (ql == 0) return ci;
  const uint8_t* q = D.qual + qo;
  if (ql & 1) {
    if (q[0] != 0x05) return ci;  // annotation / histogram / unknown
    if (ql != 3) {
      ci.err = RS_ILLEGAL_ARGUMENT;
      return ci;
    }
    const int64_t n = append_count(D.val + vo, vl);
    if (n < 0) ci.err = RS_ILLEGAL_DATA;
    else if (n > 0) {
      ci.type = CT_APPEND;
      ci.cells = n;
    }
    return ci;
  }
  // a data column: no value bytes, or a first qualifier running past the
  // column, is a corrupt cell (see the oracle)
  if (vl == 0) {
    ci.err = RS_ILLEGAL_DATA;
    return ci;
  }
  const bool ms0 = (q[0] & 0xF0) == 0xF0;
  if (ms0 && ql < 4) {
    ci.err = RS_ILLEGAL_DATA;
    return ci;
  }
  if (ql == 2) {
    int vskip, bad;
    const uint8_t nf = fixup2(q[1], D.val + vo, vl, vskip, bad);
    if (bad) {
      ci.err = RS_ILLEGAL_DATA;
      return ci;
    }
    ci.type = CT_ONE;
    ci.cells = 1;
    ci.fixed = vskip != 0 || nf != q[1];
    return ci;
  }
  if (ql == 4 && ms0) {
    ci.type = CT_ONE;
    ci.cells = 1;
    return ci;
  }
  ci.type = CT_MULTI;
  ci.cells = -1;
  return ci;
}

// Wave walk over the points of one compacted column in column order
// (ColumnDatapointIterator.update/advance :167-187): point starts are a scan
// of the 2-/4-byte qualifier widths over 2-byte units (fmap recurrence of
// decode.hip), value offsets a scan of the lengths; the column ends at the
// first point whose value offset is past the value bytes.  A 4-byte
// qualifier cut by the column end, when reached, is an error (trunc).
struct ColWalk {
  const uint8_t* q;
  int64_t units, vlen;
  int64_t u0 = 0, carry_n = 0, carry_vo = 0;
  int carry_start = 1;
  bool done = false;
  // per-lane point of the current chunk
  bool cell;
  int ms, ql, vl, trunc;
  int32_t off;
  int64_t k, qo, vo;
  uint64_t mask;

  DEV ColWalk(const uint8_t* q_, int64_t qlen, int64_t vlen_)
      : q(q_), units(qlen >> 1), vlen(vlen_) {}

  DEV bool step() {
    if (done || u0 >= units) return false;
    const int lane = LANE;
    const int64_t u = u0 + lane;
    const bool in = u < units;
    const uint8_t b0 = in ? q[2 * u] : 0;
    const int msu = in && ((b0 & 0xF0) == 0xF0);
    int F = in ? (msu ? 0x1 : 0x3) : 0x2;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int g = __shfl_up(F, d);
      if (lane >= d) F = fmap_compose(F, g);
    }
    int Fex = __shfl_up(F, 1);
    if (lane == 0) Fex = 0x2;
    const int start = in && fmap_apply(Fex, carry_start);
    const int tr = start && msu && (u + 1 >= units);
    uint32_t qv = 0;
    if (start && !tr)
      qv = msu ? ((uint32_t)b0 << 24) | ((uint32_t)q[2 * u + 1] << 16) |
                     ((uint32_t)q[2 * u + 2] << 8) | (uint32_t)q[2 * u + 3]
               : ((uint32_t)b0 << 8) | (uint32_t)q[2 * u + 1];
    const int l = (start && !tr) ? (int)(qv & 0x7) + 1 : 0;
    const int64_t incl = wave_incl_scan(l);
    vo = carry_vo + incl - l;
    const bool reach = start && vo < vlen;
    trunc = reach && tr;
    cell = reach && !tr;
    if (__ballot(start && (vo >= vlen || tr))) done = true;
    mask = __ballot(cell);
    k = carry_n + __popcll(mask & ((1ULL << lane) - 1));
    ms = msu;
    ql = msu ? 4 : 2;
    vl = l;
    qo = 2 * u;
    off = qual_off_ms(qv, msu);
    carry_n += __popcll(mask);
    carry_vo += __shfl(incl, 63);
    carry_start = fmap_apply(__shfl(F, 63), carry_start);
    u0 += 64;
    return true;
  }
};

DEV bool bytes_equal_padded(const uint8_t* val, int64_t a, int la, int aav,
                            int64_t b, int lb, int bav) {
  if (la != lb) return false;
  for (int i = 0; i < la; ++i) {
    const uint8_t x = i < aav ? val[a + i] : 0;
    const uint8_t y = i < bav ? val[b + i] : 0;
    if (x != y) return false;
  }
  return true;
}

struct LoneOut {
  int64_t nq, nv, kept;
  int err;
  int meta;  // the meta byte written when kept > 1
};

// A row with one data column: the one-iterator heap.  Points in column
// order; a point whose offset equals the previous point's is a duplicate of
// the run's first (kept) point — compared byte for byte (Arrays.copyOfRange:
// zero-padded past the column) and an error unless fix_duplicates.  WRITE:
// the kept points' bytes go to oq / ov.
template <bool WRITE>
DEV LoneOut lone_walk(const RawDev& D, int64_t c, int fix, uint8_t* oq,
                      uint8_t* ov) {
  const int lane = LANE;
  LoneOut o{0, 0, 0, 0, 0};
  const int64_t qb = D.col_qoff[c], ql = D.col_qoff[c + 1] - qb;
  const int64_t vb = D.col_voff[c], vl = D.col_voff[c + 1] - vb;
  const uint8_t* q = D.qual + qb;
  if (ql == 2) {  // a fixed-up single cell (the unfixed one is VERBATIM)
    int vskip, bad;
    const uint8_t nf = fixup2(q[1], D.val + vb, vl, vskip, bad);
    const int cur = (nf & 0x7) + 1;
    if (cur > vl - vskip) {
      o.err = RS_ILLEGAL_DATA;
      return o;
    }
    o.nq = 2;
    o.nv = cur;
    o.kept = 1;
    if (WRITE && lane == 0) {
      oq[0] = q[0];
      oq[1] = nf;
      for (int i = 0; i < cur; ++i) ov[i] = D.val[vb + vskip + i];
    }
    return o;
  }
  ColWalk w(q, ql, vl);
  bool have_prev = false;
  int32_t prev_off = 0;
  int64_t lvo = 0;  // the current run's kept point
  int lvl = 0, lvav = 0;
  int ms_in = 0, s_in = 0, bad = 0;
  while (w.step()) {
    const uint64_t m = w.mask;
    if (w.trunc) bad = 1;
    const int pl = lane_prev(m, lane);
    int32_t poff = __shfl(w.off, pl < 0 ? 0 : pl);
    const bool hp = pl >= 0 || have_prev;
    if (pl < 0) poff = prev_off;
    const bool dup = w.cell && hp && w.off == poff;
    const bool lead = w.cell && !dup;
    const int vav = (int)(w.vo + w.vl <= vl ? w.vl : vl - w.vo);
    const uint64_t lm = __ballot(lead);
    const int ll = lane_last_le(lm, lane);
    int64_t rvo = __shfl(w.vo, ll < 0 ? 0 : ll);
    int rvl = __shfl(w.vl, ll < 0 ? 0 : ll);
    int rvav = __shfl(vav, ll < 0 ? 0 : ll);
    if (ll < 0) {
      rvo = lvo;
      rvl = lvl;
      rvav = lvav;
    }
    if (dup && !fix &&
        !bytes_equal_padded(D.val, vb + w.vo, w.vl, vav, vb + rvo, rvl, rvav))
      bad = 1;
    if (lead && w.vo + w.vl > vl) bad = 1;  // a kept value past the column
    const int64_t kq = lead ? w.ql : 0, kv = lead ? w.vl : 0;
    const int64_t iq = wave_incl_scan(kq), iv = wave_incl_scan(kv);
    if (WRITE && lead && !bad) {
      uint8_t* dq = oq + o.nq + iq - kq;
      uint8_t* dv = ov + o.nv + iv - kv;
      for (int i = 0; i < w.ql; ++i) dq[i] = q[w.qo + i];
      for (int i = 0; i < w.vl; ++i) dv[i] = D.val[vb + w.vo + i];
    }
    ms_in |= __ballot(lead && w.ms) != 0;
    s_in |= __ballot(lead && !w.ms) != 0;
    o.nq += __shfl(iq, 63);
    o.nv += __shfl(iv, 63);
    o.kept += __popcll(lm);
    if (m) {
      const int last = 63 - __builtin_clzll(m);
      prev_off = __shfl(w.off, last);
      have_prev = true;
    }
    if (lm) {
      const int last = 63 - __builtin_clzll(lm);
      lvo = __shfl(w.vo, last);
      lvl = __shfl(w.vl, last);
      lvav = __shfl(vav, last);
    }
    if (__ballot(bad)) {
      o.err = RS_ILLEGAL_DATA;
      return o;
    }
  }
  if (o.kept > 1) {
    o.meta = (ms_in && s_in) ? 1 : 0;
    if (WRITE && lane == 0) ov[o.nv] = (uint8_t)o.meta;
    o.nv += 1;
  }
  return o;
}

// The common LONE column, decided without the walk (k_rows_plan): every
// qualifier has the width of the first (no MS_MIXED_COMPACT), time offsets
// strictly increase (no repeated offset for the one-iterator heap to merge),
// the value lengths add up to the column's value bytes less the meta byte,
// and the meta byte is the 0 buildCompactedColumn writes for one resolution
// (CompactionQueue.java:594-616).  Such a column is what a TSD compaction
// wrote, and the merge rebuilds it byte for byte: VERBATIM.  Anything else
// is decided by lone_walk's exact replay.  One 16-byte qualifier load per
// lane (8 second or 4 ms qualifiers), 1 KB of qualifiers per pass.

// ---------------------------------------------------------------- planning
// The exact plan of one row (wave-level): column classification, the lone
// column's one-iterator replay, GENERAL / LARGE cell counts.
DEV void plan_row(const RawDev& D, int fix, int64_t r, uint8_t* __restrict__ kind,
                  int64_t* __restrict__ lone, int64_t* __restrict__ gen_n,
                  int64_t* __restrict__ out_q, int64_t* __restrict__ out_v,
                  int64_t* __restrict__ kept, unsigned long long* first_err,
                  const LargeSlots& LS) {
  const int lane = LANE;
  const int64_t c0 = D.row_col_off[r], c1 = D.row_col_off[r + 1];
  int64_t n_data = 0, cells = 0, first_c = -1;
  int first_type = CT_SKIP, first_fixed = 0, merge_bad = 0;
  int err = 0;
  for (int64_t cc = c0; cc < c1; cc += 64) {
    const int64_t c = cc + lane;
    ColInfo ci{CT_SKIP, 0, 0, 0};
    if (c < c1) ci = col_info(D, c);
    const uint64_t em = __ballot(ci.err != 0);
    if (em) {  // the first failing column in column order
      err = __shfl(ci.err, __builtin_ctzll(em));
      break;
    }
    const uint64_t dm = __ballot(ci.type != CT_SKIP);
    if (dm && first_c < 0) {
      const int fl = __builtin_ctzll(dm);
      first_c = cc + fl;
      first_type = __shfl(ci.type, fl);
      first_fixed = __shfl(ci.fixed, fl);
    }
    n_data += __popcll(dm);
    cells += wave_sum_l(ci.type == CT_ONE || ci.type == CT_APPEND ? ci.cells : 0);
  }
  // multi-point columns of GENERAL rows: counted by a wave walk (a lone
  // column is decided below, by lone_uniform or lone_walk)
  for (int64_t cc = c0; !err && n_data > 1 && cc < c1; cc += 64) {
    const int64_t c = cc + lane;
    const ColInfo ci = c < c1 ? col_info(D, c) : ColInfo{CT_SKIP, 0, 0, 0};
    uint64_t mm = __ballot(ci.type == CT_MULTI);
    while (mm) {
      const int b = __builtin_ctzll(mm);
      mm &= mm - 1;
      const int64_t col = cc + b;
      const int64_t qb = D.col_qoff[col], vb = D.col_voff[col];
      ColWalk w(D.qual + qb, D.col_qoff[col + 1] - qb, D.col_voff[col + 1] - vb);
      int64_t n = 0;
      while (w.step()) {
        if (__ballot(w.trunc)) merge_bad = 1;
        n += __popcll(w.mask);
      }
      cells += n;
    }
  }
  auto put = [&](uint8_t k, int64_t nq, int64_t nv, int64_t g) {
    if (lane == 0) {
      kind[r] = k;
      lone[r] = first_c;
      gen_n[r] = g;
      out_q[r] = nq;
      out_v[r] = nv;
      kept[r] = (k == RK_EMPTY) ? 0 : 1;
    }
  };
  if (err) {
    if (lane == 0) row_error(first_err, r, err);
    put(RK_EMPTY, 0, 0, 0);
    return;
  }
  if (n_data == 0) {
    put(RK_EMPTY, 0, 0, 0);
    return;
  }
  if (n_data == 1 && first_type != CT_APPEND) {
    const int64_t ql = D.col_qoff[first_c + 1] - D.col_qoff[first_c];
    const int64_t vl = D.col_voff[first_c + 1] - D.col_voff[first_c];
    if (first_type == CT_ONE && !first_fixed) {  // noMergesOrFixups
      put(RK_VERBATIM, ql, vl, 0);
      return;
    }
    const LoneOut o = lone_walk<false>(D, first_c, fix, nullptr, nullptr);
    if (o.err) {
      if (lane == 0) row_error(first_err, r, o.err);
      put(RK_EMPTY, 0, 0, 0);
      return;
    }
    // a column the one-iterator merge rebuilds byte for byte (no repeated
    // offset, every value byte used, the same meta byte: what a TSD
    // compaction wrote) is copied as stored
    if (o.kept > 1 && o.nq == ql && o.nv == vl &&
        D.val[D.col_voff[first_c] + vl - 1] == (uint8_t)o.meta) {
      put(RK_VERBATIM, ql, vl, 0);
      return;
    }
    put(o.kept ? RK_LONE : RK_EMPTY, o.nq, o.nv, 0);
    return;
  }
  if (merge_bad) {
    if (lane == 0) row_error(first_err, r, RS_ILLEGAL_DATA);
    put(RK_EMPTY, 0, 0, 0);
    return;
  }
  if (cells > kRowCellCap || n_data > kRowColCap) {
    // past the LDS caps: the global-memory merge (k_large_*); a slot, its
    // ranked-column range (slots and ranges in claim order: the layout may
    // vary, the merged rows do not)
    if (lane == 0) {
      const unsigned long long sl = atomicAdd(&LS.ctr[0], 1ULL);
      LS.row[sl] = r;
      LS.ncol[sl] = n_data;
      LS.cbase[sl] = (int64_t)atomicAdd(&LS.ctr[1], (unsigned long long)n_data);
    }
    put(RK_LARGE, 0, 0, cells);
    return;
  }
  put(RK_GENERAL, 0, 0, cells);
}

// One 1 KB pass of a uniform-width column's qualifiers (this lane's 16
// bytes w[], nb of them valid): widths, strictly increasing offsets across
// lanes and from the previous pass (carry), value lengths.
DEV void uniform_pass(const uint32_t* w, int nb, int qw, int32_t& carry,
                      int& bad, int32_t& vsum) {
  const int lane = LANE;
  int32_t first = INT32_MAX, last = -1;
  if (qw == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (2 * j < nb) {
        const uint32_t h = (w[j >> 1] >> (16 * (j & 1))) & 0xFFFF;
        const uint32_t qv = ((h & 0xFF) << 8) | (h >> 8);
        const int32_t o = (int32_t)(qv >> 4);
        bad |= (qv >> 12) == 0xF;  // an ms qualifier starts here
        bad |= o <= last;
        first = j == 0 ? o : first;
        last = o;
        vsum += (int32_t)(qv & 0x7) + 1;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (4 * j < nb) {
        const uint32_t qv = __builtin_bswap32(w[j]);
        const int32_t o = (int32_t)((qv & 0x0FFFFFC0u) >> 6);
        bad |= (qv >> 28) != 0xF;  // a second qualifier starts here
        bad |= o <= last;
        first = j == 0 ? o : first;
        last = o;
        vsum += (int32_t)(qv & 0x7) + 1;
      }
    }
  }
  const int32_t pl = __shfl_up(last, 1);
  const int32_t prev = lane == 0 ? carry : pl;
  if (nb > 0 && first <= prev) bad = 1;
  const uint64_t live = __ballot(nb > 0);
  carry = __shfl(last, live ? 63 - __builtin_clzll(live) : 0);
}

// this lane's 16 qualifier bytes of a pass at byte a of a column of ql bytes
// at qb (16-byte loads at any byte offset; byte loads at the pool's end)
DEV int uniform_load(const uint8_t* qual, int64_t qb, int64_t ql, int64_t a,
                     int64_t qend, uint32_t* w) {
  w[0] = w[1] = w[2] = w[3] = 0;
  const int nb = a >= ql ? 0 : (int)(ql - a < 16 ? ql - a : 16);
  if (nb == 16 && qb + a + 16 <= qend) {
    const uint4 x = *reinterpret_cast<const uint4*>(qual + qb + a);
    w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
  } else {
    for (int i = 0; i < nb; ++i)
      w[i >> 2] |= (uint32_t)qual[qb + a + i] << (8 * (i & 3));
  }
  return nb;
}

// k_rows_uniform: one wavefront per 64 rows.  Lanes read their rows' shapes
// (thread per row); single compacted columns the merge would rebuild byte
// for byte (lone_uniform's conditions) are decided VERBATIM by the wave
// with four rows' qualifier passes in flight at a time.  Every other row is
// marked RK_PENDING (pending[0] = 1) for k_rows_plan's exact plan — a
// separate kernel, so this one keeps a small register footprint (more
// waves in flight for its dependent loads).
__global__ __launch_bounds__(256) void k_rows_uniform(
    RawDev D, uint8_t* __restrict__ kind, int64_t* __restrict__ lone,
    int64_t* __restrict__ gen_n, int64_t* __restrict__ out_q,
    int64_t* __restrict__ out_v, int64_t* __restrict__ kept,
    int* __restrict__ pending) {
  const int lane = LANE;
  const int64_t rb = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (rb >= D.R) return;
  const int64_t r = rb + lane;
  const int64_t qend = D.col_qoff[D.row_col_off[D.R]];
  bool cand = false;
  int64_t c0 = 0, qb = 0, ql = 0, vl = 0;
  int qw = 2;
  if (r < D.R) {
    c0 = D.row_col_off[r];
    if (D.row_col_off[r + 1] - c0 == 1) {
      qb = D.col_qoff[c0];
      ql = D.col_qoff[c0 + 1] - qb;
      const int64_t vb = D.col_voff[c0];
      vl = D.col_voff[c0 + 1] - vb;
      if (ql >= 4 && !(ql & 1) && vl >= 2) {
        qw = (D.qual[qb] & 0xF0) == 0xF0 ? 4 : 2;
        cand = !(ql & (qw - 1)) && ql >= 2 * qw && D.val[vb + vl - 1] == 0;
      }
    }
  }
  uint64_t done = 0;
  uint64_t small = __ballot(cand && ql <= 1024);
  uint64_t large = __ballot(cand && ql > 1024);
  while (small) {  // four one-pass rows per round
    int js[4];
    int k = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      js[i] = small ? __builtin_ctzll(small) : -1;
      if (small) {
        small &= small - 1;
        ++k;
      }
    }
    uint32_t w[4][4];
    int nb[4], qwk[4];
    int64_t vlk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      nb[i] = 0;
      qwk[i] = 2;
      vlk[i] = 0;
      w[i][0] = w[i][1] = w[i][2] = w[i][3] = 0;
      if (i < k) {
        const int64_t b = readlane_l(qb, js[i]), l = readlane_l(ql, js[i]);
        qwk[i] = __builtin_amdgcn_readlane(qw, js[i]);
        vlk[i] = readlane_l(vl, js[i]);
        nb[i] = uniform_load(D.qual, b, l, 16 * lane, qend, w[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < k) {
        int32_t carry = -1, vsum = 0;
        int bad = 0;
        uniform_pass(w[i], nb[i], qwk[i], carry, bad, vsum);
        vsum = wave_sum_i(vsum);
        if (!__ballot(bad) && (int64_t)vsum + 1 == vlk[i])
          done |= 1ULL << js[i];
      }
    }
  }
  while (large) {  // multi-pass rows (long ms columns), one at a time
    const int j = __builtin_ctzll(large);
    large &= large - 1;
    const int64_t b = readlane_l(qb, j), l = readlane_l(ql, j);
    const int q = __builtin_amdgcn_readlane(qw, j);
    int32_t carry = -1;
    int32_t vsum = 0;
    int bad = 0;
    for (int64_t p = 0; p < l && !bad; p += 1024) {
      uint32_t w[4];
      const int nb = uniform_load(D.qual, b, l, p + 16 * lane, qend, w);
      uniform_pass(w, nb, q, carry, bad, vsum);
      bad = __ballot(bad) != 0;
    }
    vsum = wave_sum_i(vsum);
    if (!bad && (int64_t)vsum + 1 == readlane_l(vl, j)) done |= 1ULL << j;
  }
  if (r < D.R) {
    if ((done >> lane) & 1) {
      kind[r] = RK_VERBATIM;
      lone[r] = c0;
      gen_n[r] = 0;
      out_q[r] = ql;
      out_v[r] = vl;
      kept[r] = 1;
    } else {
      kind[r] = RK_PENDING;
    }
  }
  if (__ballot(r < D.R) & ~done && lane == 0) pending[0] = 1;
}

// k_rows_plan: the exact plan of the rows k_rows_uniform left pending, one
// wavefront per row.
__global__ __launch_bounds__(256) void k_rows_plan(
    RawDev D, int fix, uint8_t* __restrict__ kind, int64_t* __restrict__ lone,
    int64_t* __restrict__ gen_n, int64_t* __restrict__ out_q,
    int64_t* __restrict__ out_v, int64_t* __restrict__ kept,
    unsigned long long* first_err, LargeSlots LS) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= D.R || kind[r] != RK_PENDING) return;
  plan_row(D, fix, r, kind, lone, gen_n, out_q, out_v, kept, first_err, LS);
}

// ---------------------------------------------------------- GENERAL rows
union GenLds {
  uint64_t keys[kRowCellCap];
  struct {
    int64_t ts[kRowColCap];
    int32_t cidx[kRowColCap];
    int32_t base[kRowColCap + 1];
  } col;
  struct {
    int32_t hoff[kRowColCap];
    int32_t head[kRowColCap];
    int32_t end[kRowColCap];
  } hp;
};

DEV void write_cell(const RawDev& D, const CellRec& x, uint8_t* dq,
                    uint8_t* dv) {
  const uint8_t* qs = (x.flags & RF_QINVAL) ? D.val : D.qual;
  for (int i = 0; i < x.ql; ++i)
    dq[i] = (i == 1 && (x.flags & RF_QFIX)) ? x.qfix : qs[x.qpos + i];
  for (int i = 0; i < x.vl; ++i) dv[i] = D.val[x.vpos + i];
}

// The heap order over keys sorted by (offset, rank-order record index)
// (defaultMergeDataPoints, CompactionQueue.java:549-584): the first cell of
// each offset is kept and written to the staging area, later ones are
// duplicates compared with it (IllegalDataException unless fix_duplicates);
// an append column's TreeMap-replaced pair is never popped.  keys: LDS
// (GENERAL rows) or global memory (LARGE rows).
DEV void merge_sorted(const RawDev& D, int fix, const CellRec* R, int64_t n,
                      const uint64_t* keys, uint8_t* sq, uint8_t* sv,
                      int64_t& nq, int64_t& nv, int64_t& nk, int& ms_in,
                      int& s_in, int& bad) {
  const int lane = LANE;
  int64_t lvpos = 0;
  int lvl = 0, lvav = 0;
  for (int64_t p0 = 0; p0 < n; p0 += 64) {
    const int64_t p = p0 + lane;
    const bool in = p < n;
    CellRec x{};
    bool lead = false, dup = false;
    if (in) {
      const uint64_t key = keys[p];
      x = R[(uint32_t)key];
      if (p == 0 || (keys[p - 1] >> 32) != (key >> 32)) {
        lead = true;
      } else {
        const CellRec& y = R[(uint32_t)keys[p - 1]];
        // a pair an append column's TreeMap replaced: never popped
        dup = !((x.flags & RF_APPEND) && y.col == x.col);
      }
    }
    const uint64_t lm = __ballot(lead);
    const int ll = lane_last_le(lm, lane);
    int64_t rvpos = __shfl(x.vpos, ll < 0 ? 0 : ll);
    int rvl = __shfl((int)x.vl, ll < 0 ? 0 : ll);
    int rvav = __shfl((int)x.vav, ll < 0 ? 0 : ll);
    if (ll < 0) {
      rvpos = lvpos;
      rvl = lvl;
      rvav = lvav;
    }
    if (dup && !fix &&
        !bytes_equal_padded(D.val, x.vpos, x.vl, x.vav, rvpos, rvl, rvav))
      bad = 1;
    if (lead && (x.flags & RF_OVERRUN)) bad = 1;
    const int64_t kq = lead ? x.ql : 0, kv = lead ? x.vl : 0;
    const int64_t iq = wave_incl_scan(kq), iv = wave_incl_scan(kv);
    if (lead && !bad) write_cell(D, x, sq + nq + iq - kq, sv + nv + iv - kv);
    ms_in |= __ballot(lead && (x.flags & RF_MS)) != 0;
    s_in |= __ballot(lead && !(x.flags & RF_MS)) != 0;
    nq += __shfl(iq, 63);
    nv += __shfl(iv, 63);
    nk += __popcll(lm);
    if (lm) {
      const int last = 63 - __builtin_clzll(lm);
      lvpos = __shfl(x.vpos, last);
      lvl = __shfl((int)x.vl, last);
      lvav = __shfl((int)x.vav, last);
    }
    if (__ballot(bad)) break;
  }
}

// buildCompactedColumn (CompactionQueue.java:594-616): the meta byte of a
// multi-value column, the row's output sizes (or its error)
DEV void finish_row(int64_t r, int bad, int64_t nq, int64_t nv, int64_t nk,
                    int ms_in, int s_in, uint8_t* sv, int64_t* out_q,
                    int64_t* out_v, unsigned long long* first_err) {
  const int lane = LANE;
  if (__ballot(bad)) {
    if (lane == 0) {
      row_error(first_err, r, RS_ILLEGAL_DATA);
      out_q[r] = 0;
      out_v[r] = 0;
    }
    return;
  }
  if (nk > 1) {
    if (lane == 0) sv[nv] = (ms_in && s_in) ? 1 : 0;
    nv += 1;
  }
  if (lane == 0) {
    out_q[r] = nq;
    out_v[r] = nv;
  }
}

__global__ __launch_bounds__(64) void k_rows_general(
    RawDev D, int fix, const uint8_t* __restrict__ kind,
    const int64_t* __restrict__ gen_base, CellRec* __restrict__ rec,
    uint8_t* __restrict__ stq, uint8_t* __restrict__ stv,
    int64_t* __restrict__ out_q, int64_t* __restrict__ out_v,
    unsigned long long* first_err) {
  __shared__ GenLds sm;
  const int lane = LANE;
  const int64_t r = blockIdx.x;
  if (r >= D.R || kind[r] != RK_GENERAL) return;
  const int64_t gb = gen_base[r];
  CellRec* R = rec + gb;
  uint8_t* sq = stq + 4 * gb;
  uint8_t* sv = stv + 9 * gb;
  const int64_t c0 = D.row_col_off[r], c1 = D.row_col_off[r + 1];
  // 1. data columns in column order: HBase timestamp, index, point count
  int k = 0;
  for (int64_t cc = c0; cc < c1; cc += 64) {
    const int64_t c = cc + lane;
    ColInfo ci{CT_SKIP, 0, 0, 0};
    if (c < c1) ci = col_info(D, c);
    const uint64_t dm = __ballot(ci.type != CT_SKIP);
    const int slot = k + __popcll(dm & ((1ULL << lane) - 1));
    if (ci.type != CT_SKIP) {
      sm.col.ts[slot] = D.col_ts ? D.col_ts[c] : c;
      sm.col.cidx[slot] = (int32_t)(c - c0);
      sm.col.base[slot] = (int32_t)(ci.type == CT_MULTI ? 0 : ci.cells);
    }
    uint64_t mm = __ballot(ci.type == CT_MULTI);
    while (mm) {
      const int b = __builtin_ctzll(mm);
      mm &= mm - 1;
      const int64_t col = cc + b;
      const int64_t qb = D.col_qoff[col], vb = D.col_voff[col];
      ColWalk w(D.qual + qb, D.col_qoff[col + 1] - qb, D.col_voff[col + 1] - vb);
      int64_t n = 0;
      while (w.step()) n += __popcll(w.mask);
      if (lane == 0) sm.col.base[k + __popcll(dm & ((1ULL << b) - 1))] = (int32_t)n;
    }
    k += __popcll(dm);
  }
  int k2 = 1;
  while (k2 < k) k2 <<= 1;
  for (int i = k + lane; i < k2; i += 64) {
    sm.col.ts[i] = INT64_MIN;
    sm.col.cidx[i] = INT32_MIN;
    sm.col.base[i] = 0;
  }
  wave_sync();
  // 2. column rank: bitonic sort by (timestamp desc, index desc)
  for (int kk = 2; kk <= k2; kk <<= 1)
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = lane; i < k2; i += 64) {
        const int l = i ^ j;
        if (l <= i) continue;
        const int64_t ti = sm.col.ts[i], tl = sm.col.ts[l];
        const int32_t ci_ = sm.col.cidx[i], cl = sm.col.cidx[l];
        // "before": newer first, then the later column
        const bool l_before_i = tl > ti || (tl == ti && cl > ci_);
        const bool i_before_l = ti > tl || (ti == tl && ci_ > cl);
        const bool up = (i & kk) == 0;
        if (up ? l_before_i : i_before_l) {
          sm.col.ts[i] = tl;
          sm.col.ts[l] = ti;
          sm.col.cidx[i] = cl;
          sm.col.cidx[l] = ci_;
          const int32_t b = sm.col.base[i];
          sm.col.base[i] = sm.col.base[l];
          sm.col.base[l] = b;
        }
      }
      wave_sync();
    }
  // 3. record bases in rank order (exclusive scan of the counts)
  {
    int32_t carry = 0;
    for (int i0 = 0; i0 < k; i0 += 64) {
      const int i = i0 + lane;
      const int32_t n = i < k ? sm.col.base[i] : 0;
      int32_t x = n;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
      }
      if (i < k) sm.col.base[i] = carry + x - n;
      carry += __shfl(x, 63);
    }
    if (lane == 0) sm.col.base[k] = carry;
    wave_sync();
  }
  const int n = sm.col.base[k];
  // 4. cell records, columns in rank order; append pairs in reverse arrival
  //    (the later of equal offsets first); a multi-point column whose
  //    offsets go back in time sends the row to the heap emulation
  int unsorted = 0, has_append = 0;
  for (int i0 = 0; i0 < k; i0 += 64) {
    const int i = i0 + lane;
    int type = CT_SKIP;
    int64_t c = 0;
    if (i < k) {
      c = c0 + sm.col.cidx[i];
      const int64_t ql = D.col_qoff[c + 1] - D.col_qoff[c];
      const uint8_t q0 = D.qual[D.col_qoff[c]];
      type = (ql & 1) ? CT_APPEND
                      : (ql == 2 || (ql == 4 && (q0 & 0xF0) == 0xF0)) ? CT_ONE
                                                                      : CT_MULTI;
    }
    if (type == CT_ONE) {  // one lane per single-point column
      const int64_t qb = D.col_qoff[c], ql = D.col_qoff[c + 1] - qb;
      const int64_t vb = D.col_voff[c], vl = D.col_voff[c + 1] - vb;
      CellRec x;
      x.col = i;
      x.qpos = qb;
      x.ql = (uint8_t)ql;
      if (ql == 2) {
        int vskip, bad;
        const uint8_t nf = fixup2(D.qual[qb + 1], D.val + vb, vl, vskip, bad);
        const int cur = (nf & 0x7) + 1;
        x.flags = RF_QFIX;
        x.qfix = nf;
        x.vpos = vb + vskip;
        x.vl = (uint8_t)cur;
        x.vav = (uint8_t)(cur <= vl - vskip ? cur : vl - vskip);
        if (cur > vl - vskip) x.flags |= RF_OVERRUN;
        x.off = (int32_t)((((uint32_t)D.qual[qb] << 8) | nf) >> 4) * 1000;
      } else {
        const uint32_t qv = ((uint32_t)D.qual[qb] << 24) |
                            ((uint32_t)D.qual[qb + 1] << 16) |
                            ((uint32_t)D.qual[qb + 2] << 8) | D.qual[qb + 3];
        const int cur = (int)(qv & 0x7) + 1;
        x.flags = RF_MS;
        x.qfix = 0;
        x.vpos = vb;
        x.vl = (uint8_t)cur;
        x.vav = (uint8_t)(cur <= vl ? cur : vl);
        if (cur > vl) x.flags |= RF_OVERRUN;
        x.off = qual_off_ms(qv, 1);
      }
      R[sm.col.base[i]] = x;
    }
    uint64_t om = __ballot(type == CT_MULTI || type == CT_APPEND);
    has_append |= __ballot(type == CT_APPEND) != 0;
    while (om) {
      const int b = __builtin_ctzll(om);
      om &= om - 1;
      const int ii = i0 + b;
      const int64_t cb = c0 + sm.col.cidx[ii];
      const int64_t qb = D.col_qoff[cb], vb = D.col_voff[cb];
      const int64_t ql = D.col_qoff[cb + 1] - qb, vl = D.col_voff[cb + 1] - vb;
      CellRec* out = R + sm.col.base[ii];
      if (ql & 1) {  // append: lane 0 walks the pairs
        if (lane == 0) {
          const int64_t np = sm.col.base[ii + 1] - sm.col.base[ii];
          int64_t p = 0;
          for (int64_t j = 0; j < np; ++j) {
            const uint8_t* e = D.val + vb + p;
            const int eql = (e[0] & 0xF0) == 0xF0 ? 4 : 2;
            uint32_t qv = 0;
            for (int t = 0; t < eql; ++t) qv = (qv << 8) | e[t];
            const int cur = (int)(qv & 0x7) + 1;
            CellRec x;
            x.qpos = vb + p;
            x.vpos = vb + p + eql;
            x.off = qual_off_ms(qv, eql == 4);
            x.col = ii;
            x.ql = (uint8_t)eql;
            x.vl = x.vav = (uint8_t)cur;
            x.flags = RF_QINVAL | RF_APPEND | (eql == 4 ? RF_MS : 0);
            x.qfix = 0;
            out[np - 1 - j] = x;
            p += eql + cur;
          }
        }
      } else {
        ColWalk w(D.qual + qb, ql, vl);
        bool hp = false;
        int32_t prev = 0;
        while (w.step()) {
          const int pl = lane_prev(w.mask, lane);
          int32_t po = __shfl(w.off, pl < 0 ? 0 : pl);
          const bool have = pl >= 0 || hp;
          if (pl < 0) po = prev;
          if (__ballot(w.cell && have && w.off < po)) unsorted = 1;
          if (w.cell) {
            CellRec x;
            x.qpos = qb + w.qo;
            x.vpos = vb + w.vo;
            x.off = w.off;
            x.col = ii;
            x.ql = (uint8_t)w.ql;
            x.vl = (uint8_t)w.vl;
            x.vav = (uint8_t)(w.vo + w.vl <= vl ? w.vl : vl - w.vo);
            x.flags = (w.ms ? RF_MS : 0) |
                      (w.vo + w.vl > vl ? RF_OVERRUN : 0);
            x.qfix = 0;
            out[w.k] = x;
          }
          if (w.mask) {
            prev = __shfl(w.off, 63 - __builtin_clzll(w.mask));
            hp = true;
          }
        }
      }
    }
  }
  // the records are read back by other lanes: device-scope fence (the
  // write-through L1 is invalidated)
  __threadfence();
  wave_sync();
  int64_t nq = 0, nv = 0, nk = 0;
  int ms_in = 0, s_in = 0, bad = 0;
  if (!unsorted) {
    // 5a. the heap order = sort by (offset, rank, position)
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int i = lane; i < n2; i += 64)
      sm.keys[i] = i < n ? ((uint64_t)(uint32_t)R[i].off << 32) | (uint32_t)i
                         : ~0ULL;
    wave_sync();
    for (int kk = 2; kk <= n2; kk <<= 1)
      for (int j = kk >> 1; j > 0; j >>= 1) {
        for (int i = lane; i < n2; i += 64) {
          const int l = i ^ j;
          if (l <= i) continue;
          const uint64_t a = sm.keys[i], b = sm.keys[l];
          const bool up = (i & kk) == 0;
          if (up ? b < a : a < b) {
            sm.keys[i] = b;
            sm.keys[l] = a;
          }
        }
        wave_sync();
      }
    merge_sorted(D, fix, R, n, sm.keys, sq, sv, nq, nv, nk, ms_in, s_in, bad);
  } else if (has_append) {
    // not reached by the write path or compaction: appended pairs next to a
    // compacted column whose offsets go back in time
    if (lane == 0) row_error(first_err, r, RS_UNSUPPORTED);
    if (lane == 0) {
      out_q[r] = 0;
      out_v[r] = 0;
    }
    return;
  } else {
    // 5b. heap emulation: per column head; each step the least (offset,
    //     rank) head pops (wave arg-min), lane 0 merges it
    for (int i = lane; i < k; i += 64) {
      const int32_t b0 = sm.col.base[i], b1 = sm.col.base[i + 1];
      sm.hp.head[i] = b0;
      sm.hp.end[i] = b1;
    }
    wave_sync();
    for (int i = lane; i < k; i += 64)
      sm.hp.hoff[i] = sm.hp.head[i] < sm.hp.end[i] ? R[sm.hp.head[i]].off : -1;
    wave_sync();
    bool have_prev = false;
    int32_t prev = 0;
    int64_t lvpos = 0;
    int lvl = 0, lvav = 0;
    for (int step = 0; step < n; ++step) {
      uint64_t best = ~0ULL;
      for (int i = lane; i < k; i += 64) {
        const int32_t o = sm.hp.hoff[i];
        if (o >= 0) {
          const uint64_t key = ((uint64_t)(uint32_t)o << 32) | (uint32_t)i;
          best = key < best ? key : best;
        }
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t y = __shfl_xor(best, d);
        best = y < best ? y : best;
      }
      if (best == ~0ULL) break;
      const int ci_ = (int)(uint32_t)best;
      const CellRec x = R[sm.hp.head[ci_]];
      if (lane == 0) {
        if (have_prev && x.off == prev) {
          if (!fix &&
              !bytes_equal_padded(D.val, x.vpos, x.vl, x.vav, lvpos, lvl, lvav))
            bad = 1;
        } else if (x.flags & RF_OVERRUN) {
          bad = 1;
        } else {
          write_cell(D, x, sq + nq, sv + nv);
          nq += x.ql;
          nv += x.vl;
          nk += 1;
          if (x.flags & RF_MS) ms_in = 1;
          else s_in = 1;
          prev = x.off;
          have_prev = true;
          lvpos = x.vpos;
          lvl = x.vl;
          lvav = x.vav;
        }
        const int32_t h = sm.hp.head[ci_] + 1;
        sm.hp.head[ci_] = h;
        sm.hp.hoff[ci_] = h < sm.hp.end[ci_] ? R[h].off : -1;
      }
      wave_sync();
      if (__builtin_amdgcn_readfirstlane(bad)) break;
    }
    nq = readlane_l(nq, 0);
    nv = readlane_l(nv, 0);
    nk = readlane_l(nk, 0);
    ms_in = __builtin_amdgcn_readfirstlane(ms_in);
    s_in = __builtin_amdgcn_readfirstlane(s_in);
    bad = __builtin_amdgcn_readfirstlane(bad);
  }
  finish_row(r, bad, nq, nv, nk, ms_in, s_in, sv, out_q, out_v, first_err);
}

// ------------------------------------------------------------- LARGE rows
// A row past the LDS caps (an hour of millisecond points written as single
// cells is up to 3.6 M columns) runs the same merge through global memory:
//   k_large_cols    its data columns, index order reversed, keyed by the
//                   HBase timestamp (descending) -> a stable segmented radix
//                   sort gives the rank order (newer cell first, then the
//                   later column: ColumnDatapointIterator.compareTo);
//   k_large_count   cells per ranked column (multi-point columns walked);
//                   an exclusive scan gives each column's record base;
//   k_large_recs    the cell records in rank order and their keys
//                   (offset << 32 | record index);
//   segmented radix sort of the keys = the heap order;
//   k_large_merge   merge_sorted + finish_row, one wavefront per row.
// A LARGE row holding a column whose cells go back in time (never written by
// the write path or compaction): that column's cells are keyed past every
// offset (kLargeUnsorted), so the sort leaves the in-order columns' cells
// merged in heap order and the unsorted columns' cells after them, column by
// column in rank order; k_large_merge then replays the heap over those
// streams (the merged in-order cells are one stream — popping the least head
// among in-order columns IS their merged order — and each unsorted column
// one more), up to 63 unsorted columns per row.
// sort key offset of a cell of an unsorted column (past every 22-bit ms
// offset; the segmented key sort runs over bits [0, kLargeKeyBits))
constexpr uint32_t kLargeUnsorted = 1u << 22;
constexpr int kLargeKeyBits = 55;

struct LargeWs {
  LargeSlots LS;
  uint64_t* ckey;     // [NC] rank keys
  int64_t* cidx;      // [NC] column index (sorted alongside)
  int64_t* cslot;     // [NC] slot of each ranked position
  int64_t* ccount;    // [NC + 1] cells per ranked column
  int64_t* cbase;     // [NC + 1] exclusive scan of ccount
  int* bad;           // [slots] unsorted columns seen
};

__global__ __launch_bounds__(256) void k_large_cols(
    RawDev D, LargeSlots LS, int64_t n_slots, uint64_t* __restrict__ ckey,
    int64_t* __restrict__ cidx, int64_t* __restrict__ cslot,
    int64_t* __restrict__ segb, int64_t* __restrict__ sege) {
  const int lane = LANE;
  const int64_t sl = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sl >= n_slots) return;
  const int64_t r = LS.row[sl], nc = LS.ncol[sl], cb = LS.cbase[sl];
  const int64_t c0 = D.row_col_off[r], c1 = D.row_col_off[r + 1];
  if (lane == 0) {
    segb[sl] = cb;
    sege[sl] = cb + nc;
  }
  int64_t k = 0;
  for (int64_t cc = c0; cc < c1; cc += 64) {
    const int64_t c = cc + lane;
    ColInfo ci{CT_SKIP, 0, 0, 0};
    if (c < c1) ci = col_info(D, c);
    const uint64_t dm = __ballot(ci.type != CT_SKIP);
    if (ci.type != CT_SKIP) {
      const int64_t kk = k + __popcll(dm & ((1ULL << lane) - 1));
      const int64_t pos = cb + (nc - 1 - kk);  // index order reversed
      const int64_t ts = D.col_ts ? D.col_ts[c] : c;
      // ascending key = descending timestamp (signed order)
      ckey[pos] = ~((uint64_t)ts ^ 0x8000000000000000ULL);
      cidx[pos] = c;
      cslot[pos] = sl;
    }
    k += __popcll(dm);
  }
}

// Cells of ranked columns [w*64, w*64+64) (mode 0: count; mode 1: write
// the records and keys at the scanned bases)
__global__ __launch_bounds__(256) void k_large_recs(
    RawDev D, LargeSlots LS, int64_t NC, const int64_t* __restrict__ cidx,
    const int64_t* __restrict__ cslot, const int64_t* __restrict__ gen_base,
    int64_t* __restrict__ ccount, const int64_t* __restrict__ cbase,
    CellRec* __restrict__ rec, uint64_t* __restrict__ rkey,
    int* __restrict__ bad, int mode) {
  const int lane = LANE;
  const int64_t p0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (p0 >= NC) return;
  const int64_t pos = p0 + lane;
  const bool in = pos < NC;
  int64_t c = 0, sl = 0, rbase = 0, rank = 0, base_in_row = 0;
  int type = CT_SKIP;
  ColInfo ci{CT_SKIP, 0, 0, 0};
  if (in) {
    c = cidx[pos];
    sl = cslot[pos];
    ci = col_info(D, c);
    type = ci.type;
    rank = pos - LS.cbase[sl];
    if (mode) {
      rbase = gen_base[LS.row[sl]];
      base_in_row = cbase[pos] - cbase[LS.cbase[sl]];
    }
  }
  auto key_of = [](int32_t off, int64_t i) {
    return ((uint64_t)(uint32_t)off << 32) | (uint64_t)(uint32_t)i;
  };
  if (type == CT_ONE || type == CT_APPEND) {
    if (!mode) ccount[pos] = ci.cells;
  }
  if (mode && type == CT_ONE) {
    const int64_t qb = D.col_qoff[c], ql = D.col_qoff[c + 1] - qb;
    const int64_t vb = D.col_voff[c], vl = D.col_voff[c + 1] - vb;
    CellRec x;
    x.col = (int32_t)rank;
    x.qpos = qb;
    x.ql = (uint8_t)ql;
    if (ql == 2) {
      int vskip, bd;
      const uint8_t nf = fixup2(D.qual[qb + 1], D.val + vb, vl, vskip, bd);
      const int cur = (nf & 0x7) + 1;
      x.flags = RF_QFIX;
      x.qfix = nf;
      x.vpos = vb + vskip;
      x.vl = (uint8_t)cur;
      x.vav = (uint8_t)(cur <= vl - vskip ? cur : vl - vskip);
      if (cur > vl - vskip) x.flags |= RF_OVERRUN;
      x.off = (int32_t)((((uint32_t)D.qual[qb] << 8) | nf) >> 4) * 1000;
    } else {
      const uint32_t qv = ((uint32_t)D.qual[qb] << 24) |
                          ((uint32_t)D.qual[qb + 1] << 16) |
                          ((uint32_t)D.qual[qb + 2] << 8) | D.qual[qb + 3];
      const int cur = (int)(qv & 0x7) + 1;
      x.flags = RF_MS;
      x.qfix = 0;
      x.vpos = vb;
      x.vl = (uint8_t)cur;
      x.vav = (uint8_t)(cur <= vl ? cur : vl);
      if (cur > vl) x.flags |= RF_OVERRUN;
      x.off = qual_off_ms(qv, 1);
    }
    rec[rbase + base_in_row] = x;
    rkey[rbase + base_in_row] = key_of(x.off, base_in_row);
  }
  uint64_t om = __ballot(type == CT_MULTI || (mode && type == CT_APPEND));
  while (om) {
    const int b = __builtin_ctzll(om);
    om &= om - 1;
    const int64_t cb = __shfl(c, b);
    const int64_t rb = __shfl(rbase, b), bir = __shfl(base_in_row, b);
    const int64_t rk = __shfl(rank, b), bsl = __shfl(sl, b);
    const int btype = __shfl(type, b);
    const int64_t qb = D.col_qoff[cb], vb = D.col_voff[cb];
    const int64_t ql = D.col_qoff[cb + 1] - qb, vl = D.col_voff[cb + 1] - vb;
    if (btype == CT_APPEND) {  // lane 0 walks the pairs (reverse arrival)
      if (lane == 0) {
        const int64_t np = cbase[p0 + b + 1] - cbase[p0 + b];
        int64_t p = 0;
        for (int64_t j = 0; j < np; ++j) {
          const uint8_t* e = D.val + vb + p;
          const int eql = (e[0] & 0xF0) == 0xF0 ? 4 : 2;
          uint32_t qv = 0;
          for (int t = 0; t < eql; ++t) qv = (qv << 8) | e[t];
          const int cur = (int)(qv & 0x7) + 1;
          CellRec x;
          x.qpos = vb + p;
          x.vpos = vb + p + eql;
          x.off = qual_off_ms(qv, eql == 4);
          x.col = (int32_t)rk;
          x.ql = (uint8_t)eql;
          x.vl = x.vav = (uint8_t)cur;
          x.flags = RF_QINVAL | RF_APPEND | (eql == 4 ? RF_MS : 0);
          x.qfix = 0;
          const int64_t i = bir + np - 1 - j;
          rec[rb + i] = x;
          rkey[rb + i] = key_of(x.off, i);
          p += eql + cur;
        }
      }
      continue;
    }
    ColWalk w(D.qual + qb, ql, vl);
    int64_t n = 0;
    bool hp = false;
    int32_t prev = 0;
    int unsorted = 0;
    while (w.step()) {
      if (mode) {
        const int pl = lane_prev(w.mask, lane);
        int32_t po = __shfl(w.off, pl < 0 ? 0 : pl);
        const bool have = pl >= 0 || hp;
        if (pl < 0) po = prev;
        if (__ballot(w.cell && have && w.off < po)) unsorted = 1;
        if (w.cell) {
          CellRec x;
          x.qpos = qb + w.qo;
          x.vpos = vb + w.vo;
          x.off = w.off;
          x.col = (int32_t)rk;
          x.ql = (uint8_t)w.ql;
          x.vl = (uint8_t)w.vl;
          x.vav = (uint8_t)(w.vo + w.vl <= vl ? w.vl : vl - w.vo);
          x.flags = (w.ms ? RF_MS : 0) | (w.vo + w.vl > vl ? RF_OVERRUN : 0);
          x.qfix = 0;
          rec[rb + bir + w.k] = x;
          rkey[rb + bir + w.k] = key_of(x.off, bir + w.k);
        }
        if (w.mask) {
          prev = __shfl(w.off, 63 - __builtin_clzll(w.mask));
          hp = true;
        }
      }
      n += __popcll(w.mask);
    }
    if (!mode && lane == 0) ccount[p0 + b] = n;
    if (mode && unsorted) {
      // its cells sort after every in-order cell, in column order
      for (int64_t i = lane; i < n; i += 64)
        rkey[rb + bir + i] =
            ((uint64_t)kLargeUnsorted << 32) | (uint64_t)(uint32_t)(bir + i);
      if (lane == 0) atomicOr(&bad[bsl], 1);
    }
  }
}

__global__ void k_large_segs(LargeSlots LS, int64_t n_slots,
                             const int64_t* __restrict__ gen_base,
                             const int64_t* __restrict__ gen_n,
                             int64_t* __restrict__ segb,
                             int64_t* __restrict__ sege) {
  const int64_t sl = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (sl >= n_slots) return;
  const int64_t r = LS.row[sl];
  segb[sl] = gen_base[r];
  sege[sl] = gen_base[r] + gen_n[r];
}

// The heap order of a row with unsorted columns (CompactionQueue.
// defaultMergeDataPoints pops the least (offset, rank) head,
// CompactionQueue.java:549-584): lane 0 holds the in-order stream's head,
// lane u the u-th unsorted column's; each step the wave's least head pops
// into perm (keys in merge_sorted's form).  Returns false past 63 unsorted
// columns.
DEV bool large_heap_order(const CellRec* R, const uint64_t* keys, int64_t n,
                          uint64_t* perm) {
  const int lane = LANE;
  // the unsorted tail [m, n): its cells carry the kLargeUnsorted offset
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if ((uint32_t)(keys[mid] >> 32) >= kLargeUnsorted) hi = mid;
    else lo = mid + 1;
  }
  const int64_t m = lo;
  // stream u >= 1: the tail's u-th run of one column (rank)
  int64_t head = lane == 0 ? 0 : -1, end = lane == 0 ? m : -1;
  {
    int64_t u = 1, a = m;
    while (a < n) {
      const int32_t col = R[(uint32_t)keys[a]].col;
      int64_t e = a + 1;
      while (e < n && R[(uint32_t)keys[e]].col == col) ++e;  // (lane-uniform)
      if (u >= 64) return false;
      if (lane == u) {
        head = a;
        end = e;
      }
      ++u;
      a = e;
    }
  }
  for (int64_t o = 0; o < n; ++o) {
    uint64_t k = ~0ULL;
    if (head >= 0 && head < end) {
      const CellRec& x = R[(uint32_t)keys[head]];
      k = ((uint64_t)(uint32_t)x.off << 32) | ((uint64_t)(uint32_t)x.col << 6) |
          (uint64_t)lane;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const uint64_t y = __shfl_xor(k, d);
      k = y < k ? y : k;
    }
    const int w = (int)(k & 63);
    if (lane == w) {
      const uint32_t idx = (uint32_t)keys[head];
      perm[o] = ((uint64_t)(uint32_t)R[idx].off << 32) | idx;
      ++head;
    }
  }
  return true;
}

__global__ __launch_bounds__(64) void k_large_merge(
    RawDev D, int fix, LargeSlots LS, const int64_t* __restrict__ gen_base,
    const int64_t* __restrict__ gen_n, const CellRec* __restrict__ rec,
    const uint64_t* __restrict__ rkey, const int* __restrict__ bad_in,
    uint64_t* __restrict__ perm, uint8_t* __restrict__ stq,
    uint8_t* __restrict__ stv, int64_t* __restrict__ out_q,
    int64_t* __restrict__ out_v, unsigned long long* first_err) {
  const int lane = LANE;
  const int64_t sl = blockIdx.x;
  const int64_t r = LS.row[sl];
  const int64_t gb = gen_base[r], n = gen_n[r];
  const uint64_t* order = rkey + gb;
  if (bad_in[sl]) {
    if (!large_heap_order(rec + gb, rkey + gb, n, perm + gb)) {
      if (lane == 0) {
        row_error(first_err, r, RS_UNSUPPORTED);
        out_q[r] = 0;
        out_v[r] = 0;
      }
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    order = perm + gb;
  }
  int64_t nq = 0, nv = 0, nk = 0;
  int ms_in = 0, s_in = 0, bad = 0;
  merge_sorted(D, fix, rec + gb, n, order, stq + 4 * gb, stv + 9 * gb, nq,
               nv, nk, ms_in, s_in, bad);
  finish_row(r, bad, nq, nv, nk, ms_in, s_in, stv + 9 * gb, out_q, out_v,
             first_err);
}

// ------------------------------------------------------------------ pack
// 16 bytes per lane (gfx950 global accesses at any byte address), the last
// partial 16 bytes one per lane
DEV void wave_copy(uint8_t* dst, const uint8_t* src, int64_t n) {
  const int lane = LANE;
  for (int64_t i = (int64_t)lane * 16; i + 16 <= n; i += 64 * 16)
    *reinterpret_cast<uint4*>(dst + i) =
        *reinterpret_cast<const uint4*>(src + i);
  for (int64_t j = (n & ~(int64_t)15) + lane; j < n; j += 64) dst[j] = src[j];
}

// Can the compacted output alias the input pools?  Yes when every kept row
// is VERBATIM and the kept columns sit in the input pools exactly as the
// packed output would lay them out, at one byte shift per pool (a scanner's
// rows of single compacted columns, back to back): acc[0..1] min / max of
// the qualifier shift, acc[2..3] of the value shift, acc[4] != 0 when some
// kept row is not VERBATIM.  One thread per row.
__global__ __launch_bounds__(256) void k_rows_alias(
    RawDev D, const uint8_t* __restrict__ kind, const int64_t* __restrict__ lone,
    const int64_t* __restrict__ oq_off, const int64_t* __restrict__ ov_off,
    unsigned long long* acc) {
  // grid-stride over the rows, reduced per workgroup: one set of atomics per
  // workgroup (same-address atomics from every wave serialise)
  int64_t dq = INT64_MAX, dv = INT64_MAX, eq = INT64_MIN, ev = INT64_MIN;
  int other = 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < D.R;
       r += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t kd = kind[r];
    if (kd == RK_VERBATIM) {
      const int64_t c = lone[r];
      const int64_t x = D.col_qoff[c] - oq_off[r], y = D.col_voff[c] - ov_off[r];
      dq = min(dq, x);
      eq = max(eq, x);
      dv = min(dv, y);
      ev = max(ev, y);
    } else if (kd != RK_EMPTY) {
      other = 1;
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    dq = min(dq, (int64_t)__shfl_xor(dq, d));
    dv = min(dv, (int64_t)__shfl_xor(dv, d));
    eq = max(eq, (int64_t)__shfl_xor(eq, d));
    ev = max(ev, (int64_t)__shfl_xor(ev, d));
    other |= __shfl_xor(other, d);
  }
  __shared__ int64_t red[4][5];
  const int wv = threadIdx.x >> 6;
  if (LANE == 0) {
    red[wv][0] = dq; red[wv][1] = eq; red[wv][2] = dv; red[wv][3] = ev;
    red[wv][4] = other;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
      dq = min(dq, red[i][0]); eq = max(eq, red[i][1]);
      dv = min(dv, red[i][2]); ev = max(ev, red[i][3]);
      other |= (int)red[i][4];
    }
    // shifts are >= 0: the output packs a subset of the input in order
    if (dq != INT64_MAX) {
      atomicMin(&acc[0], (unsigned long long)dq);
      atomicMax(&acc[1], (unsigned long long)eq);
      atomicMin(&acc[2], (unsigned long long)dv);
      atomicMax(&acc[3], (unsigned long long)ev);
    }
    if (other) atomicOr(&acc[4], 1ULL);
  }
}

// The per-row arrays of an aliased output (thread per row; no bytes move).
// k_rows_shape: the storage rows' shapes only (no qualifier byte read) —
// can the query take every row verbatim?  Each row one column (no append /
// annotation column beside it) of an even qualifier length, with value
// bytes; rows of a series with strictly increasing base
// times (Span.addRow then keeps them as they are, Span.java:177-220) and
// series in order.  What compaction would still change inside such a
// column (offsets out of order or repeated, a second qualifier width,
// value lengths that do not add up) the cells fold checks as it streams
// the points (Params.check_order); any miss re-runs the full path.
__global__ __launch_bounds__(256) void k_rows_shape(
    RawDev D, const int64_t* __restrict__ row_series,
    const int64_t* __restrict__ row_base_s, int* __restrict__ bad) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int b = 0;
  if (r < D.R) {
    const int64_t c = D.row_col_off[r];
    const int64_t ql = D.col_qoff[c + 1] - D.col_qoff[c];
    const int64_t vl = D.col_voff[c + 1] - D.col_voff[c];
    b |= D.row_col_off[r + 1] - c != 1;
    // (a single 2-byte cell is verbatim unless checkForFixup changes it:
    // then its value bytes do not add up to its qualifier's length, which
    // the fold checks)
    b |= ql < 2 || (ql & 1) || vl < 1;
    if (r > 0) {
      const int64_t s0 = row_series[r - 1], s1 = row_series[r];
      b |= s1 < s0 || (s1 == s0 && row_base_s[r] <= row_base_s[r - 1]);
    }
  }
  if (__ballot(b) && LANE == 0) atomicOr(bad, 1);
}

__global__ __launch_bounds__(256) void k_rows_meta(
    int64_t R, const int64_t* __restrict__ row_series,
    const int64_t* __restrict__ row_base_s, const uint8_t* __restrict__ kind,
    const int64_t* __restrict__ oq_off, const int64_t* __restrict__ ov_off,
    const int64_t* __restrict__ k_off, int64_t* __restrict__ o_series,
    int64_t* __restrict__ o_base, int64_t* __restrict__ o_qoff,
    int64_t* __restrict__ o_voff) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R || kind[r] == RK_EMPTY) return;
  const int64_t k = k_off[r];
  if (o_series) o_series[k] = row_series ? row_series[r] : 0;
  o_base[k] = row_base_s[r];
  o_qoff[k] = oq_off[r];
  o_voff[k] = ov_off[r];
}

__global__ __launch_bounds__(256) void k_rows_write(
    RawDev D, int fix, const int64_t* __restrict__ row_series,
    const int64_t* __restrict__ row_base_s, const uint8_t* __restrict__ kind,
    const int64_t* __restrict__ lone, const int64_t* __restrict__ gen_base,
    const uint8_t* __restrict__ stq, const uint8_t* __restrict__ stv,
    const int64_t* __restrict__ out_q, const int64_t* __restrict__ out_v,
    const int64_t* __restrict__ oq_off, const int64_t* __restrict__ ov_off,
    const int64_t* __restrict__ k_off, int64_t* __restrict__ o_series,
    int64_t* __restrict__ o_base, int64_t* __restrict__ o_qoff,
    uint8_t* __restrict__ o_qual, int64_t* __restrict__ o_voff,
    uint8_t* __restrict__ o_val) {
  const int lane = LANE;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= D.R) return;
  const uint8_t kd = kind[r];
  if (kd == RK_EMPTY) return;
  const int64_t k = k_off[r];
  uint8_t* dq = o_qual + oq_off[r];
  uint8_t* dv = o_val + ov_off[r];
  if (lane == 0) {
    if (o_series) o_series[k] = row_series ? row_series[r] : 0;
    o_base[k] = row_base_s[r];
    o_qoff[k] = oq_off[r];
    o_voff[k] = ov_off[r];
  }
  if (kd == RK_VERBATIM) {
    const int64_t c = lone[r];
    wave_copy(dq, D.qual + D.col_qoff[c], out_q[r]);
    wave_copy(dv, D.val + D.col_voff[c], out_v[r]);
  } else if (kd == RK_LONE) {
    lone_walk<true>(D, lone[r], fix, dq, dv);
  } else {
    const int64_t gb = gen_base[r];
    wave_copy(dq, stq + 4 * gb, out_q[r]);
    wave_copy(dv, stv + 9 * gb, out_v[r]);
  }
}

// ------------------------------------------------------------ span assembly
// RowSeq.size / timestamp(i) over one compacted row (RowSeq.java:338-420)
DEV int64_t rs_size(const uint8_t* q, int64_t ql, const uint8_t* v,
                    int64_t vl) {
  if (vl > 0 && (v[vl - 1] & 1)) {
    int64_t n = 0;
    for (int64_t i = 0; i < ql; i += 2) {
      if ((q[i] & 0xF0) == 0xF0) i += 2;
      ++n;
    }
    return n;
  }
  if (ql > 0 && (q[0] & 0xF0) == 0xF0) return ql / 4;
  return ql / 2;
}

DEV int64_t rs_ts(int64_t base, const uint8_t* q, int64_t ql, const uint8_t* v,
                  int64_t vl, int64_t i) {
  int64_t o = -1;
  if (vl > 0 && (v[vl - 1] & 1)) {
    int64_t kk = 0;
    for (int64_t idx = 0; idx < ql; idx += 2) {
      if (kk == i) {
        o = idx;
        break;
      }
      if ((q[idx] & 0xF0) == 0xF0) idx += 2;
      ++kk;
    }
  } else if (ql > 0 && (q[0] & 0xF0) == 0xF0) {
    o = i * 4;
  } else {
    o = i * 2;
  }
  if (o < 0 || o + 2 > ql) return INT64_MIN;
  if ((q[o] & 0xF0) == 0xF0) {
    if (o + 4 > ql) return INT64_MIN;
    const uint32_t x = ((uint32_t)q[o] << 24) | ((uint32_t)q[o + 1] << 16) |
                       ((uint32_t)q[o + 2] << 8) | q[o + 3];
    return base * 1000 + qual_off_ms(x, 1);
  }
  const uint32_t x = ((uint32_t)q[o] << 8) | q[o + 1];
  return (base + qual_off_ms(x, 0) / 1000) * 1000;
}

// One RowSeq of a replayed span: its bytes live in the input or the arena
struct SpanSeq {
  int64_t base;
  const uint8_t* q;
  const uint8_t* v;
  int64_t ql, vl;
};

// a series takes the replay unless its rows' base times strictly increase
__global__ __launch_bounds__(256) void k_span_plan(
    CellsDev C, int64_t S, const int64_t* __restrict__ series_row,
    uint8_t* __restrict__ slow, int64_t* __restrict__ arena_sz,
    int64_t* __restrict__ o_rows, int64_t* __restrict__ o_q,
    int64_t* __restrict__ o_v, int* err_word) {
  const int lane = LANE;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= S) return;
  const int64_t r0 = series_row[s], r1 = series_row[s + 1];
  int bad_order = 0, empty = 0;
  for (int64_t r = r0 + lane; r < r1; r += 64) {
    if (C.qual_off[r + 1] - C.qual_off[r] < 2) empty = 1;
    if (r > r0 && C.row_base_s[r] <= C.row_base_s[r - 1]) bad_order = 1;
  }
  const bool sl = __ballot(bad_order) != 0;
  if (__ballot(empty) && lane == 0) atomicOr(err_word, 1);
  if (lane == 0) {
    const int64_t nr = r1 - r0;
    const int64_t L = (C.qual_off[r1] - C.qual_off[r0]) +
                      (C.val_off[r1] - C.val_off[r0]);
    slow[s] = sl;
    // two halves of 2 (L + rows) + 64 bytes, then the RowSeq table
    arena_sz[s] = sl ? ((2 * (2 * (L + nr) + 64) + nr * (int64_t)sizeof(SpanSeq) +
                         2 * nr * 8 + 255) & ~(int64_t)255)
                     : 0;
    o_rows[s] = nr;
    o_q[s] = C.qual_off[r1] - C.qual_off[r0];
    o_v[s] = C.val_off[r1] - C.val_off[r0];
  }
}

// Span.addRow replay of one series by lane 0 (the rare path).  Merged
// RowSeqs are allocated from the current half of the series' arena; when it
// fills, the live ones move to the other half (live bytes <= input bytes +
// one meta byte per merge, so a half always takes the next merge).
__global__ __launch_bounds__(64) void k_span_replay(
    CellsDev C, int64_t S, const int64_t* __restrict__ series_row,
    const uint8_t* __restrict__ slow, const int64_t* __restrict__ arena_off,
    uint8_t* __restrict__ arena, int64_t* __restrict__ o_rows,
    int64_t* __restrict__ o_q, int64_t* __restrict__ o_v) {
  const int64_t s = blockIdx.x;
  if (s >= S || !slow[s] || threadIdx.x != 0) return;
  const int64_t r0 = series_row[s], r1 = series_row[s + 1], nr = r1 - r0;
  const int64_t L = (C.qual_off[r1] - C.qual_off[r0]) +
                    (C.val_off[r1] - C.val_off[r0]);
  const int64_t H = 2 * (L + nr) + 64;
  uint8_t* A = arena + arena_off[s];
  SpanSeq* rs = reinterpret_cast<SpanSeq*>(A + 2 * H);
  int64_t* order = reinterpret_cast<int64_t*>(rs + nr);
  int half = 0;
  int64_t bump = 0;
  auto in_half = [&](const uint8_t* p, int h) {
    return p >= A + h * H && p < A + (h + 1) * H;
  };
  int64_t n = 0;
  for (int64_t r = r0; r < r1; ++r) {
    const uint8_t* q = C.qual + C.qual_off[r];
    const int64_t ql = C.qual_off[r + 1] - C.qual_off[r];
    const uint8_t* v = C.val + C.val_off[r];
    const int64_t vl = C.val_off[r + 1] - C.val_off[r];
    const int64_t base = C.row_base_s[r];
    int64_t target = -1;
    if (n) {
      const SpanSeq& last = rs[n - 1];
      const int64_t last_ts =
          rs_ts(last.base, last.q, last.ql, last.v, last.vl,
                rs_size(last.q, last.ql, last.v, last.vl) - 1);
      if (last_ts >= rs_ts(base, q, ql, v, vl, 0))
        for (int64_t j = 0; j < n; ++j)
          if (rs[j].base == base) {
            target = j;
            break;
          }
    }
    if (target < 0) {
      rs[n++] = SpanSeq{base, q, v, ql, vl};
      continue;
    }
    SpanSeq& T = rs[target];
    const int64_t need = T.ql + ql + T.vl + vl + 2;
    if (bump + need > H) {  // move the live RowSeqs to the other half
      const int nh = half ^ 1;
      int64_t nb = 0;
      uint8_t* dst = A + nh * H;
      for (int64_t j = 0; j < n; ++j) {
        if (in_half(rs[j].q, half)) {
          for (int64_t b = 0; b < rs[j].ql; ++b) dst[nb + b] = rs[j].q[b];
          rs[j].q = dst + nb;
          nb += rs[j].ql;
        }
        if (in_half(rs[j].v, half)) {
          for (int64_t b = 0; b < rs[j].vl; ++b) dst[nb + b] = rs[j].v[b];
          rs[j].v = dst + nb;
          nb += rs[j].vl;
        }
      }
      half = nh;
      bump = nb;
    }
    uint8_t* mq = A + half * H + bump;
    uint8_t* mv = mq + T.ql + ql;
    // RowSeq.addRow: two-pointer merge by offset, the incoming duplicate
    // dropped
    int64_t ri = 0, li = 0, mi = 0, rvi = 0, lvi = 0, mvi = 0;
    auto qlen_at = [](const uint8_t* qq, int64_t o) {
      return (qq[o] & 0xF0) == 0xF0 ? 4 : 2;
    };
    auto vlen_at = [&](const uint8_t* qq, int64_t o) {
      return (qq[o + qlen_at(qq, o) - 1] & 0x7) + 1;
    };
    auto off_at = [&](const uint8_t* qq, int64_t o) -> int32_t {
      if ((qq[o] & 0xF0) == 0xF0)
        return qual_off_ms(((uint32_t)qq[o] << 24) | ((uint32_t)qq[o + 1] << 16) |
                               ((uint32_t)qq[o + 2] << 8) | qq[o + 3],
                           1);
      return qual_off_ms(((uint32_t)qq[o] << 8) | qq[o + 1], 0);
    };
    auto take = [&](const uint8_t* qq, int64_t& qi, const uint8_t* vv,
                    int64_t& vi) {
      const int a = qlen_at(qq, qi), b = vlen_at(qq, qi);
      for (int t = 0; t < b; ++t) mv[mvi + t] = vv[vi + t];
      for (int t = 0; t < a; ++t) mq[mi + t] = qq[qi + t];
      vi += b;
      mvi += b;
      qi += a;
      mi += a;
    };
    int64_t guard = 0;
    while ((ri < ql || li < T.ql) && guard++ < ql + T.ql + 4) {
      if (ri >= ql) {
        take(T.q, li, T.v, lvi);
      } else if (li >= T.ql) {
        take(q, ri, v, rvi);
      } else {
        const int32_t a = off_at(q, ri), b = off_at(T.q, li);
        if (a == b) {
          rvi += vlen_at(q, ri);
          ri += qlen_at(q, ri);
        } else if (a < b) {
          take(q, ri, v, rvi);
        } else {
          take(T.q, li, T.v, lvi);
        }
      }
    }
    const uint8_t meta =
        ((T.vl > 0 && (T.v[T.vl - 1] & 1)) || (vl > 0 && (v[vl - 1] & 1))) ? 1
                                                                          : 0;
    // values were laid out after the qualifier bytes of both inputs: move
    // them up behind the merged qualifiers
    uint8_t* fv = mq + mi;
    for (int64_t t = 0; t < mvi; ++t) fv[t] = mv[t];
    fv[mvi] = meta;
    T.q = mq;
    T.ql = mi;
    T.v = fv;
    T.vl = mvi + 1;
    bump += mi + mvi + 1;
  }
  // checkRowOrder: stable sort by base time
  for (int64_t j = 0; j < n; ++j) order[j] = j;
  for (int64_t a = 1; a < n; ++a) {
    const int64_t x = order[a];
    int64_t b = a - 1;
    while (b >= 0 && rs[order[b]].base > rs[x].base) {
      order[b + 1] = order[b];
      --b;
    }
    order[b + 1] = x;
  }
  int64_t tq = 0, tv = 0;
  for (int64_t j = 0; j < n; ++j) {
    tq += rs[j].ql;
    tv += rs[j].vl;
  }
  o_rows[s] = n;
  o_q[s] = tq;
  o_v[s] = tv;
}

// rows of every series at their scanned output positions
__global__ __launch_bounds__(256) void k_span_write(
    CellsDev C, int64_t S, const int64_t* __restrict__ series_row,
    const uint8_t* __restrict__ slow, const int64_t* __restrict__ arena_off,
    const uint8_t* __restrict__ arena, const int64_t* __restrict__ row_off,
    const int64_t* __restrict__ q_off, const int64_t* __restrict__ v_off,
    int64_t* __restrict__ o_series, int64_t* __restrict__ o_base,
    int64_t* __restrict__ o_qoff, uint8_t* __restrict__ o_qual,
    int64_t* __restrict__ o_voff, uint8_t* __restrict__ o_val) {
  const int lane = LANE;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= S) return;
  const int64_t r0 = series_row[s], r1 = series_row[s + 1];
  int64_t k = row_off[s], qo = q_off[s], vo = v_off[s];
  if (!slow[s]) {
    const int64_t dq = qo - C.qual_off[r0], dv = vo - C.val_off[r0];
    for (int64_t r = r0 + lane; r < r1; r += 64) {
      o_series[k + r - r0] = s;
      o_base[k + r - r0] = C.row_base_s[r];
      o_qoff[k + r - r0] = C.qual_off[r] + dq;
      o_voff[k + r - r0] = C.val_off[r] + dv;
    }
    wave_copy(o_qual + qo, C.qual + C.qual_off[r0],
              C.qual_off[r1] - C.qual_off[r0]);
    wave_copy(o_val + vo, C.val + C.val_off[r0], C.val_off[r1] - C.val_off[r0]);
    return;
  }
  const int64_t nr = r1 - r0;
  const int64_t L = (C.qual_off[r1] - C.qual_off[r0]) +
                    (C.val_off[r1] - C.val_off[r0]);
  const int64_t H = 2 * (L + nr) + 64;
  const uint8_t* A = arena + arena_off[s];
  const SpanSeq* rs = reinterpret_cast<const SpanSeq*>(A + 2 * H);
  const int64_t* order = reinterpret_cast<const int64_t*>(rs + nr);
  // the replay's row count is this series' share of row_off
  const int64_t n = row_off[s + 1] - row_off[s];
  for (int64_t j = 0; j < n; ++j) {
    const SpanSeq x = rs[order[j]];
    if (lane == 0) {
      o_series[k + j] = s;
      o_base[k + j] = x.base;
      o_qoff[k + j] = qo;
      o_voff[k + j] = vo;
    }
    wave_copy(o_qual + qo, x.q, x.ql);
    wave_copy(o_val + vo, x.v, x.vl);
    qo += x.ql;
    vo += x.vl;
  }
}

#endif  // OTSDB_DS_TU

}  // namespace otsdb
