// cellfold.hip — the ordered group fold (fold.hip) fed straight from
// compacted columns: RowSeq decode (RowSeq.java:552-643, Internal.java:
// 621-690) inside the Downsampler -> AggregationIterator pass, no columnar
// copy and no series rows.
//
// Point stream.  The rows of a series are contiguous in the qualifier and
// value pools (qual_off / val_off are exclusive prefix offsets and rows are
// grouped by series), so a series whose rows all use one qualifier width qw
// is ONE qualifier stream: point p's qualifier is at qual_off[r0] + qw*p,
// whatever row it belongs to.  The fold streams it in steps of 64*K points
// that cross storage rows freely (k_bucketize_cells went one row per step,
// 360 points at @10 s, paying the per-step scan / carry / bookkeeping for
// each).  Each lane takes K consecutive points: one 16-byte qualifier load
// (2-byte qualifiers; two for 4-byte ms ones) and its K values straight from
// the value pool with unaligned 16-byte loads (gfx950 global loads at byte
// offsets run at ~95 % of aligned bandwidth, tools/unaligned_bw.hip).
//
// Rows inside a step.  A value's byte address is the row's val_off plus the
// lengths of the points before it in the row; the meta byte a multi-value
// column ends with (CompactionQueue.java:594-616) sits between rows.  A step
// holds at most three rows and every row wholly inside it has >= K points,
// so a lane's K points cross at most one row boundary: its values are one
// contiguous run with at most one skipped byte, cut out with byte-align
// funnels.  The row metadata of 64 rows at a time lives one row per lane.
//
// Value widths.  Qualifier flags give each point's length and type
// (Internal.getValueLengthFromQualifier / getFlagsFromQualifier).  The step
// loads the values speculatively with the previous step's length; a step
// whose flags are all equal (a series of one type: what compaction writes
// for doubles) decodes from those registers; a different uniform length
// reloads; mixed lengths (longs stored in 1/2/4/8 bytes) take per-point
// loads at prefix-summed offsets.
//
// Checks (Internal.extractDataPoints, Internal.java:307-321).  Every row
// boundary the stream crosses checks that the row's value bytes added up
// (the cursor lands on the next row's val_off); illegal value lengths are
// corrupt (ERR_CORRUPT_CELL).  A row whose qualifier width differs from the
// series' (MS_MIXED_COMPACT columns, or second and ms rows in one series)
// raises ERR_CELLS_GENERIC: the engine then rewrites the batch's qualifiers
// with one width (k_requal, decode.hip) and runs the fold again; what still
// does not fit (a series pool past 2^30 bytes) is decoded into columns and
// takes the columnar pipeline.  The fold itself is compiled once per
// qualifier width (QW) and launched with the width k_cells_prep saw.
#pragma once
#include "fold.hip"

namespace otsdb {

// ---------------------------------------------------------------- prep
// k_cells_prep: one thread per series.  What k_prep derives from columnar
// timestamps (SpanGroup.add filter SpanGroup.java:321-338, the seek and stop
// bounds, the first bucket past the window), in the series' point numbering,
// plus the stream's starting cursor: the row holding point lo and the byte
// offset of its value.
DEV uint32_t cells_qual_at(const CellsDev& C, int64_t qa, int qw) {
  const uint8_t* q = C.qual + qa;
  return qw == 2 ? ((uint32_t)q[0] << 8) | q[1]
                 : ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) |
                       ((uint32_t)q[2] << 8) | q[3];
}

template <class M>
__global__ __launch_bounds__(256) void k_cells_prep(Params P, CellsFold CF,
                                                    int64_t S, SeriesMeta SM,
                                                    int* err_word) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const CellsDev& C = CF.C;
  const int64_t r0 = CF.series_row[s], r1 = CF.series_row[s + 1];
  auto store = [&](bool keep, int64_t lo, int64_t hi, int64_t rlo,
                   int64_t vlo, int qw, int vl0, uint8_t of_has,
                   int64_t of_ts, double of_val) {
    SM.keep[s] = keep;
    SM.lo[s] = lo;
    SM.hi[s] = hi;
    SM.kf[s] = 0;
    SM.kl[s] = -1;
    SM.of_has[s] = of_has;
    SM.of_ts[s] = of_ts;
    SM.of_val[s] = of_val;
    CF.rlo[s] = rlo;
    CF.vlo[s] = vlo;
    CF.qw[s] = (uint8_t)qw;
    CF.vl0[s] = (uint8_t)vl0;
  };
  if (r0 >= r1) {
    store(false, 0, 0, r0, 0, 2, 8, 0, 0, 0.0);
    return;
  }
  const int64_t qb = C.qual_off[r0];
  if (C.qual_off[r0 + 1] <= qb) {  // an empty first row
    atomicOr(err_word, ERR_CELLS_GENERIC);
    store(false, 0, 0, r0, 0, 2, 8, 0, 0, 0.0);
    return;
  }
  const int qw = (C.qual[qb] & 0xF0) == 0xF0 ? 4 : 2;
  const int qsh = qw == 4 ? 2 : 1;
  // a row the stream cannot number with the series' width: the generic
  // decode takes the batch
  auto row_ok = [&](int64_t r) {
    const int64_t a = C.qual_off[r], l = C.qual_off[r + 1] - a;
    if (l <= 0 || (l & (qw - 1))) return false;
    return ((C.qual[a] & 0xF0) == 0xF0 ? 4 : 2) == qw;
  };
  auto generic = [&]() {
    atomicOr(err_word, ERR_CELLS_GENERIC);
    store(false, 0, 0, r0, 0, qw, 8, 0, 0, 0.0);
  };
  if (!row_ok(r0) || !row_ok(r1 - 1)) return generic();
  // the stream indexes a series' pools with 32-bit offsets
  if (C.qual_off[r1] - qb >= (1LL << 30) ||
      C.val_off[r1] - C.val_off[r0] >= (1LL << 30))
    return generic();
  const int64_t Ns = (C.qual_off[r1] - qb) >> qsh;
  // row holding point p: the last r in [r0, r1) with qual_off[r] <= qb+qw*p
  auto row_of = [&](int64_t p) {
    int64_t a = r0, b = r1 - 1;
    const int64_t x = qb + qw * p;
    while (a < b) {
      const int64_t m = (a + b + 1) >> 1;
      if (C.qual_off[m] <= x) a = m;
      else b = m - 1;
    }
    return a;
  };
  auto ts_at = [&](int64_t p, int64_t r) {
    return qual_ts(C.row_base_s[r] * 1000, qw, cells_qual_at(C, qb + qw * p, qw));
  };
  const int64_t t_first = ts_at(0, r0), t_last = ts_at(Ns - 1, r1 - 1);
  if (!(t_first <= P.end_ms && t_last >= P.start_ms)) {
    if (P.check_order) atomicOr(err_word, ERR_SPEC_MISS);
    store(false, 0, 0, r0, C.val_off[r0], qw, 8, 0, 0, 0.0);
    return;
  }
  bool bad = false;
  // first point at or after a (a's timestamp known < t unless a == 0) with
  // ts >= t
  auto lower = [&](int64_t a, int64_t t) -> int64_t {
    if (a >= Ns) return Ns;
    if (a == 0 && t_first >= t) return 0;
    if (t_last < t) return Ns;
    int64_t lo = a, hi = Ns - 1;  // ts(hi) >= t
    while (lo < hi) {
      const int64_t m = lo + ((hi - lo) >> 1);
      const int64_t r = row_of(m);
      bad |= !row_ok(r);
      if (ts_at(m, r) < t) lo = m + 1;
      else hi = m;
    }
    return lo;
  };
  const int64_t lo = lower(0, P.seek_ts);
  const int64_t hi = lower(lo, P.stop_ts);
  if (bad) return generic();
  // the stream's cursor at point lo: its row and value byte offset
  const int64_t rlo = lo < Ns ? row_of(lo) : r1 - 1;
  if (lo < Ns && !row_ok(rlo)) return generic();
  int64_t vlo = C.val_off[rlo];
  const int64_t ps_lo = (C.qual_off[rlo] - qb) >> qsh;
  for (int64_t i = ps_lo; i < lo; ++i)
    vlo += (cells_qual_at(C, qb + qw * i, qw) & 0x7) + 1;
  const int vl0 =
      lo < Ns ? (int)(cells_qual_at(C, qb + qw * lo, qw) & 0x7) + 1 : 8;
  // the first bucket past the window (NONE fill): its downsampled value,
  // from the points in order across rows (k_prep's of_val)
  uint8_t of_has = 0;
  int64_t of_ts = 0;
  double of_val = 0.0;
  if (!P.run_all && P.fill == 0 && hi < Ns) {
    int64_t r = row_of(hi);
    if (!row_ok(r)) return generic();
    const int64_t t = ts_at(hi, r);
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
      const int64_t vend = C.val_off[C.R];
      int64_t voff = C.val_off[r];
      for (int64_t i = (C.qual_off[r] - qb) >> qsh; i < hi; ++i)
        voff += (cells_qual_at(C, qb + qw * i, qw) & 0x7) + 1;
      int64_t next_row = r + 1 < r1 ? (C.qual_off[r + 1] - qb) >> qsh : Ns;
      M st = M::init();
      for (int64_t i = hi; i < Ns; ++i) {
        if (i == next_row) {
          ++r;
          if (!row_ok(r)) return generic();
          voff = C.val_off[r];
          next_row = r + 1 < r1 ? (C.qual_off[r + 1] - qb) >> qsh : Ns;
        }
        const uint32_t q = cells_qual_at(C, qb + qw * i, qw);
        if (qual_ts(C.row_base_s[r] * 1000, qw, q) >= e) break;
        const int l = (int)(q & 0x7) + 1;
        st.push(bits_to_double(
            dbits_of(load_be(C.val, voff, l, vend), l, (q & 0x8) != 0)));
        voff += l;
      }
      int e2 = 0;
      of_val = st.finish(&e2);
      of_has = 1;
    }
  }
  // verbatim storage rows: every point of the series must be streamed (and
  // so checked for order) by the fold
  if (P.check_order && (lo != 0 || hi != Ns)) atomicOr(err_word, ERR_SPEC_MISS);
  if (CF.wide) atomicOr(CF.wide, qw == 4 ? 1 : 2);
  store(true, lo, hi, rlo, vlo, qw, vl0, of_has, of_ts, of_val);
}

// ------------------------------------------------------------- uniform
// k_cells_uniform: one wavefront per series, after k_cells_prep.  A kept
// series is uniform when every row of it is one column of the series'
// qualifier width whose value bytes add up to (points x the length its
// first qualifier states) + the meta byte a multi-point column ends with
// (CompactionQueue.java:594-616, read back by RowSeq.java:552-643): facts of
// the row offsets alone, read coalesced 64 rows a pass — what compaction
// writes for a series of one value type.  The uniform fold then needs no
// value-length logic and no row-end checks per step; it verifies only that
// each streamed qualifier carries the series' width and flags.  Any other
// series (a row that does not add up, an illegal length, an empty row)
// makes the engine launch the general fold for the batch, which decodes
// point by point and raises the reference's errors.
template <class M>
__global__ __launch_bounds__(256) void k_cells_uniform(CellsFold CF, int64_t S,
                                                       SeriesMeta SM) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= S) return;
  const int lane = LANE;
  if (!SM.keep[s]) {
    if (lane == 0) CF.uf[s] = 0xFF;
    return;
  }
  const CellsDev& C = CF.C;
  const int64_t r0 = CF.series_row[s], r1 = CF.series_row[s + 1];
  const int qw = CF.qw[s], qsh = qw == 4 ? 2 : 1;
  const uint32_t f = C.qual[C.qual_off[r0] + qw - 1] & 0xFu;
  const int vl = (int)(f & 7) + 1;
  const bool legal = (f & 8) ? (vl == 4 || vl == 8)
                             : (vl == 1 || vl == 2 || vl == 4 || vl == 8);
  const int vsh = vl == 1 ? 0 : (vl == 2 ? 1 : (vl == 4 ? 2 : 3));
  bool bad = !legal;
  for (int64_t r = r0 + lane; r < r1; r += 64) {
    const int64_t ql = C.qual_off[r + 1] - C.qual_off[r];
    const int64_t vb = C.val_off[r + 1] - C.val_off[r];
    const int64_t n = ql >> qsh;
    bad |= ql <= 0 || (ql & (qw - 1)) != 0 ||
           vb != (n << vsh) + (n > 1 ? 1 : 0);
  }
  const bool ok = __ballot(bad) == 0;
  if (lane == 0) {
    CF.uf[s] = ok ? (uint8_t)f : (uint8_t)0xFF;
    if (!ok) atomicOr(CF.wide, 4);
  }
}

// ------------------------------------------------------------ fold prep
// k_cells_fold_prep: one thread per (series, inner window boundary j) of a
// grid wider than one fold window — k_fold_prep's WinCtx (the first point of
// window j, the series' real buckets either side, folded sequentially from
// the points like the Downsampler does) plus the cells stream's cursor there
// (row, value byte offset, value length), from the series' qualifier stream.
// A row whose qualifier width is not the series' raises ERR_CELLS_GENERIC
// (the batch is rewritten with one width, as in k_cells_prep).
template <class M>
__global__ __launch_bounds__(256) void k_cells_fold_prep(
    Params P, CellsFold CF, int64_t S, SeriesMeta SM, int64_t NW, int64_t WB,
    WinCtx* __restrict__ wc, int* err_word) {
  const int64_t nbd = NW - 1;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t s = idx / nbd;
  if (s >= S) return;
  const int64_t j = idx - s * nbd + 1;
  const int64_t o = s * nbd + j - 1;
  const CellsDev& C = CF.C;
  WinCtx c{0, INT64_MIN, 0.0, INT64_MIN, 0.0};
  const bool keep = SM.keep[s];
  const int64_t lo = keep ? SM.lo[s] : 0, hi = keep ? SM.hi[s] : 0;
  CF.wrlo[o] = CF.rlo[s];
  CF.wvlo[o] = CF.vlo[s];
  CF.wvl0[o] = CF.vl0[s];
  if (lo >= hi) {
    c.bnd = lo;
    wc[o] = c;
    return;
  }
  const int64_t r0 = CF.series_row[s], r1 = CF.series_row[s + 1];
  const int64_t qb = C.qual_off[r0];
  const int qw = CF.qw[s], qsh = qw == 4 ? 2 : 1;
  const int64_t Ns = (C.qual_off[r1] - qb) >> qsh;
  const int64_t vend = C.val_off[C.R];
  bool bad = false;
  auto row_ok = [&](int64_t r) {
    const int64_t a = C.qual_off[r], l = C.qual_off[r + 1] - a;
    if (l <= 0 || (l & (qw - 1))) return false;
    return ((C.qual[a] & 0xF0) == 0xF0 ? 4 : 2) == qw;
  };
  auto row_of = [&](int64_t p) {  // the last r with qual_off[r] <= qb+qw*p
    int64_t a = r0, b = r1 - 1;
    const int64_t x = qb + qw * p;
    while (a < b) {
      const int64_t m = (a + b + 1) >> 1;
      if (C.qual_off[m] <= x) a = m;
      else b = m - 1;
    }
    return a;
  };
  auto first_pt = [&](int64_t r) { return (C.qual_off[r] - qb) >> qsh; };
  auto qual = [&](int64_t p) { return cells_qual_at(C, qb + qw * p, qw); };
  auto ts_in = [&](int64_t p, int64_t r) {
    return qual_ts(C.row_base_s[r] * 1000, qw, qual(p));
  };
  // the value byte offset of point p of row r: the row's offset + the
  // lengths of the row's points before p, 16 qualifier bytes a load
  const int64_t qend = C.qual_off[C.R];
  auto voff_of = [&](int64_t p, int64_t r) {
    int64_t v = C.val_off[r];
    int64_t a = qb + qw * first_pt(r);
    const int64_t e = qb + qw * p;
    for (; a + 16 <= e && a + 16 <= qend; a += 16) {
      const uint4 x = *reinterpret_cast<const uint4*>(C.qual + a);
      const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // the flags byte of each qualifier: the last of its qw bytes
        if (qw == 2) v += ((w[i] >> 8) & 7) + ((w[i] >> 24) & 7) + 2;
        else v += ((w[i] >> 24) & 7) + 1;
      }
    }
    for (; a < e; a += qw) v += (C.qual[a + qw - 1] & 0x7) + 1;
    return v;
  };
  // sequential fold of points [a, e) with ts < e_ts from point a of row r at
  // value offset v, rows crossed in order
  auto fold_run = [&](int64_t a, int64_t r, int64_t v, int64_t e, int64_t e_ts,
                      int* err) {
    M st = M::init();
    int64_t next = r + 1 < r1 ? first_pt(r + 1) : Ns;
    for (int64_t i = a; i < e; ++i) {
      if (i == next) {
        ++r;
        bad |= !row_ok(r);
        v = C.val_off[r];
        next = r + 1 < r1 ? first_pt(r + 1) : Ns;
      }
      const uint32_t q = qual(i);
      if (qual_ts(C.row_base_s[r] * 1000, qw, q) >= e_ts) break;
      const int l = (int)(q & 0x7) + 1;
      st.push(bits_to_double(dbits_of(load_be(C.val, v, l, vend), l, (q & 0x8) != 0)));
      v += l;
    }
    return st.finish(err);
  };
  // the first point at or after the window start T: the first row whose
  // last point is >= T (points increase across the series' rows; bases may
  // repeat — Span.addRow keeps a second RowSeq of one row key), then its
  // first point >= T
  const int64_t T = bucket_ts(P, j * WB);
  auto last_ts = [&](int64_t r) {
    return ts_in((r + 1 < r1 ? first_pt(r + 1) : Ns) - 1, r);
  };
  int64_t r, p;
  {
    int64_t ra = r0, rb = r1;  // first r with last_ts(r) >= T, r1 if none
    while (ra < rb) {
      const int64_t m = ra + ((rb - ra) >> 1);
      if (last_ts(m) < T) ra = m + 1;
      else rb = m;
    }
    r = ra;
  }
  if (r >= r1) {
    r = r1 - 1;
    p = Ns;
  } else {
    bad |= !row_ok(r);
    int64_t pa = first_pt(r);
    int64_t pb = (r + 1 < r1 ? first_pt(r + 1) : Ns) - 1;  // ts(pb) >= T
    while (pa < pb) {
      const int64_t m = pa + ((pb - pa) >> 1);
      if (ts_in(m, r) < T) pa = m + 1;
      else pb = m;
    }
    p = pa;
  }
  if (p < lo || p > hi) {  // the seek / stop bounds cut the window: clamp
    p = p < lo ? lo : hi;
    r = p < Ns ? row_of(p) : r1 - 1;
  }
  c.bnd = p;
  int err = 0;
  if (p > lo) {
    // the bucket of point p - 1 and its points [q, p): galloping back from
    // p - 1 brackets the bucket's first point, a binary search finds it
    // (a bucket of millisecond points holds millions: no point-by-point
    // walk), each probe's row by row_of
    int64_t rq = (p - 1 >= first_pt(r) || r == r0) ? r : r - 1;
    if (p - 1 < first_pt(rq)) rq = row_of(p - 1);
    const int64_t bt = bucket_ts(P, bucket_of(P, ts_in(p - 1, rq)));
    auto ts_of = [&](int64_t m) { return ts_in(m, row_of(m)); };
    int64_t hi_q = p - 1, lo_q = lo - 1;  // ts(hi_q) >= bt; ts(lo_q) < bt
    for (int64_t step = 1;; step <<= 1) {
      const int64_t m = hi_q - step;
      if (m <= lo_q) break;
      if (ts_of(m) < bt) {
        lo_q = m;
        break;
      }
      hi_q = m;
    }
    while (hi_q - lo_q > 1) {
      const int64_t m = lo_q + ((hi_q - lo_q) >> 1);
      if (ts_of(m) < bt) lo_q = m;
      else hi_q = m;
    }
    const int64_t q = hi_q;
    rq = row_of(q);
    c.prev_ts = bt;
    c.prev_val = fold_run(q, rq, voff_of(q, rq), p, INT64_MAX, &err);
  }
  if (p < hi) {
    const int64_t k = bucket_of(P, ts_in(p, r));
    const int64_t vp = voff_of(p, r);
    c.next_ts = bucket_ts(P, k);
    c.next_val = fold_run(p, r, vp, hi, bucket_ts(P, k + 1), &err);
    // the stream's cursor at point p
    CF.wrlo[o] = r;
    CF.wvlo[o] = vp;
    CF.wvl0[o] = (uint8_t)((qual(p) & 0x7) + 1);
  }
  if (bad) atomicOr(err_word, ERR_CELLS_GENERIC);
  wc[o] = c;
}

// ---------------------------------------------------------------- stream
// The lane's value bytes from byte a of the pool as dwords: NL 16-byte loads
// (unaligned) for K values, one more for a run that skips a meta byte
// (issued by every lane: its bytes are the next lane's, cache hits).
template <int NL>
DEV void cells_vload(const uint8_t* val, uint32_t a, uint32_t* d) {
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint4 w = *reinterpret_cast<const uint4*>(val + a + 16 * i);
    d[4 * i] = w.x; d[4 * i + 1] = w.y; d[4 * i + 2] = w.z; d[4 * i + 3] = w.w;
  }
#pragma unroll
  for (int i = 4 * NL; i < 20; ++i) d[i] = 0;
}

// loads for a value length vl (wave-uniform) into d[20]
DEV void cells_vload_vl(int vl, const uint8_t* val, uint32_t a, uint32_t* d) {
  switch (vl) {
    case 8: cells_vload<5>(val, a, d); break;
    case 4: cells_vload<3>(val, a, d); break;
    case 2: cells_vload<2>(val, a, d); break;
    default: cells_vload<1>(val, a, d); break;
  }
}

// Byte-wise version near the end of the pool (never reads at or past vend).
DEV void cells_vload_bytes(const uint8_t* val, int32_t a, int32_t vend,
                           uint32_t* d) {
#pragma unroll
  for (int i = 0; i < 20; ++i) {
    uint32_t w = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int32_t x = a + 4 * i + b;
      w |= (x < vend ? (uint32_t)val[x] : 0u) << (8 * b);
    }
    d[i] = w;
  }
}

// The K values (one length VL, one type FL) of a lane whose bytes start at
// d[0]; points j >= jb sit SH (0 / 1, the skipped meta byte) further on.
// -> the folded double's bits (RowSeq extractIntegerValue /
// extractFloatingPointValue, toDouble).
template <int VL, int FL, int K>
DEV void cells_vextract(const uint32_t* d, int jb, uint32_t sh, int64_t* v) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t s = j >= jb ? sh : 0u;
    if (VL == 8) {
      const uint32_t lo = __builtin_amdgcn_alignbyte(d[2 * j + 1], d[2 * j], s);
      const uint32_t hi =
          __builtin_amdgcn_alignbyte(d[2 * j + 2], d[2 * j + 1], s);
      const int64_t x = (int64_t)(((uint64_t)__builtin_bswap32(lo) << 32) |
                                  __builtin_bswap32(hi));
      v[j] = FL ? x : __double_as_longlong((double)x);
    } else if (VL == 4) {
      const uint32_t x =
          __builtin_bswap32(__builtin_amdgcn_alignbyte(d[j + 1], d[j], s));
      v[j] = __double_as_longlong(FL ? (double)__uint_as_float(x)
                                     : (double)(int32_t)x);
    } else if (VL == 2) {
      const int i0 = j >> 1;
      const uint32_t r = 2u * (uint32_t)(j & 1) + s;  // <= 3
      const uint32_t x = __builtin_amdgcn_alignbyte(d[i0 + 1], d[i0], r);
      v[j] = __double_as_longlong(
          (double)(int16_t)(((x & 0xFF) << 8) | ((x >> 8) & 0xFF)));
    } else {
      const int i0 = j >> 2;
      const uint32_t r = (uint32_t)(j & 3) + s;  // <= 4
      const uint32_t x =
          r >= 4 ? d[i0 + 1] : __builtin_amdgcn_alignbyte(d[i0 + 1], d[i0], r);
      v[j] = __double_as_longlong((double)(int8_t)(x & 0xFF));
    }
  }
}

template <int K>
DEV void cells_vextract_vl(int vl, int fl, const uint32_t* d, int jb,
                           uint32_t sh, int64_t* v) {
  switch (vl + 16 * fl) {
    case 8 + 16: cells_vextract<8, 1, K>(d, jb, sh, v); break;
    case 4 + 16: cells_vextract<4, 1, K>(d, jb, sh, v); break;
    case 8: cells_vextract<8, 0, K>(d, jb, sh, v); break;
    case 4: cells_vextract<4, 0, K>(d, jb, sh, v); break;
    case 2: cells_vextract<2, 0, K>(d, jb, sh, v); break;
    default: cells_vextract<1, 0, K>(d, jb, sh, v); break;
  }
}

// grid-relative time of in-step point `rel` (wave-uniform; lane rel / K,
// element rel % K — a uniform select, then a readlane: no dynamic register
// index)
template <int K>
DEV uint32_t cells_pick(const uint32_t* t, int32_t rel) {
  // the element index is per lane (-1 off lane L): with a wave-uniform one
  // the compiler turns the select chain into t[e] and puts t[] in scratch
  const int L = (int)(rel / K);
  const int e = LANE == L ? (int)(rel % K) : -1;
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) x = j == e ? t[j] : x;
  return (uint32_t)__builtin_amdgcn_readlane((int)x, L);
}

// One member's points [pa, pb) straight from its compacted columns (the
// cells counterpart of fold_member; NW == 1, so no window context).  The
// grid is narrow (run_pipeline sends other grids to k_bucketize_cells):
// point times are 32-bit ms since the grid base, row bases too.
// Indexing is 32-bit and relative to the series (its point numbers, and
// value bytes from its first row's val_off; k_cells_prep sends series whose
// pools exceed 2^30 bytes to the generic decode): loads address a uniform
// base pointer plus a per-lane 32-bit offset, and no runtime multiply is
// left (qualifier width and value length are powers of two: shifts).
// QW: the series' qualifier width when the launch fixes it (every kept
// series of the batch has QW-byte qualifiers), 0: read from the member
template <class M, class A, int K, int QW>
DEV void fold_member_cells(const Params& P, const CellsDev& C, FoldSink<A>& F,
                           const FoldMember* mc, const CellsMember* cm) {
  constexpr int PTS = 64 * K;
  constexpr int32_t BIG = 0x40000000;  // first point of rows past the series
  static_assert(K == 8, "qualifier loads assume 8 points per lane");
  const int lane = LANE;
  const bool kept = uni(mc->kept) != 0;
  fold_member_init(P, F, mc);
  if (!kept) return;
  const int32_t pe = (int32_t)uni(mc->pb);
  const int64_t r1 = uni(cm->r1);
  const int qw = QW ? QW : uni(cm->qw);
  const int qsh = qw == 4 ? 2 : 1;
  const int64_t qb = uni(cm->qb), vb0 = uni(cm->vb0);
  const uint8_t* qp = C.qual + qb;  // the series' qualifier stream
  const uint8_t* vp = C.val + vb0;  // its value bytes
  // readable bytes past the bases (the pools' ends), clamped to int32
  const int64_t ql64 = uni(cm->qend) - qb, vl64 = uni(cm->vend) - vb0;
  const int32_t qlim = ql64 > INT32_MAX ? INT32_MAX : (int32_t)ql64;
  const int32_t vlim = vl64 > INT32_MAX ? INT32_MAX : (int32_t)vl64;
  int32_t vcur = (int32_t)(uni(cm->vcur) - vb0);
  int64_t ra = uni(cm->rlo);
  int vsh = 3;  // log2 of the value length the loads speculate on
  {
    const int v0 = uni(cm->vl0);
    vsh = v0 == 1 ? 0 : (v0 == 2 ? 1 : (v0 == 4 ? 2 : 3));
  }
  RowSink S{nullptr, nullptr, F.ring, FOLD_WIN - 1, 0, 0, 0, 0};
  const BatchDev Bd{0, nullptr, nullptr, nullptr, nullptr, nullptr};
  int err = 0;
  int carry_key = INT32_MIN;
  M carry = M::init();
  int32_t prev_hi = -1;
  int fault = 0;  // ERR_CELLS_GENERIC / ERR_CORRUPT_CELL / ERR_INTERNAL
  // row metadata, row mb + lane: first point, first value byte, points |
  // bad shape << 30, base time (ms since the grid base, mod 2^32)
  int64_t mb = -(int64_t)BIG;
  int32_t w_ps = 0, w_vo = 0, w_nb = 0, w_br = 0;
  const int64_t gbase = P.gbase;
  auto load_window = [&](int64_t m) {
    mb = m;
    const int64_t x = m + lane;
    w_ps = BIG;
    w_vo = 0;
    w_nb = 0;
    w_br = 0;
    if (x <= r1) {
      const int64_t qo = C.qual_off[x];
      w_ps = (int32_t)((qo - qb) >> qsh);
      w_vo = (int32_t)(C.val_off[x] - vb0);
      if (x < r1) {
        const int32_t ql = (int32_t)(C.qual_off[x + 1] - qo);
        w_nb = (ql >> qsh) | ((ql <= 0 || (ql & (qw - 1))) ? (1 << 30) : 0);
        w_br = (int32_t)(uint32_t)(C.row_base_s[x] * 1000 - gbase);
      }
    }
  };
  int32_t p = (int32_t)uni(mc->pa);
  const int32_t pa0 = p;
  uint32_t t_last_prev = 0;  // check_order: the previous step's last time
  L2Touch pq_, pv_;
  const int32_t n_guard = pe - p + 64;  // every step consumes >= 1 point
  int dbg_n = 0;
  while (p < pe) {
    FOLD_GUARD(dbg_n, n_guard, F.err, "cells stream mi=%d p=%d pe=%d\n",
               F.mi, p, pe)
    if (ra < mb || ra + 3 >= mb + 64) load_window(ra);
    const int j0 = (int)(ra - mb);
    const int32_t ps0 = __builtin_amdgcn_readlane(w_ps, j0);
    const int32_t ps1 = __builtin_amdgcn_readlane(w_ps, j0 + 1);
    const int32_t ps2 = __builtin_amdgcn_readlane(w_ps, j0 + 2);
    const int32_t ps3 = __builtin_amdgcn_readlane(w_ps, j0 + 3);
    // the step: at most three rows, every row wholly inside it >= K points
    int32_t sb = p + PTS < pe ? p + PTS : pe;
    if (ps2 <= sb && ps2 - ps1 < K) sb = ps1;
    else if (ps3 <= sb && ps3 - ps2 < K) sb = ps2;
    if (sb > ps3) sb = ps3;
    if (sb <= p) {  // the row of p is not ra: an engine invariant broke
      fault |= ERR_INTERNAL;
      break;
    }
    const int32_t nb0 = __builtin_amdgcn_readlane(w_nb, j0);
    const int32_t nb1 = __builtin_amdgcn_readlane(w_nb, j0 + 1);
    const int32_t nb2 = __builtin_amdgcn_readlane(w_nb, j0 + 2);
    if ((nb0 | (ps1 < sb ? nb1 : 0) | (ps2 < sb ? nb2 : 0)) & (1 << 30)) {
      fault |= ERR_CELLS_GENERIC;
      break;
    }
    // this row's values start here: the previous row's bytes added up
    if (p == ps0 && vcur != __builtin_amdgcn_readlane(w_vo, j0)) {
#ifdef OTSDB_CELLS_DEBUG
      if (lane == 0) printf("start mi=%d p=%d vcur=%d\n", F.mi, p, vcur);
#endif
      fault |= ERR_CORRUPT_CELL;
      break;
    }
    const int32_t m0 = (nb0 & 0xFFFFFF) > 1 ? 1 : 0;
    const int32_t m1 = (nb1 & 0xFFFFFF) > 1 ? 1 : 0;
    const int32_t m2 = (nb2 & 0xFFFFFF) > 1 ? 1 : 0;
    // ---- this lane's points p0 .. p0 + nv - 1 and the loads (only what the
    // addresses need is computed before the flush)
    const int32_t p0 = p + K * lane;
    const int32_t rem = sb - p0;
    const int nv = rem < 0 ? 0 : (rem > K ? K : rem);
    const bool act = nv > 0;
    const int32_t mbefore = (p0 >= ps1 ? m0 : 0) + (p0 >= ps2 ? m1 : 0);
    const uint32_t qoff = act ? (uint32_t)p0 << qsh : 0u;
    uint32_t dq[8], d[20];
    if (((p + PTS) << qsh) + 32 <= qlim) {
      const uint4 w = *reinterpret_cast<const uint4*>(qp + qoff);
      dq[0] = w.x; dq[1] = w.y; dq[2] = w.z; dq[3] = w.w;
      if (qw == 4) {
        const uint4 w2 = *reinterpret_cast<const uint4*>(qp + qoff + 16);
        dq[4] = w2.x; dq[5] = w2.y; dq[6] = w2.z; dq[7] = w2.w;
      } else {
        dq[4] = dq[5] = dq[6] = dq[7] = 0;
      }
    } else {  // the end of the pool: byte loads, never past it
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int32_t x = (int32_t)qoff + 4 * i + b;
          w |= (x < qlim ? (uint32_t)qp[x] : 0u) << (8 * b);
        }
        dq[i] = w;
      }
    }
    const bool vnear = vcur + 9 * PTS + 128 > vlim;
    int32_t a0 = act ? vcur + ((K * lane) << vsh) + mbefore : vcur;
    if (!vnear) cells_vload_vl(1 << vsh, vp, (uint32_t)a0, d);
    else cells_vload_bytes(vp, a0, vlim, d);
    if (OTSDB_PF_CELLS) {
      // the lines OTSDB_PF_CELLS steps ahead (at this step's value length)
      pq_.retire();
      pv_.retire();
      const int32_t pq = (p + OTSDB_PF_CELLS * PTS) << qsh;
      if (((p + (OTSDB_PF_CELLS + 1) * PTS) << qsh) + 16 <= qlim)
        pq_.touch(qp + pq + (lane << (qsh + 3)));
      const int32_t pvo = vcur + ((OTSDB_PF_CELLS * PTS) << vsh) +
                          (lane << (vsh + 3));
      if (vcur + (((OTSDB_PF_CELLS + 1) * PTS) << vsh) + 128 <= vlim)
        pv_.touch(vp + pvo);
    }
#if defined(OTSDB_CELLS_ABL) && OTSDB_CELLS_ABL == 2  // timing: loads only
    {
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) x ^= dq[i];
#pragma unroll
      for (int i = 0; i < 20; ++i) x ^= d[i];
      if (x == 42) F.emit[0] = 1;
      const int32_t hs = sb;
      vcur += ((hs - p) << vsh) + (ps1 <= hs ? m0 : 0) + (ps2 <= hs ? m1 : 0) +
              (ps3 <= hs ? m2 : 0);
      ra += (ps1 <= hs ? 1 : 0) + (ps2 <= hs ? 1 : 0) + (ps3 <= hs ? 1 : 0);
      p = hs;
      continue;
    }
#endif
    // ---- buckets below the open one are final: drain them while the
    // loads are in flight (fold_member)
    const bool carry_ok = carry_key >= 0 && carry_key < P.nb;
    int32_t limit = carry_ok ? carry_key : prev_hi + 1;
    // (the final buckets are drained at the end of the step, not here while
    // the loads are in flight: the flush's registers on top of the step's
    // load registers cost the stream loop 10 %, A/B round 4)
    // ---- the lane's rows: it crosses at most one boundary, before point jb
    const int rl = (p0 >= ps1 ? 1 : 0) + (p0 >= ps2 ? 1 : 0);
    const int32_t nbnd = rl == 0 ? ps1 : (rl == 1 ? ps2 : ps3);
    const int jb = nbnd - p0 < K ? nbnd - p0 : K;
    const bool cross = act && jb < nv;  // (jb < 0 on lanes past the step)
    const int32_t mnext = rl == 0 ? m0 : (rl == 1 ? m1 : m2);
    // row base times (grid-relative, mod 2^32)
    const uint32_t rb0 = (uint32_t)__builtin_amdgcn_readlane(w_br, j0);
    const uint32_t rb1 = (uint32_t)__builtin_amdgcn_readlane(w_br, j0 + 1);
    const uint32_t rb2 = (uint32_t)__builtin_amdgcn_readlane(w_br, j0 + 2);
    const uint32_t rb3 = (uint32_t)__builtin_amdgcn_readlane(w_br, j0 + 3);
    const uint32_t bcur = rl == 0 ? rb0 : (rl == 1 ? rb1 : rb2);
    const uint32_t bnext = rl == 0 ? rb1 : (rl == 1 ? rb2 : rb3);
    // ---- qualifiers -> timestamps, flags
    uint32_t q[K];
    if (qw == 2) {
#pragma unroll
      for (int j = 0; j < K; j += 2) {  // bytes b0 b1 b2 b3 -> b1 b0 b3 b2
        const uint32_t w = __builtin_amdgcn_perm(dq[j >> 1], dq[j >> 1], 0x02030001u);
        q[j] = w & 0xFFFFu;
        q[j + 1] = w >> 16;
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) q[j] = __builtin_bswap32(dq[j]);
    }
    const uint32_t f0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(q[0] & 0xF));
    int odd = 0, mixed = 0;
    uint32_t t[K];
    int64_t v[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const bool in = j < nv;
      const uint32_t nib = qw == 2 ? (q[j] >> 12) : (q[j] >> 28);
      odd |= in && ((qw == 2) == (nib == 0xF));
      mixed |= in && ((q[j] & 0xF) != f0);
      const uint32_t off = qw == 2 ? (q[j] >> 4) * 1000u
                                   : (q[j] & 0x0FFFFFC0u) >> 6;
      t[j] = (j >= jb ? bnext : bcur) + off;
    }
    if (__ballot(odd)) {
      fault |= ERR_CELLS_GENERIC;
      break;
    }
    if (P.check_order) {
      // verbatim storage rows: each point strictly after its predecessor
      // (the lane before it; lane 0: the previous step's last point)
      const uint32_t tp = (uint32_t)dpp32<0x138, 0xF>((int32_t)t_last_prev,
                                                      (int32_t)t[K - 1]);
      int ob = 0;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (j < nv) ob |= (j == 0 ? (p0 > pa0 && t[0] <= tp) : t[j] <= t[j - 1]);
      if (__ballot(ob)) {
        fault |= ERR_NOT_SORTED;
        break;
      }
    }
    const int32_t vo1 = __builtin_amdgcn_readlane(w_vo, j0 + 1);
    const int32_t vo2 = __builtin_amdgcn_readlane(w_vo, j0 + 2);
    const int32_t vo3 = __builtin_amdgcn_readlane(w_vo, j0 + 3);
    const int32_t vonext = rl == 0 ? vo1 : (rl == 1 ? vo2 : vo3);
    const bool uniform = __ballot(mixed) == 0;
    int vbad = 0;
    if (uniform) {
      const int vl = (int)(f0 & 0x7) + 1, fl = (f0 & 0x8) != 0;
      if (fl ? !(vl == 4 || vl == 8) : !(vl == 1 || vl == 2 || vl == 4 || vl == 8)) {
        fault |= ERR_CORRUPT_CELL;
        break;
      }
      if (vl != (1 << vsh)) {  // the speculation missed: load again
        vsh = vl == 1 ? 0 : (vl == 2 ? 1 : (vl == 4 ? 2 : 3));
        a0 = act ? vcur + ((K * lane) << vsh) + mbefore : vcur;
        if (vnear) cells_vload_bytes(vp, a0, vlim, d);
        else cells_vload_vl(vl, vp, (uint32_t)a0, d);
      }
      cells_vextract_vl<K>(vl, fl, d, jb, (uint32_t)mnext, v);
      // the boundary point lands on the next row's first value
      vbad |= cross && (a0 + (jb << vsh) + mnext != vonext);
#ifdef OTSDB_CELLS_DEBUG
      if (cross && (a0 + (jb << vsh) + mnext != vonext))
        printf("cross mi=%d p=%d lane=%d jb=%d nv=%d rl=%d a0=%d vl=%d von=%d\n",
               F.mi, p, lane, jb, nv, rl, a0, vl, vonext);
#endif
    } else {
      int lpre[K], pre = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        lpre[j] = pre;
        pre += j < nv ? (int)(q[j] & 0x7) + 1 : 0;
      }
      int tot;
      const int lex = wave_excl_scan(pre, tot);
      a0 = vcur + lex + mbefore;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        if (j < nv) {
          const int l = (int)(q[j] & 0x7) + 1;
          const int fl = (q[j] & 0x8) != 0;
          vbad |= fl ? !(l == 4 || l == 8) : !(l == 1 || l == 2 || l == 4 || l == 8);
          const int32_t a = a0 + lpre[j] + (j >= jb ? mnext : 0);
          uint64_t w = 0;
          if (!vnear) {
            w = *reinterpret_cast<const uint64_t*>(vp + (uint32_t)a);
          } else {
#pragma unroll
            for (int b = 0; b < 8; ++b)
              if (a + b < vlim) w |= (uint64_t)vp[a + b] << (8 * b);
          }
          v[j] = dbits_of(__builtin_bswap64(w) >> (64 - 8 * l), l, fl);
          if (j == jb) vbad |= a != vonext;
        } else {
          v[j] = 0;
        }
      }
    }
    if (__ballot(vbad)) {
#ifdef OTSDB_CELLS_DEBUG
      if (lane == 0) printf("vbad mi=%d p=%d uniform=%d f0=%u\n", F.mi, p, (int)uniform, f0);
#endif
      fault |= ERR_CORRUPT_CELL;
      break;
    }
    // ---- the downsample over [p, hs) (fold_member's ring bookkeeping)
    const int32_t k_hi = bucket_rel(P, cells_pick<K>(t, sb - 1 - p));
    int32_t hs = sb;
    if (k_hi >= F.flushed + FOLD_WIN) {
      const int32_t k_first = bucket_rel(P, cells_pick<K>(t, 0));
      if (carry_ok && carry_key < k_first) {
        if (lane == 0) S.put(carry_key, carry.finish(&err));
        carry_key = INT32_MIN;
        limit = k_first;
      } else if (!carry_ok) {
        limit = k_first;
      }
      fold_flush(P, F, limit);
      if (k_hi >= F.flushed + FOLD_WIN) {
        // the ring's end (k_hi lies past it, so inside the narrow grid)
        const uint32_t T =
            (uint32_t)((int64_t)(F.flushed + FOLD_WIN) * P.interval);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) cnt += (j < nv && t[j] < T) ? 1 : 0;
        hs = p + uni((int32_t)wave_sum(cnt));
      }
    }
    // ---- cursor past point hs - 1 (before the reduction: the qualifiers
    // and the timestamps' picks need no registers across it)
    int32_t used;
    if (uniform) {
      used = (hs - p) << vsh;
    } else {
      int c = 0;
#pragma unroll
      for (int j = 0; j < K; ++j)
        c += (j < nv && p0 + j < hs) ? (int)(q[j] & 0x7) + 1 : 0;
      used = uni((int32_t)wave_sum(c));
    }
    const int32_t k_last =
        hs == sb ? k_hi : bucket_rel(P, cells_pick<K>(t, hs - 1 - p));
    if (P.check_order) t_last_prev = cells_pick<K>(t, hs - 1 - p);
    // a step cut at a row rule (not at a bucket edge) leaves the bucket of
    // its last point open: it carries into the next step (keep_open)
#if defined(OTSDB_CELLS_ABL) && OTSDB_CELLS_ABL == 1  // timing: no reduction
    {
      int64_t x = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) x ^= t[j] + v[j];
      if (x == 42) F.emit[0] = 1;
    }
#else
    reduce_step<M, K, 1, uint32_t, 1>(P, Bd, 1, p, hs, p, p0, t, v, S, err,
                                      carry_key, carry, hs < pe);
#endif
    vcur += used + (ps1 <= hs ? m0 : 0) + (ps2 <= hs ? m1 : 0) +
            (ps3 <= hs ? m2 : 0);
    ra += (ps1 <= hs ? 1 : 0) + (ps2 <= hs ? 1 : 0) + (ps3 <= hs ? 1 : 0);
    prev_hi = k_last;
    {  // the buckets this step finished (the load registers are dead here)
      const int32_t lim = (carry_key >= 0 && carry_key < P.nb) ? carry_key
                                                                 : prev_hi + 1;
      if (lim - F.flushed >= FOLD_FL) fold_flush(P, F, lim);
    }
    p = hs;
  }
  if (!fault) {
    // the stream ended on a row start (the series' end, or the stop bound
    // on a row boundary): the row before it added up
    if (ra < mb || ra >= mb + 64) load_window(ra);
    const int j0 = (int)(ra - mb);
    if (p == __builtin_amdgcn_readlane(w_ps, j0) &&
        vcur != __builtin_amdgcn_readlane(w_vo, j0)) {
#ifdef OTSDB_CELLS_DEBUG
      if (lane == 0) printf("end mi=%d p=%d vcur=%d\n", F.mi, p, vcur);
#endif
      fault |= ERR_CORRUPT_CELL;
    }
  }
  if (fault) {
    // the query fails or is re-run by the generic decode; the member's
    // remaining work is moot, the chain of progress marks must still end
    if (lane == 0) atomicOr(F.err, fault);
    return;
  }
  if (carry_key >= 0 && carry_key < P.nb && lane == 0)
    S.put(carry_key, carry.finish(&err));
  if (prev_hi >= 0) fold_flush(P, F, prev_hi + 1);
  fold_member_tail(P, F, mc);
}

// The uniform cells fold: fold_member_cells for a series k_cells_uniform
// proved uniform (every kept series of the batch is).  Each value is `vl`
// bytes of one type, so a lane's values start at the stream cursor +
// (its first point's index in the step << vsh) + the meta bytes of the rows
// before it, lengths need no speculation and no prefix sums, and the rows'
// value bytes add up by construction: no row-start / row-end cursor checks,
// no value-length legality per step.  What a step still does: the row window
// (first points with the meta byte before each row packed into bit 31, base
// times), the qualifier -> time decode, one packed compare per 4 qualifier
// bytes that every streamed qualifier has the series' width and flags (a
// miss — a column whose lengths add up by accident — raises
// ERR_CELLS_NONUNI and the engine folds the batch again with the general
// kernel), the value extraction and the shared reduction.
// Reference: RowSeq.java:552-643, Internal.java:621-690.
template <int VL, int FL, int K>
DEV void cells_vload_u(const uint8_t* vp, int32_t a, bool near, int32_t vlim,
                       uint32_t* d) {
  // the lane's K values plus the one meta byte it may skip: VL*K + 1 bytes
  constexpr int NB = VL * K + 1;
  constexpr int ND = (NB + 3) / 4;
  if (near) {
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int32_t x = a + 4 * i + b;
        w |= (x < vlim ? (uint32_t)vp[x] : 0u) << (8 * b);
      }
      d[i] = w;
    }
    return;
  }
  const uint8_t* s = vp + (uint32_t)a;
  if (VL >= 2) {
#pragma unroll
    for (int i = 0; i < (VL * K) / 16; ++i) {
      const uint4 w = *reinterpret_cast<const uint4*>(s + 16 * i);
      d[4 * i] = w.x; d[4 * i + 1] = w.y; d[4 * i + 2] = w.z; d[4 * i + 3] = w.w;
    }
  } else {
    const uint2 w = *reinterpret_cast<const uint2*>(s);
    d[0] = w.x; d[1] = w.y;
  }
  d[ND - 1] = *reinterpret_cast<const uint32_t*>(s + 4 * (ND - 1));
}

// The uniform fold's value extraction: 8- and 4-byte values with one
// v_perm each 4 bytes (the byte swap and the meta-byte shift in one
// selector, per lane: 0x00010203 + shift x 0x01010101), 1- and 2-byte ones
// as cells_vextract.
template <int VL, int FL, int K>
DEV void cells_vextract_p(const uint32_t* d, int jb, uint32_t sh, int64_t* v) {
  if constexpr (VL == 8 || VL == 4) {
    const uint32_t s0 = 0x00010203u, s1 = s0 + sh * 0x01010101u;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t sel = j >= jb ? s1 : s0;
      if constexpr (VL == 8) {
        const uint32_t hi = __builtin_amdgcn_perm(d[2 * j + 1], d[2 * j], sel);
        const uint32_t lo = __builtin_amdgcn_perm(d[2 * j + 2], d[2 * j + 1], sel);
        const int64_t x = (int64_t)(((uint64_t)hi << 32) | lo);
        v[j] = FL ? x : __double_as_longlong((double)x);
      } else {
        const uint32_t x = __builtin_amdgcn_perm(d[j + 1], d[j], sel);
        v[j] = __double_as_longlong(FL ? (double)__uint_as_float(x)
                                       : (double)(int32_t)x);
      }
    }
  } else {
    cells_vextract<VL, FL, K>(d, jb, sh, v);
  }
}

template <int K>
DEV void cells_vextract_pl(int vl, int fl, const uint32_t* d, int jb,
                           uint32_t sh, int64_t* v) {
  switch (vl + 16 * fl) {
    case 8 + 16: cells_vextract_p<8, 1, K>(d, jb, sh, v); break;
    case 4 + 16: cells_vextract_p<4, 1, K>(d, jb, sh, v); break;
    case 8: cells_vextract_p<8, 0, K>(d, jb, sh, v); break;
    case 4: cells_vextract_p<4, 0, K>(d, jb, sh, v); break;
    case 2: cells_vextract_p<2, 0, K>(d, jb, sh, v); break;
    default: cells_vextract_p<1, 0, K>(d, jb, sh, v); break;
  }
}

template <class M, class A, int K, int QW>
DEV void fold_member_cells_u(const Params& P, const CellsDev& C, FoldSink<A>& F,
                             const FoldMember* mc, const CellsMember* cm) {
  constexpr int PTS = 64 * K;
  constexpr int32_t BIG = 0x40000000;  // first point of rows past the series
  constexpr int qsh = QW == 4 ? 2 : 1;
  static_assert(K == 8 && (QW == 2 || QW == 4), "8 points per lane, QW 2 / 4");
  const int lane = LANE;
  const bool kept = uni(mc->kept) != 0;
  fold_member_init(P, F, mc);
  if (!kept) return;
  const int32_t pe = (int32_t)uni(mc->pb);
  const int64_t r1 = uni(cm->r1);
  const int64_t qb = uni(cm->qb), vb0 = uni(cm->vb0);
  const uint8_t* qp = C.qual + qb;
  const uint8_t* vp = C.val + vb0;
  const int64_t ql64 = uni(cm->qend) - qb, vl64 = uni(cm->vend) - vb0;
  const int32_t qlim = ql64 > INT32_MAX ? INT32_MAX : (int32_t)ql64;
  const int32_t vlim = vl64 > INT32_MAX ? INT32_MAX : (int32_t)vl64;
  int32_t vcur = (int32_t)(uni(cm->vcur) - vb0);
  int64_t ra = uni(cm->rlo);
  const uint32_t f = (uint32_t)uni(cm->uf) & 0xFu;
  const int vl = (int)(f & 7) + 1, fl = (f & 8) ? 1 : 0;
  const int vsh = vl == 1 ? 0 : (vl == 2 ? 1 : (vl == 4 ? 2 : 3));
  // the packed check.  QW 2: a dword is two big-endian qualifiers b0 b1 |
  // b2 b3; width: b0 / b2's high nibble is not 0xF (+0x10 carries into bit
  // 8 / 24 only from 0xF0); flags: b1 / b3's low nibble is f.  QW 4: one
  // qualifier b0..b3; b0's high nibble 0xF, b3's low nibble f.
  const uint32_t fpat = QW == 2 ? (f << 8) | (f << 24) : (f << 24) | 0xF0u;
  RowSink S{nullptr, nullptr, F.ring, FOLD_WIN - 1, 0, 0, 0, 0};
  const BatchDev Bd{0, nullptr, nullptr, nullptr, nullptr, nullptr};
  int err = 0;
  int carry_key = INT32_MIN;
  M carry = M::init();
  int32_t prev_hi = -1;
  int fault = 0;  // ERR_CELLS_NONUNI / ERR_NOT_SORTED / ERR_INTERNAL
  // row window, row mb + lane: first point | (meta byte before the row) << 31,
  // base time (ms since the grid base, mod 2^32)
  int64_t mb = -(int64_t)BIG;
  int32_t w_ps = 0, w_br = 0;
  const int64_t gbase = P.gbase;
  auto load_window = [&](int64_t m) {
    mb = m;
    const int64_t x = m + lane;
    int32_t ps = BIG, br = 0;
    if (x <= r1) {
      ps = (int32_t)((C.qual_off[x] - qb) >> qsh);
      if (x < r1) br = (int32_t)(uint32_t)(C.row_base_s[x] * 1000 - gbase);
    }
    // the previous row's first point (wave_shr:1; lane 0's row is the
    // cursor's own, whose meta byte before it is never read)
    const int32_t pp = dpp32<0x138, 0xF>(ps, ps);
    const int32_t meta = (ps != BIG && ps - pp > 1) ? 1 : 0;
    w_ps = (int32_t)((uint32_t)ps | ((uint32_t)meta << 31));
    w_br = br;
  };
  int32_t p = (int32_t)uni(mc->pa);
  const int32_t pa0 = p;
  uint32_t t_last_prev = 0;  // check_order: the previous step's last time
  const int32_t n_guard = pe - p + 64;  // every step consumes >= 1 point
  int dbg_n = 0;
  L2Touch pq_, pv_;
  while (p < pe) {
    FOLD_GUARD(dbg_n, n_guard, F.err, "uniform cells stream mi=%d p=%d pe=%d\n",
               F.mi, p, pe)
    if (ra < mb || ra + 3 >= mb + 64) load_window(ra);
    const int j0 = (int)(ra - mb);
    const uint32_t x1 = (uint32_t)__builtin_amdgcn_readlane(w_ps, j0 + 1);
    const uint32_t x2 = (uint32_t)__builtin_amdgcn_readlane(w_ps, j0 + 2);
    const uint32_t x3 = (uint32_t)__builtin_amdgcn_readlane(w_ps, j0 + 3);
    const int32_t ps1 = (int32_t)(x1 & 0x7FFFFFFFu);
    const int32_t ps2 = (int32_t)(x2 & 0x7FFFFFFFu);
    const int32_t ps3 = (int32_t)(x3 & 0x7FFFFFFFu);
    const int32_t m0 = (int32_t)(x1 >> 31), m1 = (int32_t)(x2 >> 31),
                  m2 = (int32_t)(x3 >> 31);
    // the step: at most three rows, every row wholly inside it >= K points
    int32_t sb = p + PTS < pe ? p + PTS : pe;
    if (ps2 <= sb && ps2 - ps1 < K) sb = ps1;
    else if (ps3 <= sb && ps3 - ps2 < K) sb = ps2;
    if (sb > ps3) sb = ps3;
    if (sb <= p) {  // the row of p is not ra: an engine invariant broke
      fault |= ERR_INTERNAL;
      break;
    }
    const bool full = sb - p == PTS;  // (wave-uniform) every lane holds K points
    const uint32_t rb0 = (uint32_t)__builtin_amdgcn_readlane(w_br, j0);
    const uint32_t rb1 = (uint32_t)__builtin_amdgcn_readlane(w_br, j0 + 1);
    const uint32_t rb2 = (uint32_t)__builtin_amdgcn_readlane(w_br, j0 + 2);
    const uint32_t rb3 = (uint32_t)__builtin_amdgcn_readlane(w_br, j0 + 3);
    // ---- this lane's points p0 .. p0 + nv - 1: its row, the boundary it
    // may cross before point jb, the meta byte there
    const int32_t p0 = p + K * lane;
    const int32_t rem = sb - p0;
    const int nv = rem < 0 ? 0 : (rem > K ? K : rem);
    const bool c1 = p0 >= ps1, c2 = p0 >= ps2;
    const int32_t nbnd = c2 ? ps3 : (c1 ? ps2 : ps1);
    const int jb = nbnd - p0 < K ? nbnd - p0 : K;
    const int32_t mnext = c2 ? m2 : (c1 ? m1 : m0);
    const int32_t mbefore = (c1 ? m0 : 0) + (c2 ? m1 : 0);
    const uint32_t bcur = c2 ? rb2 : (c1 ? rb1 : rb0);
    const uint32_t bnext = c2 ? rb3 : (c1 ? rb2 : rb1);
    // ---- loads: qualifiers, then values (the lane's K values from its
    // row's cursor; lanes past the step load inside the pools too)
    uint32_t dq[QW == 4 ? 8 : 4];
    if (((p + PTS) << qsh) + 32 <= qlim) {
      const uint32_t qoff = (uint32_t)p0 << qsh;
      const uint4 w = *reinterpret_cast<const uint4*>(qp + qoff);
      dq[0] = w.x; dq[1] = w.y; dq[2] = w.z; dq[3] = w.w;
      if constexpr (QW == 4) {
        const uint4 w2 = *reinterpret_cast<const uint4*>(qp + qoff + 16);
        dq[4] = w2.x; dq[5] = w2.y; dq[6] = w2.z; dq[7] = w2.w;
      }
    } else {  // the end of the pool: byte loads, never past it
      const int32_t qoff = nv > 0 ? p0 << qsh : 0;
#pragma unroll
      for (int i = 0; i < (QW == 4 ? 8 : 4); ++i) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int32_t x = qoff + 4 * i + b;
          w |= (x < qlim ? (uint32_t)qp[x] : 0u) << (8 * b);
        }
        dq[i] = w;
      }
    }
    const bool vnear = vcur + 9 * PTS + 128 > vlim;
    const int32_t a0 = vcur + ((K * lane) << vsh) + mbefore;
    if (OTSDB_PF_CELLS) {
      // the lines OTSDB_PF_CELLS steps ahead into L2 (one dword a lane: the
      // lane's 64 value bytes and 16 qualifier bytes of that step)
      pq_.retire();
      pv_.retire();
      if (((p + (OTSDB_PF_CELLS + 1) * PTS) << qsh) + 16 <= qlim)
        pq_.touch(qp + ((uint32_t)(p + OTSDB_PF_CELLS * PTS + K * lane) << qsh));
      const int32_t pvo = vcur + ((OTSDB_PF_CELLS * PTS + K * lane) << vsh);
      if (vcur + (((OTSDB_PF_CELLS + 1) * PTS) << vsh) + 128 <= vlim)
        pv_.touch(vp + (uint32_t)pvo);
    }
    uint32_t d[17];
    switch (vsh) {
      case 3: cells_vload_u<8, 0, K>(vp, a0, vnear, vlim, d); break;
      case 2: cells_vload_u<4, 0, K>(vp, a0, vnear, vlim, d); break;
      case 1: cells_vload_u<2, 0, K>(vp, a0, vnear, vlim, d); break;
      default: cells_vload_u<1, 0, K>(vp, a0, vnear, vlim, d); break;
    }
#if defined(OTSDB_CELLS_ABL) && OTSDB_CELLS_ABL == 2  // timing: loads only
    {
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < (QW == 4 ? 8 : 4); ++i) x ^= dq[i];
#pragma unroll
      for (int i = 0; i < 17; ++i) x ^= d[i];
      if (x == 42) F.emit[0] = 1;
      vcur += ((sb - p) << vsh) + (ps1 <= sb ? m0 : 0) + (ps2 <= sb ? m1 : 0) +
              (ps3 <= sb ? m2 : 0);
      ra += (ps1 <= sb ? 1 : 0) + (ps2 <= sb ? 1 : 0) + (ps3 <= sb ? 1 : 0);
      p = sb;
      continue;
    }
#endif
    // ---- every streamed qualifier: the series' width and flags
    // (flags: xor with the pattern, or-accumulated, masked once; QW 2's
    // width: +0x10 carries out of a 0xF0 nibble only; qualifiers of a
    // lane's points past the step replaced by the pattern itself)
    constexpr int NQ = QW == 4 ? 8 : 4;
    uint32_t qc[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) qc[i] = dq[i];
    if (!full) {
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const uint32_t m = QW == 2 ? ((2 * i < nv ? 0x0000FFFFu : 0u) |
                                      (2 * i + 1 < nv ? 0xFFFF0000u : 0u))
                                   : (i < nv ? 0xFFFFFFFFu : 0u);
        qc[i] = (qc[i] & m) | (fpat & ~m);
      }
    }
    uint32_t fx = 0, wx = 0;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      fx |= qc[i] ^ fpat;
      if constexpr (QW == 2) wx |= (qc[i] & 0x00F000F0u) + 0x00100010u;
    }
    const uint32_t bad = (fx & (QW == 2 ? 0x0F000F00u : 0x0F0000F0u)) |
                         (wx & 0x01000100u);
#if defined(OTSDB_CELLS_ABL) && OTSDB_CELLS_ABL == 3  // timing: no check
    if (bad == 0x12345678u) F.emit[1] = 1;
#else
    if (__ballot(bad != 0)) {
      fault |= ERR_CELLS_NONUNI;
      break;
    }
#endif
    // ---- qualifiers -> grid-relative times
    uint32_t t[K];
    if constexpr (QW == 2) {
#pragma unroll
      for (int j = 0; j < K; j += 2) {  // bytes b0 b1 b2 b3 -> b1 b0 b3 b2
        const uint32_t w = __builtin_amdgcn_perm(dq[j >> 1], dq[j >> 1], 0x02030001u);
        t[j] = ((w >> 4) & 0xFFFu) * 1000u + (j >= jb ? bnext : bcur);
        t[j + 1] = ((w >> 20) & 0xFFFu) * 1000u + (j + 1 >= jb ? bnext : bcur);
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j)
        t[j] = ((__builtin_bswap32(dq[j]) & 0x0FFFFFC0u) >> 6) +
               (j >= jb ? bnext : bcur);
    }
    if (P.check_order) {
      // verbatim storage rows: each point strictly after its predecessor
      // (the lane before it; lane 0: the previous step's last point)
      const uint32_t tp = (uint32_t)dpp32<0x138, 0xF>((int32_t)t_last_prev,
                                                      (int32_t)t[K - 1]);
      int ob = 0;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (j < nv) ob |= (j == 0 ? (p0 > pa0 && t[0] <= tp) : t[j] <= t[j - 1]);
      if (__ballot(ob)) {
        fault |= ERR_NOT_SORTED;
        break;
      }
    }
    // ---- values (the boundary's meta byte skipped from point jb on)
    int64_t v[K];
    cells_vextract_pl<K>(vl, fl, d, jb, (uint32_t)mnext, v);
    // ---- the downsample over [p, hs) (fold_member's ring bookkeeping)
    const int32_t k_hi = bucket_rel(
        P, full ? (uint32_t)__builtin_amdgcn_readlane((int32_t)t[K - 1], 63)
                : cells_pick<K>(t, sb - 1 - p));
    const bool carry_ok = carry_key >= 0 && carry_key < P.nb;
    int32_t limit = carry_ok ? carry_key : prev_hi + 1;
    int32_t hs = sb;
    if (k_hi >= F.flushed + FOLD_WIN) {
      const int32_t k_first = bucket_rel(P, cells_pick<K>(t, 0));
      if (carry_ok && carry_key < k_first) {
        if (lane == 0) S.put(carry_key, carry.finish(&err));
        carry_key = INT32_MIN;
        limit = k_first;
      } else if (!carry_ok) {
        limit = k_first;
      }
      fold_flush(P, F, limit);
      if (k_hi >= F.flushed + FOLD_WIN) {
        // the ring's end (k_hi lies past it, so inside the narrow grid)
        const uint32_t T =
            (uint32_t)((int64_t)(F.flushed + FOLD_WIN) * P.interval);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) cnt += (j < nv && t[j] < T) ? 1 : 0;
        hs = p + uni((int32_t)wave_sum(cnt));
      }
    }
    const int32_t k_last =
        hs == sb ? k_hi : bucket_rel(P, cells_pick<K>(t, hs - 1 - p));
    if (P.check_order) t_last_prev = cells_pick<K>(t, hs - 1 - p);
#if defined(OTSDB_CELLS_ABL) && OTSDB_CELLS_ABL == 1  // timing: no reduction
    {
      int64_t x = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) x ^= t[j] + v[j];
      if (x == 42) F.emit[0] = 1;
    }
#else
    reduce_step<M, K, 1, uint32_t, 1>(P, Bd, 1, p, hs, p, p0, t, v, S, err,
                                      carry_key, carry, hs < pe);
#endif
    vcur += ((hs - p) << vsh) + (ps1 <= hs ? m0 : 0) + (ps2 <= hs ? m1 : 0) +
            (ps3 <= hs ? m2 : 0);
    ra += (ps1 <= hs ? 1 : 0) + (ps2 <= hs ? 1 : 0) + (ps3 <= hs ? 1 : 0);
    prev_hi = k_last;
    {  // the buckets this step finished (the load registers are dead here)
      const int32_t lim = (carry_key >= 0 && carry_key < P.nb) ? carry_key
                                                                 : prev_hi + 1;
      if (lim - F.flushed >= FOLD_FL) fold_flush(P, F, lim);
    }
    p = hs;
  }
  if (fault) {
    // the query fails or is re-run by the general fold; the member's
    // remaining work is moot, the chain of progress marks must still end
    if (lane == 0) atomicOr(F.err, fault);
    return;
  }
  if (carry_key >= 0 && carry_key < P.nb && lane == 0)
    S.put(carry_key, carry.finish(&err));
  if (prev_hi >= 0) fold_flush(P, F, prev_hi + 1);
  fold_member_tail(P, F, mc);
}

}  // namespace otsdb
