"""Encodes columnar points into OpenTSDB compacted columns, the way the write
path + compaction lay them out (TSDB.addPoint value widths,
TSDB.java:1051-1147; Internal.buildQualifier, Internal.java:848-863;
CompactionQueue.buildCompactedColumn, CompactionQueue.java:594-616):
one row per (series, hour), 2-byte qualifiers for whole seconds, 4-byte ms
qualifiers otherwise, smallest of 1/2/4/8 bytes for longs, 4 or 8 bytes for
floats, trailing meta byte (bit0 = mixed s/ms) on multi-value columns."""
import struct

import numpy as np


def _long_bytes(v):
    for n, fmt in ((1, ">b"), (2, ">h"), (4, ">i"), (8, ">q")):
        lo, hi = -(1 << (8 * n - 1)), (1 << (8 * n - 1)) - 1
        if lo <= v <= hi:
            return struct.pack(fmt, v)
    raise ValueError(v)


def encode_point(ts_ms, base_s, bits, is_float, float4=False, force_ms=False):
    off_ms = ts_ms - base_s * 1000
    if is_float:
        d = float(np.int64(bits).view(np.float64))
        vb = struct.pack(">f", d) if float4 else struct.pack(">d", d)
        flags = 0x8 | (len(vb) - 1)
    else:
        vb = _long_bytes(int(bits))
        flags = len(vb) - 1
    if off_ms % 1000 == 0 and not force_ms:
        q = struct.pack(">H", ((off_ms // 1000) << 4) | flags)
    else:
        q = struct.pack(">I", 0xF0000000 | (off_ms << 6) | flags)
    return q, vb


def encode_series(ts, bits, isf, rng=None, float4_frac=0.0, ms_frac=0.0):
    """Rows (base_s, qual bytes, value bytes) of one series."""
    rows = []
    if len(ts) == 0:
        return rows
    bases = (ts // 1000) - (ts // 1000) % 3600
    for base in np.unique(bases):
        sel = np.nonzero(bases == base)[0]
        q, v = b"", b""
        kinds = set()
        for i in sel:
            f4 = bool(rng is not None and isf[i] and rng.random() < float4_frac)
            fm = bool(rng is not None and rng.random() < ms_frac)
            qq, vv = encode_point(int(ts[i]), int(base), int(bits[i]),
                                  bool(isf[i]), f4, fm)
            q += qq
            v += vv
            kinds.add(len(qq))
        if len(sel) > 1:
            v += bytes([1 if len(kinds) > 1 else 0])
        rows.append((int(base), q, v))
    return rows


def encode_batch(batch, rng=None, float4_frac=0.0, ms_frac=0.0):
    """-> dict of numpy arrays forming an otsdb_cells."""
    rs, rb, qo, vo = [], [], [0], [0]
    qb, vb = bytearray(), bytearray()
    isf = batch.is_float
    for s in range(batch.n_series):
        a, b = batch.offsets[s], batch.offsets[s + 1]
        f = isf[a:b] if isf is not None else np.ones(b - a, np.uint8)
        for base, q, v in encode_series(batch.ts[a:b], batch.val[a:b], f, rng,
                                        float4_frac, ms_frac):
            rs.append(s)
            rb.append(base)
            qb += q
            vb += v
            qo.append(len(qb))
            vo.append(len(vb))
    return dict(row_series=np.array(rs, np.int64),
                row_base_s=np.array(rb, np.int64),
                qual_off=np.array(qo, np.int64),
                qual=np.frombuffer(bytes(qb) + b"\0", np.uint8),
                val_off=np.array(vo, np.int64),
                val=np.frombuffer(bytes(vb) + b"\0", np.uint8))


def batch_from_rows(rows, like):
    """A HostBatch of the points in compacted rows [(series, base_s, qual,
    val)] (rows of a series in base-time order; RowSeq decode by the
    oracle), with `like`'s series count and groups."""
    from oracle import pyoracle
    from opentsdb_amd.batch import HostBatch
    per = [[] for _ in range(like.n_series)]
    for s, base, q, v in rows:
        per[s].append(pyoracle.decode_row(q, v, base))
    offs, ts, bits, isf = [0], [], [], []
    for s in range(like.n_series):
        pts = (np.concatenate(per[s]) if per[s]
               else np.zeros(0, pyoracle.POINT))
        ts.append(pts["ts"])
        bits.append(pts["bits"])
        isf.append(1 - pts["is_int"].astype(np.uint8))
        offs.append(offs[-1] + len(pts))
    return HostBatch(np.array(offs, np.int64), np.concatenate(ts),
                     np.concatenate(bits), np.concatenate(isf), None,
                     like.group_offsets, like.group_members)
