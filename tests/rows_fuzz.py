"""Seeded generators of storage rows for the compaction / span-assembly tests:
single cells (2-byte seconds, 4-byte ms), compacted columns (sometimes out of
time order or with a repeated offset), append columns (pairs in any order,
repeated offsets), annotations / histograms, legacy cells needing the
fix-ups, and deliberately corrupt columns.  Plain numpy / bytes."""
import struct

import numpy as np

BASE = 1356998400


def sec_qual(off_s, flags):
    return struct.pack(">H", ((off_s << 4) | flags) & 0xFFFF)


def ms_qual(off_ms, flags):
    return struct.pack(">I", 0xF0000000 | (off_ms << 6) | flags)


def enc_value(rng, kind=None):
    """(flags, value bytes) of a random well-formed value."""
    kind = kind if kind is not None else int(rng.integers(0, 6))
    if kind == 0:
        return 0x0, struct.pack(">b", int(rng.integers(-128, 128)))
    if kind == 1:
        return 0x1, struct.pack(">h", int(rng.integers(-30000, 30000)))
    if kind == 2:
        return 0x3, struct.pack(">i", int(rng.integers(-2**31, 2**31)))
    if kind == 3:
        return 0x7, struct.pack(">q", int(rng.integers(-2**62, 2**62)))
    if kind == 4:
        return 0xB, struct.pack(">f", float(rng.normal()))
    return 0xF, struct.pack(">d", float(rng.normal()))


def cell(rng, off_ms, ms=None, value=None):
    """One (qualifier, value) point at offset off_ms."""
    if ms is None:
        ms = off_ms % 1000 != 0 or rng.random() < 0.2
    fl, v = value if value is not None else enc_value(rng)
    q = ms_qual(off_ms, fl) if ms else sec_qual(off_ms // 1000, fl)
    return q, v


def compacted(cells, meta=None):
    """A compacted column of (qualifier, value) points, meta byte appended
    for more than one point (bit 0 = seconds and ms mixed)."""
    q = b"".join(c[0] for c in cells)
    v = b"".join(c[1] for c in cells)
    if len(cells) > 1:
        if meta is None:
            kinds = {len(c[0]) for c in cells}
            meta = 1 if len(kinds) > 1 else 0
        v += bytes([meta])
    return q, v


def random_offsets(rng, n, pool_s=40, ms_frac=0.3):
    out = []
    for _ in range(n):
        if rng.random() < ms_frac:
            out.append(int(rng.integers(0, pool_s * 1000)))
        else:
            out.append(int(rng.integers(0, pool_s)) * 1000)
    return out


def random_row(rng, corrupt=0.0, unsorted=0.1, max_cols=6):
    """Columns [(qualifier, value, hbase_ts)] of one storage row."""
    cols = []
    ncol = int(rng.integers(1, max_cols + 1))
    shared = random_offsets(rng, 4)  # offsets several columns hit
    vals = {}
    ts_pool = list(rng.permutation(ncol * 3))
    for ci in range(ncol):
        ts = int(ts_pool[ci]) if rng.random() < 0.8 else 0  # ties sometimes
        kind = rng.random()
        def pick_off():
            return shared[int(rng.integers(0, 4))] if rng.random() < 0.4 else \
                random_offsets(rng, 1)[0]
        def val_for(off):
            # duplicates mostly carry the same value
            if off in vals and rng.random() < 0.7:
                return vals[off]
            v = enc_value(rng)
            vals.setdefault(off, v)
            return v
        if kind < 0.35:  # single cell
            off = pick_off()
            q, v = cell(rng, off, value=val_for(off))
            cols.append((q, v, ts))
        elif kind < 0.7:  # compacted column
            n = int(rng.integers(2, 12))
            offs = sorted(pick_off() for _ in range(n))
            if rng.random() < 0.2 and n > 2:  # a repeated offset
                offs[1] = offs[0]
            if rng.random() < unsorted:
                i = int(rng.integers(0, n - 1))
                offs[i], offs[i + 1] = offs[i + 1], offs[i]
            cs = [cell(rng, o, value=val_for(o)) for o in offs]
            q, v = compacted(cs)
            cols.append((q, v, ts))
        elif kind < 0.85:  # append column
            n = int(rng.integers(1, 8))
            offs = [pick_off() for _ in range(n)]
            pairs = b""
            for o in offs:
                q, v = cell(rng, o, value=val_for(o))
                pairs += q + v
            cols.append((bytes([5, 0, 0]), pairs, ts))
        elif kind < 0.92:  # annotation / histogram
            pre = 1 if rng.random() < 0.7 else 6
            cols.append((bytes([pre, 0, int(rng.integers(0, 255))]),
                         b'{"x":1}', ts))
        else:  # legacy single cells needing a fix-up
            off = int(rng.integers(0, 40))
            if rng.random() < 0.5:  # a 4-byte float stored in 8 bytes
                f = struct.pack(">f", float(rng.normal()))
                cols.append((sec_qual(off, 0xB), b"\0\0\0\0" + f, ts))
            else:  # length bits disagree with the value
                cols.append((sec_qual(off, 0x3),
                             struct.pack(">q", int(rng.integers(-99, 99))), ts))
    if corrupt and rng.random() < corrupt:
        k = int(rng.integers(0, 6))
        if k == 0:  # float fix-up with a non-zero high half
            cols.append((sec_qual(7, 0xB), b"\1\0\0\0\0\0\0\1", 0))
        elif k == 1:  # append pairs that do not break down
            cols.append((bytes([5, 0, 0]), sec_qual(3, 0x7) + b"\0\0\0", 0))
        elif k == 2:  # an append qualifier of the wrong length
            cols.append((bytes([5, 0, 0, 0, 0]), b"", 0))
        elif k == 3:  # a compacted column whose values are short
            q, v = compacted([cell(rng, 1000, False), cell(rng, 2000, False)])
            cols.append((q, v[:-3], 0))
        elif k == 4:  # a data column without value bytes
            cols.append((sec_qual(9, 0x7), b"", 0))
        else:  # a 2-byte qualifier with the ms flag
            cols.append((bytes([0xF0, 0x07]), b"\0" * 8, 0))
    order = rng.permutation(len(cols))
    return [cols[i] for i in order]


def random_compacted_row(rng, n=None, ms_frac=0.2, pool_s=3600):
    """A well-formed compacted column (strictly increasing offsets)."""
    n = n or int(rng.integers(1, 20))
    offs = sorted(set(random_offsets(rng, n, pool_s=pool_s, ms_frac=ms_frac)))
    return compacted([cell(rng, o, o % 1000 != 0) for o in offs])


def scatter_row(rng, points, mode=None):
    """Columns [(qualifier, value, hbase_ts)] holding exactly the points
    [(qualifier, value)] of one row (strictly increasing offsets) after the
    reference's compaction: one compacted column, single-point cells in any
    column order, several compacted pieces plus repeated cells with equal
    bytes, an append column with repeated pairs, or a mix with annotations."""
    n = len(points)
    mode = int(rng.integers(0, 5)) if mode is None else mode
    ts = lambda: int(rng.integers(0, 1000))  # noqa: E731
    if mode == 0 or n == 1:
        q, v = compacted(points)
        return [(q, v, ts())]
    if mode == 1:
        cols = [(q, v, ts()) for q, v in points]
        return [cols[i] for i in rng.permutation(n)]
    if mode == 2:
        cuts = sorted(set(int(x) for x in rng.integers(1, n, size=2)))
        pieces, a = [], 0
        for c in cuts + [n]:
            if c > a:
                pieces.append(points[a:c])
            a = c
        cols = [compacted(p) + (ts(),) for p in pieces]
        for _ in range(int(rng.integers(1, 4))):
            q, v = points[int(rng.integers(0, n))]
            cols.append((q, v, ts()))
        return [cols[i] for i in rng.permutation(len(cols))]
    if mode == 3:
        pairs = list(points) + [points[int(rng.integers(0, n))]
                                for _ in range(int(rng.integers(0, 3)))]
        order = rng.permutation(len(pairs))
        return [(bytes([5, 0, 0]), b"".join(pairs[i][0] + pairs[i][1]
                                            for i in order), ts())]
    h = n // 2
    cols = [compacted(points[:h]) + (ts(),),
            (bytes([5, 0, 0]), b"".join(q + v for q, v in points[h:]), ts()),
            (bytes([1, 0, 0]), b'{"note":1}', ts())]
    return [cols[i] for i in rng.permutation(3)]


def split_points(q, v):
    """(qualifier, value) points of a well-formed compacted column."""
    out, qi, vi = [], 0, 0
    while qi < len(q):
        ql = 4 if (q[qi] & 0xF0) == 0xF0 else 2
        vl = (q[qi + ql - 1] & 0x7) + 1
        out.append((q[qi:qi + ql], v[vi:vi + vl]))
        qi += ql
        vi += vl
    return out


def _offsets(q):
    out, qi = [], 0
    while qi + 2 <= len(q):
        if (q[qi] & 0xF0) == 0xF0:
            if qi + 4 > len(q):
                break
            out.append((int.from_bytes(q[qi:qi + 4], "big") & 0x0FFFFFC0) >> 6)
            qi += 4
        else:
            out.append((int.from_bytes(q[qi:qi + 2], "big") >> 4) * 1000)
            qi += 2
    return out


def heap_with_append(cols):
    """True when a row holds an append column next to a data column whose
    offsets go back in time: the GPU's documented UnsupportedOperation case
    (rows.hip), which the write path and compaction never produce."""
    app = any(len(q) % 2 == 1 and q[0] == 5 for q, _, _ in cols)
    if not app:
        return False
    for q, _, _ in cols:
        if len(q) % 2 == 0 and len(q) > 2:
            o = _offsets(q)
            if any(b < a for a, b in zip(o, o[1:])):
                return True
    return False
