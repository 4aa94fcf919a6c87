"""Storage rows as the scanner returns them, and the query-time compaction /
span assembly entry points over them.

A storage row is one (series, base hour) row key with its columns: single
point cells, compacted columns, append columns (qualifier ``05 00 00``),
annotations (``01 ..``) and histograms (``06 ..``).  ``TsdbQuery`` hands each
row to ``TSDB.compact`` (``SaltScanner.java:849-881``) and the compacted
column to ``Span.addRow`` (``Span.java:177-220``); ``otsdb_compact_rows_device``
and ``otsdb_span_assemble_device`` are those two steps for a whole query on
the GPU, and ``otsdb_agg_run_raw[_device]`` chains them into the fused
cells query.  Host-side packing only; every byte is merged on the device.
"""
import ctypes as C

import numpy as np

from . import abi


class HostRawRows:
    """Packs rows [(series, base_s, [(qualifier, value[, hbase_ts]), ...])]
    into the CSR arrays of ``otsdb_raw_rows`` (host numpy)."""

    def __init__(self, rows, with_ts=None):
        self.n_rows = len(rows)
        self.row_series = np.asarray([r[0] for r in rows] or [0], np.int64)
        self.row_base_s = np.asarray([r[1] for r in rows] or [0], np.int64)
        cols = [c for r in rows for c in r[2]]
        ncol = np.asarray([len(r[2]) for r in rows], np.int64)
        self.row_col_off = np.concatenate([[0], np.cumsum(ncol)]).astype(np.int64)
        qs = [bytes(c[0]) for c in cols]
        vs = [bytes(c[1]) for c in cols]
        self.col_qual_off = np.concatenate(
            [[0], np.cumsum([len(q) for q in qs])]).astype(np.int64)
        self.col_val_off = np.concatenate(
            [[0], np.cumsum([len(v) for v in vs])]).astype(np.int64)
        self.qual = np.frombuffer(b"".join(qs) + b"\0" * 16, np.uint8).copy()
        self.val = np.frombuffer(b"".join(vs) + b"\0" * 16, np.uint8).copy()
        if with_ts is None:
            with_ts = any(len(c) > 2 for c in cols)
        self.col_ts = (np.asarray([c[2] if len(c) > 2 else i
                                   for i, c in enumerate(cols)] or [0], np.int64)
                       if with_ts else None)
        self.n_series = int(self.row_series[:self.n_rows].max()) + 1 \
            if self.n_rows else 0

    def as_abi(self):
        p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        return abi.RawRows(self.n_rows, p(self.row_series), p(self.row_base_s),
                           p(self.row_col_off), p(self.col_qual_off),
                           p(self.qual), p(self.col_val_off), p(self.val),
                           p(self.col_ts))

    def to_device(self, device="cuda"):
        import torch
        t = {k: torch.from_numpy(getattr(self, k)).to(device)
             for k in ("row_series", "row_base_s", "row_col_off",
                       "col_qual_off", "qual", "col_val_off", "val")}
        t["col_ts"] = (None if self.col_ts is None
                       else torch.from_numpy(self.col_ts).to(device))
        return DeviceRawRows(t, self.n_rows, self.n_series,
                             int(self.col_qual_off[-1]),
                             int(self.col_val_off[-1]))


class DeviceRawRows:
    def __init__(self, t, n_rows, n_series, qbytes, vbytes):
        self.t, self.n_rows, self.n_series = t, n_rows, n_series
        self.qbytes, self.vbytes = qbytes, vbytes

    def as_abi(self):
        t = self.t
        return abi.RawRows(self.n_rows, t["row_series"].data_ptr(),
                           t["row_base_s"].data_ptr(),
                           t["row_col_off"].data_ptr(),
                           t["col_qual_off"].data_ptr(), t["qual"].data_ptr(),
                           t["col_val_off"].data_ptr(), t["val"].data_ptr(),
                           None if t["col_ts"] is None
                           else t["col_ts"].data_ptr())


def raw_rows_from_cells(cells):
    """DeviceCells -> DeviceRawRows holding each compacted row as a storage
    row with that one column (what the scanner returns for hours already
    compacted by the TSD); the tensors are shared, not copied."""
    import torch
    t = cells.t
    R = cells.n_rows
    dev = t["qual"].device
    rt = dict(row_series=t["row_series"], row_base_s=t["row_base_s"],
              row_col_off=torch.arange(R + 1, dtype=torch.int64, device=dev),
              col_qual_off=t["qual_off"], qual=t["qual"],
              col_val_off=t["val_off"], val=t["val"], col_ts=None)
    return DeviceRawRows(rt, R, cells.n_series,
                         int(t["qual_off"][-1].item()),
                         int(t["val_off"][-1].item()))


def _cells_out(R, Q, V, device):
    import torch
    t = dict(row_series=torch.zeros(max(R, 1), dtype=torch.int64, device=device),
             row_base_s=torch.zeros(max(R, 1), dtype=torch.int64, device=device),
             qual_off=torch.zeros(R + 1, dtype=torch.int64, device=device),
             val_off=torch.zeros(R + 1, dtype=torch.int64, device=device),
             qual=torch.zeros(Q + 16, dtype=torch.uint8, device=device),
             val=torch.zeros(V + 16, dtype=torch.uint8, device=device))
    o = abi.CellsOut(t["row_series"].data_ptr(), t["row_base_s"].data_ptr(),
                     t["qual_off"].data_ptr(), t["qual"].data_ptr(),
                     t["val_off"].data_ptr(), t["val"].data_ptr())
    return t, o


def compact_rows_device(engine, raw, fix_duplicates=True):
    """otsdb_compact_rows_device -> DeviceCells of the kept rows (with the
    kept row count); raises OtsdbError on the reference's exceptions."""
    from .workload import DeviceCells
    dev = raw.t["qual"].device
    R = raw.n_rows
    Q = raw.qbytes + raw.vbytes
    V = raw.vbytes + R
    t, o = _cells_out(R, Q, V, dev)
    n = C.c_int64()
    r = raw.as_abi()
    engine._check(engine.lib.otsdb_compact_rows_device(
        engine.ctx, C.byref(r), 1 if fix_duplicates else 0, C.byref(o), Q, V,
        C.byref(n), None))
    k = n.value
    for key in ("row_series", "row_base_s"):
        t[key] = t[key][:k]
    t["qual_off"] = t["qual_off"][:k + 1]
    t["val_off"] = t["val_off"][:k + 1]
    return DeviceCells(t, raw.n_series)


def span_assemble_device(engine, cells):
    """otsdb_span_assemble_device -> DeviceCells in span order."""
    from .workload import DeviceCells
    dev = cells.t["qual"].device
    R = cells.n_rows
    Q = int(cells.t["qual_off"][-1].item()) if R else 0
    V = int(cells.t["val_off"][-1].item()) + R if R else 0
    t, o = _cells_out(R, Q, V, dev)
    n = C.c_int64()
    c = cells.as_abi()
    engine._check(engine.lib.otsdb_span_assemble_device(
        engine.ctx, C.byref(c), cells.n_series, C.byref(o), Q, V, C.byref(n),
        None))
    k = n.value
    for key in ("row_series", "row_base_s"):
        t[key] = t[key][:k]
    t["qual_off"] = t["qual_off"][:k + 1]
    t["val_off"] = t["val_off"][:k + 1]
    return DeviceCells(t, cells.n_series)


def cells_rows(cells):
    """DeviceCells -> [(series, base_s, qualifier bytes, value bytes)]."""
    t = {k: v.cpu().numpy() for k, v in cells.t.items()}
    out = []
    for i in range(cells.n_rows):
        q = bytes(t["qual"][t["qual_off"][i]:t["qual_off"][i + 1]])
        v = bytes(t["val"][t["val_off"][i]:t["val_off"][i + 1]])
        out.append((int(t["row_series"][i]), int(t["row_base_s"][i]), q, v))
    return out


def run_raw_device(engine, spec, raw, db_groups, result, fix_duplicates=True):
    """otsdb_agg_run_raw_device: the query from storage rows."""
    b = abi.Batch()
    b.n_series = db_groups.n_series
    b.n_points = 0
    b.n_groups = db_groups.n_groups
    b.group_offsets = db_groups.group_offsets.data_ptr()
    b.group_members = db_groups.group_members.data_ptr()
    r = raw.as_abi()
    res = result.as_abi()
    engine._check(engine.lib.otsdb_agg_run_raw_device(
        engine.ctx, C.byref(spec), C.byref(r), 1 if fix_duplicates else 0,
        C.byref(b), C.byref(res), None))


def run_raw(engine, spec, raw, group_offsets, group_members, capacity,
            fix_duplicates=True):
    """otsdb_agg_run_raw (host buffers, the JNI entry) -> (offsets, ts, val,
    is_int) numpy arrays."""
    go = np.ascontiguousarray(group_offsets, np.int64)
    gm = np.ascontiguousarray(group_members, np.int64)
    b = abi.Batch()
    b.n_series = raw.n_series
    b.n_points = 0
    b.n_groups = len(go) - 1
    b.group_offsets = go.ctypes.data
    b.group_members = gm.ctypes.data if len(gm) else None
    offs = np.zeros(len(go), np.int64)
    ts = np.zeros(max(capacity, 1), np.int64)
    val = np.zeros(max(capacity, 1), np.int64)
    isi = np.zeros(max(capacity, 1), np.uint8)
    res = abi.Result(capacity, offs.ctypes.data, ts.ctypes.data, val.ctypes.data,
                     isi.ctypes.data)
    r = raw.as_abi()
    engine._check(engine.lib.otsdb_agg_run_raw(
        engine.ctx, C.byref(spec), C.byref(r), 1 if fix_duplicates else 0,
        C.byref(b), C.byref(res)))
    n = int(offs[-1])
    return offs, ts[:n], val[:n], isi[:n]


def run_cells(engine, spec, cells, n_series, group_offsets, group_members,
              capacity):
    """otsdb_agg_run_cells (host buffers: the JNI entry at the TsdbQuery
    seam).  cells: dict of numpy arrays (row_series, row_base_s, qual_off,
    qual, val_off, val) -> (offsets, ts, val, is_int)."""
    R = len(cells["row_series"])
    arr = {k: np.ascontiguousarray(v) for k, v in cells.items()}
    c = abi.Cells(R, arr["row_series"].ctypes.data, arr["row_base_s"].ctypes.data,
                  arr["qual_off"].ctypes.data, arr["qual"].ctypes.data,
                  arr["val_off"].ctypes.data, arr["val"].ctypes.data)
    go = np.ascontiguousarray(group_offsets, np.int64)
    gm = np.ascontiguousarray(group_members, np.int64)
    b = abi.Batch()
    b.n_series = n_series
    b.n_points = 0
    b.n_groups = len(go) - 1
    b.group_offsets = go.ctypes.data
    b.group_members = gm.ctypes.data if len(gm) else None
    offs = np.zeros(len(go), np.int64)
    ts = np.zeros(max(capacity, 1), np.int64)
    val = np.zeros(max(capacity, 1), np.int64)
    isi = np.zeros(max(capacity, 1), np.uint8)
    res = abi.Result(capacity, offs.ctypes.data, ts.ctypes.data, val.ctypes.data,
                     isi.ctypes.data)
    engine._check(engine.lib.otsdb_agg_run_cells(
        engine.ctx, C.byref(spec), C.byref(c), C.byref(b), C.byref(res)))
    n = int(offs[-1])
    return offs, ts[:n], val[:n], isi[:n]
