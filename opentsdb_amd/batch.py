"""Columnar query batch (the otsdb_batch of include/otsdb_agg.h) on the host.

A batch is what TsdbQuery.GroupByAndAggregateCB hands to the engine: the
spans of one query in SpanCmp order (TsdbQuery.java:1862-1892) flattened to
CSR columns, plus the group membership built by the group-by step
(TsdbQuery.java:1062-1112).
"""
import numpy as np

from . import abi


def _ptr(a):
    return None if a is None else a.ctypes.data


class HostBatch:
    def __init__(self, offsets, ts, val, is_float=None, series_float=None,
                 group_offsets=None, group_members=None):
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self.ts = np.ascontiguousarray(ts, dtype=np.int64)
        self.val = np.ascontiguousarray(val, dtype=np.int64)
        self.is_float = (None if is_float is None else
                         np.ascontiguousarray(is_float, dtype=np.uint8))
        self.series_float = (None if series_float is None else
                             np.ascontiguousarray(series_float, dtype=np.uint8))
        S = len(self.offsets) - 1
        if group_offsets is None:  # one group with every series
            group_offsets = np.array([0, S], dtype=np.int64)
            group_members = np.arange(S, dtype=np.int64)
        self.group_offsets = np.ascontiguousarray(group_offsets, np.int64)
        self.group_members = np.ascontiguousarray(group_members, np.int64)

    @property
    def n_series(self):
        return len(self.offsets) - 1

    @property
    def n_groups(self):
        return len(self.group_offsets) - 1

    def as_abi(self):
        b = abi.Batch()
        b.n_series = self.n_series
        b.n_points = int(self.offsets[-1]) if len(self.offsets) else 0
        b.offsets = _ptr(self.offsets)
        b.ts_ms = _ptr(self.ts)
        b.val = _ptr(self.val)
        b.is_float = _ptr(self.is_float)
        b.series_float = _ptr(self.series_float)
        b.n_groups = self.n_groups
        b.group_offsets = _ptr(self.group_offsets)
        b.group_members = _ptr(self.group_members)
        return b

    # -------------------------------------------------------------- builders
    @staticmethod
    def from_groups(groups):
        """groups: list of groups; each group a list of spans; each span a
        list of (ts_ms, value, is_float) triples (the DataPoint[] of a
        MockSeekableView).  Series are numbered in group order."""
        offs = [0]
        ts, val, isf = [], [], []
        g_off = [0]
        members = []
        s = 0
        for g in groups:
            for span in g:
                for (t, v, f) in span:
                    ts.append(int(t))
                    if f:
                        val.append(np.float64(v).view(np.int64))
                    else:
                        val.append(int(v))
                    isf.append(1 if f else 0)
                offs.append(len(ts))
                members.append(s)
                s += 1
            g_off.append(len(members))
        return HostBatch(np.array(offs, np.int64), np.array(ts, np.int64),
                         np.array(val, np.int64), np.array(isf, np.uint8),
                         None, np.array(g_off, np.int64),
                         np.array(members, np.int64))


def groups_from_ids(group_id, n_groups=None):
    """Stable CSR group membership from a per-series group id (series keep
    their SpanCmp order inside each group)."""
    gid = np.asarray(group_id, dtype=np.int64)
    G = int(gid.max()) + 1 if n_groups is None else int(n_groups)
    order = np.argsort(gid, kind="stable").astype(np.int64)
    counts = np.bincount(gid, minlength=G)
    g_off = np.zeros(G + 1, np.int64)
    np.cumsum(counts, out=g_off[1:])
    return g_off, order
