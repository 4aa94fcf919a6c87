"""BASELINE.json workloads and their synthetic data.

Series s of the synthetic dataset has tags host = s // 10, cpu = s % 10,
dc = host % 16; series are numbered in SpanCmp order (host, cpu UIDs are
assigned in that order).  The per-series generator (seed 42, T0 =
1356998400 s, 10 s cadence, 2 % dropped points, 0-2 outages of 1-6 h, 5 %
late-start/early-end series) runs on the GPU through the C-ABI
(otsdb_gen_*_device) and is restated bit for bit by the oracle
(or_gen_fill) for parity tests.
"""
import numpy as np

from . import abi, core

T0_S = 1356998400
DAY_MS = 86400 * 1000

# name -> (n_series, days, value kind, query) ; query = (agg, ds, rate opts,
# group-by tag)
CONFIGS = {
    # configs[0]: CPU reference
    "C1": dict(n_series=1000, days=1, kind=0, agg="sum", ds="1m-avg",
               rate=None, group="host"),
    # configs[1]: the single-GPU bench workload
    "C2": dict(n_series=100000, days=7, kind=0, agg="zimsum", ds="5m-avg",
               rate=None, group="host"),
    # configs[2]: 8 GPU, LERP, cross-rank partial all-reduce
    "C3": dict(n_series=1000000, days=1, kind=0, agg="avg", ds="1h-max",
               rate=None, group="dc"),
    # configs[3]: counters
    "C4": dict(n_series=500000, days=1, kind=2, agg="dev", ds="1m-sum",
               rate=(True, 2**63 - 1, 1000000), group=None),
    # configs[4]: percentiles with fill=nan
    "C5": dict(n_series=1000000, days=1, kind=0, agg="p99", ds="1m-avg-nan",
               rate=None, group=None),
}


def gen_spec(name):
    c = CONFIGS[name]
    return abi.GenSpec(42, T0_S * 1000, c["days"] * DAY_MS, 10000, c["kind"],
                       0)


def group_of(name, s):
    g = CONFIGS[name]["group"]
    if g == "host":
        return s // 10
    if g == "dc":
        return (s // 10) % 16
    return 0


def group_ids(name, series0, n):
    s = np.arange(series0, series0 + n, dtype=np.int64)
    g = CONFIGS[name]["group"]
    if g == "host":
        return s // 10
    if g == "dc":
        return (s // 10) % 16
    return np.zeros(n, np.int64)


def query_spec(name, series0=0):
    """The TsdbQuery a user would send: [T0, T0 + days - 1 s]; the SpanGroup
    window comes from getScanStart/EndTimeSeconds (TsdbQuery.java:1573-1675)
    normalised to ms (SpanGroup.java:267-270)."""
    c = CONFIGS[name]
    ds = core.DownsamplingSpecification(c["ds"])
    q_start = T0_S
    q_end = T0_S + c["days"] * 86400 - 1
    start_s = core.get_scan_start_time_seconds(q_start, ds)
    end_s = core.get_scan_end_time_seconds(q_end, ds)
    ro = core.RateOptions(*c["rate"]) if c["rate"] else None
    return core.make_spec(start_s, end_s, core.Aggregators.get(c["agg"]), ds,
                          q_start * 1000, q_end * 1000, c["rate"] is not None,
                          ro, normalize=True)


# configs quoted on 8 GPUs: the config's series count is the node total
NODE_CONFIGS = {"C3": 8, "C5": 8}


def default_series_per_gpu(name):
    c = CONFIGS[name]
    return c["n_series"] // NODE_CONFIGS.get(name, 1)


def n_groups_global(name, n_series_total):
    g = CONFIGS[name]["group"]
    if g == "host":
        return (n_series_total + 9) // 10
    if g == "dc":
        return min(16, (n_series_total + 9) // 10)
    return 1


def spans_ranks(name):
    """Groups of this config can hold series of several ranks."""
    return CONFIGS[name]["group"] != "host"


def global_groups(name, series0, n, G):
    """Group CSR of series [series0, series0+n) over ALL G global groups
    (empty groups where this shard has no member) — the layout of the
    cross-rank protocols."""
    gid = group_ids(name, series0, n)
    order = np.argsort(gid, kind="stable").astype(np.int64)
    counts = np.bincount(gid, minlength=G)
    g_off = np.zeros(G + 1, np.int64)
    np.cumsum(counts, out=g_off[1:])
    return g_off, order


def local_groups(name, series0, n):
    """Group CSR for series [series0, series0+n) with group ids made dense
    and kept in ByteMap (= numeric) order; returns (g_off, members,
    global_group_ids)."""
    gid = group_ids(name, series0, n)
    uniq, dense = np.unique(gid, return_inverse=True)
    order = np.argsort(dense, kind="stable").astype(np.int64)
    counts = np.bincount(dense, minlength=len(uniq))
    g_off = np.zeros(len(uniq) + 1, np.int64)
    np.cumsum(counts, out=g_off[1:])
    return g_off, order, uniq


def generate_device(engine, gspec, series0, n_series, group_size=None,
                    config=None, device="cuda", n_groups=None):
    """Generates series [series0, series0+n) straight into HBM and returns a
    DeviceBatch (torch tensors)."""
    import ctypes as C
    import torch
    from .engine import DeviceBatch
    counts = torch.zeros(n_series, dtype=torch.int64, device=device)
    engine._check(engine.lib.otsdb_gen_counts_device(
        engine.ctx, C.byref(gspec), series0, n_series, counts.data_ptr(),
        None))
    offsets = torch.zeros(n_series + 1, dtype=torch.int64, device=device)
    torch.cumsum(counts, 0, out=offsets[1:])
    N = int(offsets[-1].item())
    ts = torch.empty(max(N, 2), dtype=torch.int64, device=device)
    val = torch.empty(max(N, 2), dtype=torch.int64, device=device)
    engine._check(engine.lib.otsdb_gen_fill_device(
        engine.ctx, C.byref(gspec), series0, n_series, offsets.data_ptr(),
        ts.data_ptr(), val.data_ptr(), None))
    torch.cuda.synchronize()
    if config is not None and n_groups is not None:
        g_off, members = global_groups(config, series0, n_series, n_groups)
    elif config is not None:
        g_off, members, _ = local_groups(config, series0, n_series)
    else:
        gs = group_size or n_series
        gid = (np.arange(series0, series0 + n_series) // gs)
        gid = gid - gid[0] if n_series else gid
        from .batch import groups_from_ids
        g_off, members = groups_from_ids(gid)
    sf = torch.full((n_series,), 1 if gspec.kind == 0 else 0,
                    dtype=torch.uint8, device=device)
    db = DeviceBatch(offsets, ts[:N] if N else ts[:0], val[:N] if N else val[:0],
                     torch.from_numpy(g_off).to(device),
                     torch.from_numpy(members).to(device), None, sf)
    db.n_points_total = N
    return db


class DeviceCells:
    """Compacted RowSeq columns in HBM (otsdb_cells), kept alive with their
    torch tensors."""

    def __init__(self, t, n_series):
        self.t = t
        self.n_series = n_series
        self.n_rows = t["row_series"].numel()
        self.n_bytes = (t["qual"].numel() + t["val"].numel() +
                        16 * self.n_rows)

    def as_abi(self):
        t = self.t
        return abi.Cells(self.n_rows, t["row_series"].data_ptr(),
                         t["row_base_s"].data_ptr(), t["qual_off"].data_ptr(),
                         t["qual"].data_ptr(), t["val_off"].data_ptr(),
                         t["val"].data_ptr())


def encode_cells_device(engine, db):
    """The columnar DeviceBatch db as compacted cells in HBM
    (otsdb_encode_cells_device: count, scan, fill)."""
    import ctypes as C
    import torch
    dev = db.ts.device
    S = db.n_series
    cnt = [torch.zeros(S, dtype=torch.int64, device=dev) for _ in range(3)]
    b = db.as_abi()
    engine._check(engine.lib.otsdb_encode_cells_device(
        engine.ctx, C.byref(b), cnt[0].data_ptr(), cnt[1].data_ptr(),
        cnt[2].data_ptr(), None, None))
    tot = [int(c.sum().item()) for c in cnt]
    base = [torch.cumsum(c, 0) - c for c in cnt]  # exclusive prefix sums
    R, Q, V = tot
    t = dict(row_series=torch.empty(max(R, 1), dtype=torch.int64, device=dev),
             row_base_s=torch.empty(max(R, 1), dtype=torch.int64, device=dev),
             qual_off=torch.empty(R + 1, dtype=torch.int64, device=dev),
             val_off=torch.empty(R + 1, dtype=torch.int64, device=dev),
             qual=torch.zeros(Q + 16, dtype=torch.uint8, device=dev),
             val=torch.zeros(V + 16, dtype=torch.uint8, device=dev))
    out = abi.CellsOut(t["row_series"].data_ptr(), t["row_base_s"].data_ptr(),
                       t["qual_off"].data_ptr(), t["qual"].data_ptr(),
                       t["val_off"].data_ptr(), t["val"].data_ptr())
    engine._check(engine.lib.otsdb_encode_cells_device(
        engine.ctx, C.byref(b), base[0].data_ptr(), base[1].data_ptr(),
        base[2].data_ptr(), C.byref(out), None))
    t["qual_off"][R] = Q
    t["val_off"][R] = V
    t["row_series"] = t["row_series"][:R]
    t["row_base_s"] = t["row_base_s"][:R]
    torch.cuda.synchronize()
    return DeviceCells(t, S)


def decode_cells_device(engine, cells, capacity=None, out=None):
    """otsdb_decode_cells_device -> (offsets, ts, val, is_float) tensors.
    out: preallocated (offsets, ts, val, is_float) to decode into (the
    bench times the decode without the allocation)."""
    import ctypes as C
    import torch
    dev = cells.t["qual"].device
    S = cells.n_series
    c = cells.as_abi()
    if out is not None:
        offsets, ts, val, isf = out
        capacity = int(ts.numel())
    else:
        offsets = torch.zeros(S + 1, dtype=torch.int64, device=dev)
    if capacity is None:
        engine._check(engine.lib.otsdb_decode_cells_device(
            engine.ctx, C.byref(c), S, offsets.data_ptr(), None, None, None,
            0, None))
        capacity = int(offsets[-1].item())
    if out is None:
        ts = torch.empty(max(capacity, 2), dtype=torch.int64, device=dev)
        val = torch.empty_like(ts)
        isf = torch.empty(max(capacity, 2), dtype=torch.uint8, device=dev)
    engine._check(engine.lib.otsdb_decode_cells_device(
        engine.ctx, C.byref(c), S, offsets.data_ptr(), ts.data_ptr(),
        val.data_ptr(), isf.data_ptr(), capacity, None))
    return offsets, ts[:capacity], val[:capacity], isf[:capacity]


def run_cells_device(engine, spec, cells, db_groups, result):
    """otsdb_agg_run_cells_device: the query straight from compacted columns
    (decode fused into the downsample).  db_groups: a DeviceBatch-like object
    supplying n_series and the group arrays."""
    import ctypes as C
    b = abi.Batch()
    b.n_series = cells.n_series
    b.n_points = 0
    b.n_groups = db_groups.n_groups
    b.group_offsets = db_groups.group_offsets.data_ptr()
    b.group_members = db_groups.group_members.data_ptr()
    c = cells.as_abi()
    r = result.as_abi()
    engine._check(engine.lib.otsdb_agg_run_cells_device(
        engine.ctx, C.byref(spec), C.byref(c), C.byref(b), C.byref(r), None))
