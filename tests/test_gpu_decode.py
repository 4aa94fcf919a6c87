"""Compacted-cell decode on the GPU (RowSeq semantics) against the oracle's
RowSeq.Iterator restatement, and decode -> aggregate against the columnar
path."""
import ctypes as C

import numpy as np
import pytest

from opentsdb_amd import abi, core
from opentsdb_amd.engine import Engine
from oracle import pyoracle
from tests import cells, datasets

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = Engine(0)
    yield e
    e.close()


def decode_gpu(engine, enc, S):
    import torch
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
         for k, v in enc.items()}
    cs = abi.Cells(len(enc["row_series"]), d["row_series"].data_ptr(),
                   d["row_base_s"].data_ptr(), d["qual_off"].data_ptr(),
                   d["qual"].data_ptr(), d["val_off"].data_ptr(),
                   d["val"].data_ptr())
    offs = torch.zeros(S + 1, dtype=torch.int64, device="cuda")
    engine._check(engine.lib.otsdb_decode_cells_device(
        engine.ctx, C.byref(cs), S, offs.data_ptr(), None, None, None, 0,
        None))
    n = int(offs[-1].item())
    ts = torch.empty(max(n, 2), dtype=torch.int64, device="cuda")
    val = torch.empty(max(n, 2), dtype=torch.int64, device="cuda")
    isf = torch.empty(max(n, 2), dtype=torch.uint8, device="cuda")
    engine._check(engine.lib.otsdb_decode_cells_device(
        engine.ctx, C.byref(cs), S, offs.data_ptr(), ts.data_ptr(),
        val.data_ptr(), isf.data_ptr(), n, None))
    torch.cuda.synchronize()
    return (offs.cpu().numpy(), ts[:n].cpu().numpy(), val[:n].cpu().numpy(),
            isf[:n].cpu().numpy())


@pytest.mark.parametrize("kind,f4,ms", [("float", 0.0, 0.0), ("int", 0, 0.0),
                                        ("mixed", 0.3, 0.2), ("float", 0, 1.0)])
def test_decode_roundtrip_and_oracle(engine, kind, f4, ms):
    rng = np.random.default_rng(5)
    b = datasets.random_batch(3, n_series=20, n_groups=2, value_kind=kind,
                              cadence_ms=7000 if ms else 10000)
    if ms:  # millisecond timestamps
        b.ts = b.ts + rng.integers(0, 999, len(b.ts))
        b.ts.sort()  # keep rows sorted
        for s in range(b.n_series):
            a, z = b.offsets[s], b.offsets[s + 1]
            b.ts[a:z] = np.sort(b.ts[a:z])
    enc = cells.encode_batch(b, rng, f4, ms)
    offs, ts, val, isf = decode_gpu(engine, enc, b.n_series)
    # oracle: RowSeq.Iterator row by row
    ref_ts, ref_bits, ref_int = [], [], []
    for r in range(len(enc["row_series"])):
        q = enc["qual"][enc["qual_off"][r]:enc["qual_off"][r + 1]]
        v = enc["val"][enc["val_off"][r]:enc["val_off"][r + 1]]
        p = pyoracle.decode_row(q.tobytes(), v.tobytes(), enc["row_base_s"][r])
        ref_ts.append(p["ts"])
        ref_bits.append(p["bits"])
        ref_int.append(p["is_int"])
    assert np.array_equal(ts, np.concatenate(ref_ts))
    assert np.array_equal(val, np.concatenate(ref_bits))
    assert np.array_equal(isf == 0, np.concatenate(ref_int).astype(bool))
    assert np.array_equal(offs, b.offsets)
    if f4 == 0:  # lossless encoding: the columns come back exactly
        assert np.array_equal(ts, b.ts)
        assert np.array_equal(val, b.val)


def test_decode_corrupt_column(engine):
    b = datasets.random_batch(4, n_series=3, n_groups=1, empty_frac=0)
    enc = cells.encode_batch(b)
    enc["val_off"] = enc["val_off"].copy()
    enc["val_off"][1] -= 1  # first row loses a value byte
    with pytest.raises(core.IllegalDataException):
        decode_gpu(engine, enc, b.n_series)


def test_cells_to_aggregate_matches_columns(engine):
    """decode -> aggregate == aggregate of the original columns."""
    from opentsdb_amd.batch import HostBatch
    b = datasets.random_batch(8, n_series=30, n_groups=3, value_kind="mixed")
    enc = cells.encode_batch(b)
    offs, ts, val, isf = decode_gpu(engine, enc, b.n_series)
    hb = HostBatch(offs, ts, val, isf, None, b.group_offsets, b.group_members)
    spec = core.make_spec(datasets.T0, datasets.T0 + 3 * 3600 * 1000,
                          core.Aggregators.SUM,
                          core.DownsamplingSpecification("1m-avg"))
    got = engine.run(spec, hb)
    ref = engine.run(spec, b)
    for g, r in zip(got, ref):
        assert np.array_equal(g.ts, r.ts) and np.array_equal(g.bits, r.bits)


def _device_batch(hb, kind):
    """A HostBatch with one value type per series on the device."""
    import torch
    from opentsdb_amd.engine import DeviceBatch
    sf = np.full(hb.n_series, 1 if kind == "float" else 0, np.uint8)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa
    ts = torch.zeros(max(len(hb.ts), 2), dtype=torch.int64, device="cuda")
    val = torch.zeros_like(ts)
    ts[:len(hb.ts)] = t(hb.ts)
    val[:len(hb.ts)] = t(hb.val)
    return DeviceBatch(t(hb.offsets), ts[:len(hb.ts)], val[:len(hb.ts)],
                       t(hb.group_offsets), t(hb.group_members), None, t(sf))


@pytest.mark.parametrize("kind,seconds", [("float", False), ("float", True),
                                          ("int", True), ("int", False)])
def test_device_encoder_matches_host_encoder(engine, kind, seconds):
    """otsdb_encode_cells_device writes byte for byte the columns
    tests/cells.py lays out (the write path + compaction format), and the
    decoder turns them back into the same points."""
    from opentsdb_amd import workload
    hb = datasets.random_batch(17, n_series=25, n_groups=1, span_ms=3 * 3600000,
                               value_kind=kind, empty_frac=0.1,
                               cadence_ms=10000 if seconds else 7001)
    if seconds:
        hb.ts[:] = hb.ts - hb.ts % 1000
    hb.is_float = np.full(len(hb.ts), 1 if kind == "float" else 0, np.uint8)
    ref = cells.encode_batch(hb)
    db = _device_batch(hb, kind)
    dc = workload.encode_cells_device(engine, db)
    got = {k: v.cpu().numpy() for k, v in dc.t.items()}
    for k in ("row_series", "row_base_s", "qual_off", "val_off"):
        assert np.array_equal(got[k], ref[k]), k
    Q, V = ref["qual_off"][-1], ref["val_off"][-1]
    assert np.array_equal(got["qual"][:Q], ref["qual"][:Q])
    assert np.array_equal(got["val"][:V], ref["val"][:V])
    offs, ts, val, isf = workload.decode_cells_device(engine, dc)
    assert np.array_equal(offs.cpu().numpy(), hb.offsets)
    assert np.array_equal(ts.cpu().numpy(), hb.ts)
    assert np.array_equal(val.cpu().numpy(), hb.val)


@pytest.mark.parametrize("flags", [0, 1])
def test_full_size_cells_roundtrip(engine, flags):
    """C2's whole per-GPU dataset (100k series x 7 days) encoded to compacted
    cells and decoded back: every timestamp and value bit identical (the
    decode's size-independent property at full size)."""
    import gc
    import torch
    from opentsdb_amd import workload
    g = workload.gen_spec("C2")
    g.flags = flags
    n = 100000 if flags else 40000
    db = workload.generate_device(engine, g, 0, n, config="C2")
    dc = workload.encode_cells_device(engine, db)
    offs, ts, val, isf = workload.decode_cells_device(engine, dc)
    assert torch.equal(offs, db.offsets)
    assert torch.equal(ts, db.ts)
    assert torch.equal(val, db.val)
    assert bool((isf == 1).all())
    del db, dc, offs, ts, val, isf
    gc.collect()
    torch.cuda.empty_cache()


def _result_points(res, G):
    from opentsdb_amd.engine import DataPoints
    offs = res.offsets.cpu().numpy()
    return [DataPoints(res.ts[offs[g]:offs[g + 1]].cpu().numpy(),
                       res.val[offs[g]:offs[g + 1]].cpu().numpy(),
                       res.is_int[offs[g]:offs[g + 1]].cpu().numpy())
            for g in range(G)]


FUSED = [("sum", "1m-avg", False), ("zimsum", "5m-sum", False),
         ("avg", "10m-max", False), ("dev", "1m-min", False),
         ("count", "2m-count", False), ("max", "1m-first-nan", False),
         ("min", "1m-last-zero", False), ("p99", "1m-avg", False),
         ("mimmax", "30s-max", False), ("sum", "1m-sum", True),
         ("sum", "1hc-avg", False),
         # buckets spanning storage rows (intervals that do not divide an
         # hour): the open bucket carries from one row to the next
         ("sum", "7m-avg", False), ("avg", "90m-sum", False),
         ("zimsum", "7m-count", False)]


@pytest.mark.parametrize("agg,ds,rate", FUSED,
                         ids=["%s:%s%s" % (a, d, ":rate" if r else "")
                              for a, d, r in FUSED])
@pytest.mark.parametrize("kind,seconds", [("float", True), ("int", True),
                                          ("float", False)])
def test_fused_cells_query(engine, agg, ds, rate, kind, seconds):
    """otsdb_agg_run_cells_device (decode fused into the downsample) against
    the oracle on the same points: timestamps and emission exact, values
    bit-exact for order-free functions, 1e-12 otherwise."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_parity import compare
    hb = datasets.random_batch(29, n_series=40, n_groups=4, span_ms=4 * 3600000,
                               value_kind=kind, counter=rate,
                               cadence_ms=10000 if seconds else 7001)
    if seconds:
        hb.ts[:] = hb.ts - hb.ts % 1000
        # keep the series strictly increasing after flooring
        for s in range(hb.n_series):
            a, b = hb.offsets[s], hb.offsets[s + 1]
            assert (np.diff(hb.ts[a:b]) > 0).all()
    isf = 1 if (kind == "float" and not rate) else 0
    hb.is_float = np.full(len(hb.ts), isf, np.uint8)
    db = _device_batch(hb, "float" if isf else "int")
    cells_d = workload.encode_cells_device(engine, db)
    d = core.DownsamplingSpecification(ds)
    ro = core.RateOptions(True, core.LONG_MAX, 0) if rate else None
    t0, t1 = datasets.T0 + 600000, datasets.T0 + 3 * 3600000
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg), d, t0, t1, rate,
                          ro)
    ref = pyoracle.group_by(spec, hb)
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    workload.run_cells_device(engine, spec, cells_d, db, res)
    got = _result_points(res, db.n_groups)
    fn = ds.split("-")[1]
    exact = fn in ("max", "min", "count", "first", "last") and agg in (
        "max", "min", "count", "mimmax", "p99") and not rate
    # integer data spans both signs: the sums can cancel (60 terms: 6 points
    # per bucket x 10 series); float data is positive
    from tests.test_gpu_parity import cancel_floor
    fl = cancel_floor(hb, 60) if kind == "int" else 0.0
    compare(got, ref, exact, where="fused/%s/%s" % (agg, ds), floor=fl)


@pytest.mark.parametrize("n_series,n_groups", [(40, 4), (1100, 1100)])
@pytest.mark.parametrize("agg,ds", [("sum", "1m-avg"), ("zimsum", "1m-sum"),
                                    ("avg", "1m-max"), ("max", "1m-min-nan"),
                                    ("dev", "1m-avg-zero"), ("count", "1m-count")])
def test_fused_cells_query_multi_window(engine, n_series, n_groups, agg, ds):
    """The cells fold over grids of several fold windows: two days of 1 m
    buckets (2,880 > one 2,048-bucket window; few tiles: narrowed windows of
    128+ buckets; 1,100 single-series groups: two full windows), windows
    starting from k_cells_fold_prep's cursors (row, value offset, length)
    and boundary context (the real buckets either side, LERP across the
    boundary, fills), against the oracle."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_parity import compare
    hb = datasets.random_batch(31, n_series=n_series, n_groups=n_groups,
                               span_ms=2 * 86400000, cadence_ms=20000)
    hb.ts[:] = hb.ts - hb.ts % 1000
    for s in range(hb.n_series):
        a, b = hb.offsets[s], hb.offsets[s + 1]
        assert (np.diff(hb.ts[a:b]) > 0).all()
    hb.is_float = np.ones(len(hb.ts), np.uint8)
    db = _device_batch(hb, "float")
    cells_d = workload.encode_cells_device(engine, db)
    t0, t1 = datasets.T0 + 600000, datasets.T0 + 2 * 86400000 - 300000
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification(ds), t0, t1)
    ref = pyoracle.group_by(spec, hb)
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    workload.run_cells_device(engine, spec, cells_d, db, res)
    got = _result_points(res, db.n_groups)
    exact = ds.split("-")[1] in ("max", "min", "count") and agg in (
        "max", "count")
    compare(got, ref, exact, where="cellsmw/%d/%s/%s" % (n_series, agg, ds))


def test_fused_cells_corrupt_column(engine):
    """A column whose value bytes do not match its qualifiers:
    IllegalDataException, as the decode (Internal.java:307-321)."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult
    hb = datasets.random_batch(31, n_series=6, n_groups=1, span_ms=3600000)
    hb.ts[:] = hb.ts - hb.ts % 1000
    db = _device_batch(hb, "float")
    cd = workload.encode_cells_device(engine, db)
    # drop the last value byte of row 1: every later offset shifts
    cd.t["val_off"][2:] -= 1
    spec = core.make_spec(datasets.T0, datasets.T0 + 3600000,
                          core.Aggregators.SUM,
                          core.DownsamplingSpecification("1m-avg"))
    res = DeviceResult(torch, db.n_groups, 4096, "cuda")
    with pytest.raises(core.IllegalDataException):
        workload.run_cells_device(engine, spec, cd, db, res)


# (name, value kind, int range or None, float4 fraction, ms fraction): cell
# layouts the device encoder does not write — 4-byte floats, 1/2/4/8-byte
# longs of one width per column (the fused kernel's wave-uniform decode),
# mixed widths (its per-point decode), 4-byte ms qualifiers
HOST_FORMATS = [("f8", "float", None, 0.0, 0.0), ("f4", "float", None, 1.0, 0.0),
                ("f4f8", "float", None, 0.5, 0.0), ("i1", "int", (-120, 120), 0, 0),
                ("i2", "int", (-30000, 30000), 0, 0),
                ("i4", "int", (1 << 20, 1 << 30), 0, 0),
                ("i8", "int", (1 << 40, 1 << 50), 0, 0),
                ("imix", "int", (-(1 << 40), 1 << 40), 0, 0),
                ("f8ms", "float", None, 0.0, 1.0), ("i2ms", "int", (300, 30000), 0, 1.0)]


@pytest.mark.parametrize("name,kind,rng_i,f4,ms", HOST_FORMATS,
                         ids=[f[0] for f in HOST_FORMATS])
@pytest.mark.parametrize("agg,ds", [("sum", "1m-avg"), ("max", "5m-max")])
def test_fused_cells_host_formats(engine, name, kind, rng_i, f4, ms, agg, ds):
    """The fused cells query over host-encoded columns of every value width
    and qualifier width against the oracle run on the points RowSeq
    decodes from the same columns."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.batch import HostBatch
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_parity import compare
    rng = np.random.default_rng(11)
    b = datasets.random_batch(17, n_series=24, n_groups=3, value_kind=kind,
                              cadence_ms=7000 if ms else 10000)
    if ms:
        b.ts = b.ts + rng.integers(0, 999, len(b.ts))
        for s in range(b.n_series):
            a, z = b.offsets[s], b.offsets[s + 1]
            b.ts[a:z] = np.sort(b.ts[a:z])
    else:
        b.ts = b.ts - b.ts % 1000
    if rng_i is not None:
        b.val = rng.integers(rng_i[0], rng_i[1], len(b.ts)).astype(np.int64)
        b.is_float = np.zeros(len(b.ts), np.uint8)
    else:
        b.is_float = np.ones(len(b.ts), np.uint8)
    enc = cells.encode_batch(b, rng, f4, ms)
    # the reference points: RowSeq.Iterator over every row
    ts, bits, isint = [], [], []
    for s in range(b.n_series):
        for r in np.nonzero(enc["row_series"] == s)[0]:
            q = enc["qual"][enc["qual_off"][r]:enc["qual_off"][r + 1]]
            v = enc["val"][enc["val_off"][r]:enc["val_off"][r + 1]]
            p = pyoracle.decode_row(q.tobytes(), v.tobytes(),
                                    enc["row_base_s"][r])
            ts.append(p["ts"])
            bits.append(p["bits"])
            isint.append(p["is_int"])
    cat = lambda xs, dt: (np.concatenate(xs).astype(dt) if xs  # noqa
                          else np.zeros(0, dt))
    rts, rbits = cat(ts, np.int64), cat(bits, np.int64)
    risf = (cat(isint, np.uint8) == 0).astype(np.uint8)
    assert len(rts) == len(b.ts)
    hb = HostBatch(b.offsets, rts, rbits, risf, None, b.group_offsets,
                   b.group_members)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
         for k, v in enc.items()}
    dc = workload.DeviceCells(d, b.n_series)
    db = _device_batch(hb, kind)
    t0, t1 = datasets.T0 + 600000, datasets.T0 + 3 * 3600000
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification(ds), t0, t1)
    ref = pyoracle.group_by(spec, hb)
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    workload.run_cells_device(engine, spec, dc, db, res)
    got = _result_points(res, db.n_groups)
    from tests.test_gpu_parity import cancel_floor
    fl = cancel_floor(hb, 60) if kind == "int" else 0.0  # mixed signs
    compare(got, ref, agg == "max", floor=fl,
            where="fused-host/%s/%s/%s" % (name, agg, ds))


def _ragged_rows_batch(seed, n_series, hours, kind):
    """Series whose storage rows hold 1 (no meta byte), 2-7 (fewer than a
    lane's 8 points: the cells fold cuts its step before such a row when it
    sits inside one), ~30 or 360 points, in random order — the row shapes
    sparse or irregular series give."""
    from opentsdb_amd.batch import HostBatch, groups_from_ids
    rng = np.random.default_rng(seed)
    offs, tss, vals = [0], [], []
    for s in range(n_series):
        t = []
        for h in range(hours):
            n = int(rng.choice([0, 1, 2, 3, 5, 7, 8, 30, 360],
                               p=[.05, .15, .1, .1, .1, .1, .1, .15, .15]))
            if n:
                sec = np.sort(rng.choice(3600, n, replace=False))
                t.append(datasets.T0 + h * 3600000 + sec * 1000)
        t = np.concatenate(t) if t else np.zeros(0, np.int64)
        if kind == "float":
            v = (rng.random(len(t)) * 100.0).view(np.int64)
        else:  # 1/2/4/8-byte longs mixed inside rows
            v = rng.integers(-(1 << 40), 1 << 40, len(t)) >> rng.integers(0, 40, len(t))
        tss.append(t.astype(np.int64))
        vals.append(v.astype(np.int64))
        offs.append(offs[-1] + len(t))
    gid = np.arange(n_series) % 3
    g_off, members = groups_from_ids(gid, 3)
    ts, val = np.concatenate(tss), np.concatenate(vals)
    isf = np.full(len(ts), 1 if kind == "float" else 0, np.uint8)
    return HostBatch(np.array(offs, np.int64), ts, val, isf, None, g_off,
                     members)


@pytest.mark.parametrize("kind", ["float", "int"])
@pytest.mark.parametrize("agg,ds,window", [
    ("sum", "5m-avg", "whole"), ("max", "1m-max", "whole"),
    ("zimsum", "7m-count", "whole"), ("avg", "10m-sum", "mid-row"),
    ("min", "1m-first", "mid-row")])
def test_fused_cells_ragged_rows(engine, kind, agg, ds, window):
    """The cells fold over rows of 1 to 360 points (steps cut before short
    inner rows, single-point rows without a meta byte, lanes crossing row
    boundaries), windows starting and ending inside rows, doubles and
    mixed-width longs: against the oracle on the points RowSeq decodes."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_parity import compare, cancel_floor
    hb = _ragged_rows_batch(7 if kind == "float" else 8, 45, 24, kind)
    enc = cells.encode_batch(hb)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
         for k, v in enc.items()}
    dc = workload.DeviceCells(d, hb.n_series)
    db = _device_batch(hb, kind)
    if window == "whole":
        t0, t1 = datasets.T0, datasets.T0 + 24 * 3600000 - 1000
    else:
        t0, t1 = datasets.T0 + 1234567, datasets.T0 + 20 * 3600000 + 777000
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification(ds), t0, t1)
    ref = pyoracle.group_by(spec, hb)
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    workload.run_cells_device(engine, spec, dc, db, res)
    got = _result_points(res, db.n_groups)
    fn = ds.split("-")[1]
    exact = fn in ("max", "count", "first") and agg in ("max", "min")
    fl = cancel_floor(hb, 400) if kind == "int" else 0.0  # mixed signs
    compare(got, ref, exact, where="ragged/%s/%s/%s" % (kind, agg, ds),
            floor=fl)


@pytest.mark.parametrize("layout", ["in-row", "by-row", "by-series", "sparse"])
@pytest.mark.parametrize("agg,ds,rate,days", [
    ("sum", "1m-avg", False, 0), ("dev", "5m-dev", False, 0),
    ("max", "1m-max-nan", False, 0), ("sum", "5m-sum", True, 0),
    ("zimsum", "7m-count", False, 0), ("avg", "1m-avg-zero", False, 2)])
def test_fused_cells_mixed_widths(engine, layout, agg, ds, rate, days):
    """Columns mixing 2-byte second and 4-byte millisecond qualifiers
    (MS_MIXED_COMPACT inside rows, RowSeq.java:338-356), or series whose
    rows alternate between the two widths, or a batch whose series each
    keep one width but not the same one, or sparse rows of both: k_requal
    rewrites them with 4-byte qualifiers and the cells fold streams them
    (one window and, over two days of 1 m buckets, several) — against the
    oracle on the points RowSeq decodes from the original columns."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.batch import HostBatch
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_parity import compare, cancel_floor
    rng = np.random.default_rng(23 + days)
    span = (days or 4) * (86400000 if days else 3600000)
    if layout == "sparse":
        b = _ragged_rows_batch(9, 36, span // 3600000, "int")
        b.ts = b.ts + rng.integers(0, 999, len(b.ts)) * (rng.random(len(b.ts)) < 0.5)
    else:
        b = datasets.random_batch(41 + days, n_series=30, n_groups=3,
                                  span_ms=span, value_kind="int", counter=rate,
                                  cadence_ms=20000 if days else 7000)
        b.ts = b.ts - b.ts % 1000
        ms = rng.integers(1, 999, len(b.ts))
        if layout == "in-row":  # about half the points on milliseconds
            b.ts = b.ts + ms * (rng.random(len(b.ts)) < 0.5)
        elif layout == "by-row":  # odd hours on ms, even hours on seconds
            b.ts = b.ts + ms * (((b.ts - datasets.T0) // 3600000) % 2)
        else:  # odd series on ms (4-byte rows), even ones on seconds
            sid = np.repeat(np.arange(b.n_series), np.diff(b.offsets))
            b.ts = b.ts + ms * (sid % 2)
    for s in range(b.n_series):
        a, z = b.offsets[s], b.offsets[s + 1]
        b.ts[a:z] = np.sort(b.ts[a:z])
        assert (np.diff(b.ts[a:z]) > 0).all()
    b.is_float = np.zeros(len(b.ts), np.uint8)
    enc = cells.encode_batch(b)
    widths = set()
    for r in range(len(enc["row_series"])):
        q = enc["qual"][enc["qual_off"][r]:enc["qual_off"][r + 1]]
        if len(q):
            widths.add(4 if q[0] >> 4 == 0xF else 2)
    assert widths == {2, 4}
    ts, bits, isint = [], [], []
    for r in range(len(enc["row_series"])):
        q = enc["qual"][enc["qual_off"][r]:enc["qual_off"][r + 1]]
        v = enc["val"][enc["val_off"][r]:enc["val_off"][r + 1]]
        p = pyoracle.decode_row(q.tobytes(), v.tobytes(), enc["row_base_s"][r])
        ts.append(p["ts"])
        bits.append(p["bits"])
        isint.append(p["is_int"])
    rts = np.concatenate(ts).astype(np.int64)
    assert np.array_equal(rts, b.ts)
    hb = HostBatch(b.offsets, rts, np.concatenate(bits).astype(np.int64),
                   (np.concatenate(isint) == 0).astype(np.uint8), None,
                   b.group_offsets, b.group_members)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
         for k, v in enc.items()}
    dc = workload.DeviceCells(d, b.n_series)
    db = _device_batch(hb, "int")
    t0, t1 = datasets.T0 + 600000, datasets.T0 + span - 300000
    ro = core.RateOptions(True, core.LONG_MAX, 0) if rate else None
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification(ds), t0, t1, rate, ro)
    ref = pyoracle.group_by(spec, hb)
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    workload.run_cells_device(engine, spec, dc, db, res)
    got = _result_points(res, db.n_groups)
    exact = ds.split("-")[1] in ("max", "count", "dev") and agg in (
        "max", "zimsum", "dev")
    fl = 0.0 if rate else cancel_floor(hb, 400)
    compare(got, ref, exact, floor=fl,
            where="mixedw/%s/%s/%s" % (layout, agg, ds))


def test_fused_cells_mixed_cut_qualifier(engine):
    """A mixed-width column whose last qualifier is a 4-byte one cut after
    two bytes: IllegalDataException, as RowSeq's walk."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult
    b = datasets.random_batch(43, n_series=4, n_groups=1, span_ms=3600000,
                              value_kind="int", cadence_ms=7000)
    b.ts = b.ts - b.ts % 1000
    b.ts[1::2] += 500  # every other point on milliseconds
    b.is_float = np.zeros(len(b.ts), np.uint8)
    enc = cells.encode_batch(b)
    # row 0: append the first half of a 4-byte qualifier
    qo, q = enc["qual_off"].copy(), enc["qual"]
    z = int(qo[1])
    enc["qual"] = np.concatenate([q[:z], np.array([0xF0, 0x00], np.uint8), q[z:]])
    qo[1:] += 2
    enc["qual_off"] = qo
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
         for k, v in enc.items()}
    dc = workload.DeviceCells(d, b.n_series)
    db = _device_batch(b, "int")
    spec = core.make_spec(datasets.T0, datasets.T0 + 3600000,
                          core.Aggregators.SUM,
                          core.DownsamplingSpecification("1m-avg"))
    res = DeviceResult(torch, db.n_groups, 4096, "cuda")
    with pytest.raises(core.IllegalDataException):
        workload.run_cells_device(engine, spec, dc, db, res)


# (name, value kind, int range, float4 fraction, ms fraction, what the
# kernel choice must be): the uniform cells fold (every kept series one value
# length / type and one qualifier width, k_cells_uniform) for every value
# width and both qualifier widths; batches with a series of mixed lengths
# (the general kernel), and with a series whose rows add up although a point
# is an 8-byte long among 8-byte doubles (the uniform kernel misses on its
# flags and the engine re-runs the general one)
UNIFORM_CASES = [("f8", "float", None, 0.0, 0.0, "uniform"),
                 ("f4", "float", None, 1.0, 0.0, "uniform"),
                 ("i1", "int", (-120, 120), 0, 0, "uniform"),
                 ("i2", "int", (300, 30000), 0, 0, "uniform"),
                 ("i4", "int", (1 << 20, 1 << 30), 0, 0, "uniform"),
                 ("i8", "int", (1 << 40, 1 << 50), 0, 0, "uniform"),
                 ("f8ms", "float", None, 0.0, 1.0, "uniform"),
                 ("i2ms", "int", (300, 30000), 0, 1.0, "uniform"),
                 ("imix", "int", (-(1 << 40), 1 << 40), 0, 0, "general"),
                 ("f8i8", "float", None, 0.0, 0.0, "miss")]


@pytest.mark.parametrize("name,kind,rng_i,f4,ms,path", UNIFORM_CASES,
                         ids=[c[0] for c in UNIFORM_CASES])
@pytest.mark.parametrize("agg,ds,span", [("sum", "1m-avg", 3), ("dev", "5m-sum", 3),
                                         ("zimsum", "1m-max", 40)])
def test_fused_cells_uniform_kernel(engine, name, kind, rng_i, f4, ms, path,
                                    agg, ds, span):
    """The cells fold's uniform kernel (fold_member_cells_u) against the
    oracle on the points RowSeq decodes, and which kernel ran
    (otsdb_ctx_counters): uniform for uniform series (one and several fold
    windows: 40 h of 1 m buckets), the general kernel for a batch with a
    mixed-length series, and a re-run with the general kernel when a row's
    lengths add up but a qualifier's flags differ."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.batch import HostBatch
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_parity import cancel_floor, compare
    rng = np.random.default_rng(23)
    b = datasets.random_batch(19, n_series=24, n_groups=3, value_kind=kind,
                              span_ms=span * 3600000,
                              cadence_ms=7000 if ms else 10000)
    if ms:
        b.ts = b.ts + rng.integers(0, 999, len(b.ts))
        for s in range(b.n_series):
            a, z = b.offsets[s], b.offsets[s + 1]
            b.ts[a:z] = np.sort(b.ts[a:z])
    else:
        b.ts = b.ts - b.ts % 1000
    if rng_i is not None:
        b.val = rng.integers(rng_i[0], rng_i[1], len(b.ts)).astype(np.int64)
        b.is_float = np.zeros(len(b.ts), np.uint8)
    else:
        b.is_float = np.ones(len(b.ts), np.uint8)
    if name == "f8i8":  # series 5: every 7th point an 8-byte long
        a, z = b.offsets[5], b.offsets[6]
        assert z - a > 50
        sel = np.arange(a, z, 7)
        b.val[sel] = (1 << 40) + sel
        b.is_float[sel] = 0
    enc = cells.encode_batch(b, rng, f4, ms)
    ts, bits, isint = [], [], []
    for s in range(b.n_series):
        for r in np.nonzero(enc["row_series"] == s)[0]:
            q = enc["qual"][enc["qual_off"][r]:enc["qual_off"][r + 1]]
            v = enc["val"][enc["val_off"][r]:enc["val_off"][r + 1]]
            p = pyoracle.decode_row(q.tobytes(), v.tobytes(),
                                    enc["row_base_s"][r])
            ts.append(p["ts"])
            bits.append(p["bits"])
            isint.append(p["is_int"])
    rts = np.concatenate(ts).astype(np.int64)
    rbits = np.concatenate(bits).astype(np.int64)
    risf = (np.concatenate(isint).astype(np.uint8) == 0).astype(np.uint8)
    hb = HostBatch(b.offsets, rts, rbits, risf, None, b.group_offsets,
                   b.group_members)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
         for k, v in enc.items()}
    dc = workload.DeviceCells(d, b.n_series)
    db = _device_batch(hb, "float" if kind == "float" else "int")
    t0 = datasets.T0 + 600000
    t1 = datasets.T0 + span * 3600000 - 300000
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification(ds), t0, t1)
    ref = pyoracle.group_by(spec, hb)
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    c0 = engine.counters()
    workload.run_cells_device(engine, spec, dc, db, res)
    c1 = engine.counters()
    du = c1["cells_uniform"] - c0["cells_uniform"]
    dg = c1["cells_general"] - c0["cells_general"]
    dm = c1["cells_uniform_miss"] - c0["cells_uniform_miss"]
    assert (du, dg, dm) == {"uniform": (1, 0, 0), "general": (0, 1, 0),
                            "miss": (1, 1, 1)}[path], (du, dg, dm)
    got = _result_points(res, db.n_groups)
    fl = cancel_floor(hb, 60) if kind == "int" else 0.0
    compare(got, ref, agg == "zimsum" and kind == "int", floor=fl,
            where="uniform/%s/%s/%s" % (name, agg, ds))
