"""One context, many calls (Needs an MI355X).

The engine keeps state between calls to save launches on small queries
(round 5): the device error word is zeroed by the one-pass compaction at the
end of a successful pipeline and the next call skips its memset; look-back
granules and ticket slots are retired by a per-call epoch instead of a
memset; emit flags are only zeroed when a group has no member.  These
tests interleave failing and succeeding queries, host and device entries,
empty groups and short result buffers on ONE context, and compare every
successful call with the oracle (a stale error bit, a stale granule or a
stale emit flag would show up as a wrong status or wrong points)."""
import ctypes as C

import numpy as np
import pytest

from opentsdb_amd import abi, core
from opentsdb_amd.batch import HostBatch, groups_from_ids
from oracle import pyoracle
from tests import datasets
from tests.test_gpu_parity import _spec, compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def _device(hb):
    from opentsdb_amd import dist as odist
    return odist.to_device(hb)


def _run_device(engine, spec, db, cap=None):
    import torch
    from opentsdb_amd.engine import DataPoints, DeviceResult, run_device
    sz = engine.plan(spec, db)
    res = DeviceResult(torch, db.n_groups,
                       int(sz.max_out_points) if cap is None else cap, "cuda")
    run_device(engine, spec, db, res)
    torch.cuda.synchronize()
    offs = res.offsets.cpu().numpy()
    ts, val, ii = (res.ts.cpu().numpy(), res.val.cpu().numpy(),
                   res.is_int.cpu().numpy())
    return [DataPoints(ts[offs[g]:offs[g + 1]], val[offs[g]:offs[g + 1]],
                       ii[offs[g]:offs[g + 1]]) for g in range(db.n_groups)]


def test_failures_between_good_calls(engine):
    """good, IllegalData (`none` over two spans), good, Infinity, good, with
    host and device entries alternating: every failure raises, every good
    call equals the oracle."""
    good = datasets.random_batch(301, n_series=30, n_groups=5)
    bad_none = datasets.random_batch(81, n_series=6, n_groups=2,
                                     outside=False, empty_frac=0)
    big = 1.5e308
    bad_inf = HostBatch.from_groups(
        [[[(datasets.T0 + 1000 * i, big, 1) for i in range(5)]] * 3])
    s_good = _spec("sum", "avg")
    s_none = _spec("none", "avg")
    s_inf = _spec("sum", "max", end=datasets.T0 + 60000)
    ref = pyoracle.group_by(s_good, good)
    dgood = _device(good)
    for k in range(3):
        for entry in ("host", "device"):
            run = (engine.run if entry == "host" else
                   (lambda s, b: _run_device(engine, s, _device(b))))
            compare(run(s_good, good), ref, False, where="good%d%s" % (k, entry))
            with pytest.raises(core.IllegalDataException):
                run(s_none, bad_none)
            compare(_run_device(engine, s_good, dgood), ref, False,
                    where="after-none%d%s" % (k, entry))
            with pytest.raises(core.IllegalStateException):
                run(s_inf, bad_inf)
            compare(engine.run(s_good, good), ref, False,
                    where="after-inf%d%s" % (k, entry))


def test_empty_groups_and_changing_shapes(engine):
    """Groups with no member between others (their emit rows are the only
    ones the engine zeroes), then batches of other group counts and grids on
    the same context: the look-back granules of the earlier, larger calls
    must not leak into the later ones."""
    hb = datasets.random_batch(303, n_series=40, n_groups=8)
    gid = np.asarray([g if g not in (2, 5) else 7 for g in
                      np.arange(40) % 8])          # groups 2 and 5 empty
    hb.group_offsets, hb.group_members = groups_from_ids(gid, 9)  # 8 empty too
    for interval, agg in (("1m", "sum"), ("30s", "max"), ("5m", "avg"),
                          ("1h", "count"), ("1m", "sum")):
        spec = _spec(agg, "avg", interval=interval)
        ref = pyoracle.group_by(spec, hb)
        got = _run_device(engine, spec, _device(hb))
        assert [len(g.ts) for g in got][2] == 0 == len(ref[2])
        # (avg buckets reduce in a lane tree: only counts are bit-exact)
        compare(got, ref, agg == "count", where="empty/%s" % interval)
        small = datasets.random_batch(304, n_series=7, n_groups=2)
        compare(_run_device(engine, spec, _device(small)),
                pyoracle.group_by(spec, small), agg == "count",
                where="small/%s" % interval)


def test_one_and_two_pass_compactions_alternate(engine):
    """Grids of up to 2,048 buckets compact in one pass (k_compact1, ticket
    slots rotating with the call epoch), longer ones in two launches
    (k_compact_count / k_compact_scatter): alternating them on one context
    must leave every ticket slot clean for the next one-pass call."""
    hb = datasets.random_batch(307, n_series=30, n_groups=5)
    db = _device(hb)
    for k in range(6):
        for interval in ("1m", "1s", "1s", "30s", "1m"):   # 180 / 10,800 / 360
            spec = _spec("count", "count", interval=interval)
            compare(_run_device(engine, spec, db),
                    pyoracle.group_by(spec, hb), True,
                    where="alt%d/%s" % (k, interval))


def test_long_grid_dense_and_sparse_groups(engine):
    """Grids past 2,048 buckets compact in three launches; a group whose
    every bucket is emitted (FillingDownsampler) takes the scatter's straight
    copy, the others the flag-driven one; is_int is zeroed over each group's
    range by wide stores.  Host and device entries, and a device result one
    point short of the total."""
    hb = datasets.random_batch(308, n_series=24, n_groups=4)
    end = datasets.T0 + 8 * 3600 * 1000
    for fill in ("zero", "none"):
        spec = _spec("sum", "sum", fill=fill, interval="10s", end=end)
        ref = pyoracle.group_by(spec, hb)
        compare(engine.run(spec, hb), ref, False, where="host/" + fill)
        got = _run_device(engine, spec, _device(hb))
        compare(got, ref, False, where="device/" + fill)
        for g in got:
            assert not np.any(g.is_int)
        total = sum(len(g) for g in ref)
        with pytest.raises(core.OpenTSDBException):
            _run_device(engine, spec, _device(hb), cap=total - 1)


def test_short_result_then_good(engine):
    """A device result too small (E_CAPACITY: nothing written past it, the
    error word and look-back state left consistent), then the same query with
    room."""
    hb = datasets.random_batch(305, n_series=25, n_groups=5)
    spec = _spec("sum", "avg")
    ref = pyoracle.group_by(spec, hb)
    db = _device(hb)
    with pytest.raises(core.OpenTSDBException):
        _run_device(engine, spec, db, cap=3)
    compare(_run_device(engine, spec, db), ref, False, where="after-short")


def test_host_group_offsets_match_readback(engine):
    """otsdb_batch.group_offsets_host (ABI 4) is only a copy: the same query
    with it and without it (the engine reads the offsets back) gives the
    same bits."""
    import torch
    from opentsdb_amd.engine import DeviceResult
    hb = datasets.random_batch(306, n_series=50, n_groups=6)
    db = _device(hb)
    spec = _spec("avg", "avg")
    out = []
    for host_copy in (True, False):
        b = db.as_abi()
        if not host_copy:
            b.group_offsets_host = None
        sz = engine.plan(spec, db)
        res = DeviceResult(torch, db.n_groups, int(sz.max_out_points), "cuda")
        r = res.as_abi()
        engine._check(engine.lib.otsdb_agg_run_device(
            engine.ctx, C.byref(spec), C.byref(b), C.byref(r), None))
        torch.cuda.synchronize()
        n = int(res.offsets[-1].item())
        out.append((res.offsets.cpu().numpy(), res.ts[:n].cpu().numpy(),
                    res.val[:n].cpu().numpy()))
    for a, z in zip(out[0], out[1]):
        assert np.array_equal(a, z)


def test_compaction_epoch_wrap():
    """The one-pass compaction takes a look-back granule as this call's by
    its epoch alone.  On a fresh context, three small calls (epochs 1-3),
    then a 1,000-group call leaves granules of epoch 4; the epoch is moved
    on to 2^24 - 4, three small calls, and the next call wraps to epoch 4
    again — a 1,000-group call over other data, whose look-back must not
    read the first one's granules (other counts) as published: the engine
    clears every granule at the wrap (the advisor's round-5 finding).  Every
    call is compared with the oracle; the hook refuses to move back."""
    from opentsdb_amd.engine import Engine
    engine = Engine(0)
    try:
        big = datasets.random_batch(311, n_series=1000, n_groups=1000,
                                    span_ms=3600 * 1000)
        big2 = datasets.random_batch(313, n_series=1000, n_groups=1000,
                                     span_ms=3600 * 1000)
        small = datasets.random_batch(312, n_series=12, n_groups=5)
        spec = _spec("count", "count")
        ref_small = pyoracle.group_by(spec, small)
        dsmall = _device(small)
        for k in range(3):   # epochs 1, 2, 3
            compare(_run_device(engine, spec, dsmall), ref_small, True,
                    where="small%d" % k)
        compare(_run_device(engine, spec, _device(big)),
                pyoracle.group_by(spec, big), True, where="big@4")
        lib = engine.lib
        assert lib.otsdb_test_set_compact_epoch(engine.ctx, 3) != 0  # back
        # (forward by whole rotations of the 4 ticket slots)
        assert lib.otsdb_test_set_compact_epoch(engine.ctx, (1 << 24) - 3) != 0
        assert lib.otsdb_test_set_compact_epoch(engine.ctx, (1 << 24) - 4) == 0
        for k in range(3):   # epochs 2^24-3, 2^24-2, 2^24-1
            compare(_run_device(engine, spec, dsmall), ref_small, True,
                    where="small-wrap%d" % k)
        compare(_run_device(engine, spec, _device(big2)),   # wraps to 4
                pyoracle.group_by(spec, big2), True, where="big2@4")
        compare(_run_device(engine, spec, dsmall), ref_small, True,
                where="small@5")
    finally:
        engine.close()
