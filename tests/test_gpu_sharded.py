"""Series-sharded (multi-GPU) path on the one GPU of the test box.

The cross-rank protocols are exercised exactly as ranks run them, with the
collectives done in-process: each emulated rank has its own context, its
shard of the series (contiguous SpanCmp range, dist.shard_host_batch) and
group offsets over every global group.  Then two real processes run
dist.run_sharded_any over gloo (both on cuda:0) — the code path bench.py and
a node launch take, with RCCL swapped for gloo.  Reference: the oracle over
the unsharded batch.
"""
import os
import socket

import numpy as np
import pytest

from opentsdb_amd import core, dist as odist
from opentsdb_amd.engine import DataPoints, Engine
from oracle import pyoracle
from tests import datasets
from tests.test_gpu_parity import ORDER_FREE, compare, _spec

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engines():
    from opentsdb_amd import build
    build.build()
    es = [Engine(0) for _ in range(3)]
    yield es
    for e in es:
        e.close()


def _host(res, G):
    offs = res.offsets.cpu().numpy()
    ts, val, ii = (res.ts.cpu().numpy(), res.val.cpu().numpy(),
                   res.is_int.cpu().numpy())
    return [DataPoints(ts[offs[g]:offs[g + 1]], val[offs[g]:offs[g + 1]],
                       ii[offs[g]:offs[g + 1]]) for g in range(G)]


def _partials_emulated(engines, spec, hb, world):
    import ctypes as C
    import torch
    from opentsdb_amd.engine import DeviceResult
    G = hb.n_groups
    parts, emits, nb = [], [], None
    for r in range(world):
        e = engines[0]
        db = odist.to_device(odist.shard_host_batch(hb, world, r))
        nb = int(e.plan(spec, db).n_buckets)
        GB = G * nb
        p = torch.zeros((max(GB, 1), 4), dtype=torch.int64, device="cuda")
        m = torch.zeros(max(GB, 1), dtype=torch.uint8, device="cuda")
        b = db.as_abi()
        e._check(e.lib.otsdb_agg_partials_device(
            e.ctx, C.byref(spec), C.byref(b), p.data_ptr(), m.data_ptr(), None))
        parts.append(p[:GB])
        emits.append(m[:GB])
    gp = torch.stack(parts).contiguous()
    ge = torch.stack(emits).contiguous()
    res = DeviceResult(torch, G, max(G * nb, 1), "cuda")
    r = res.as_abi()
    e = engines[0]
    e._check(e.lib.otsdb_agg_finalize_device(
        e.ctx, C.byref(spec), G, nb, world, gp.data_ptr(), ge.data_ptr(),
        C.byref(r), None))
    torch.cuda.synchronize()
    return _host(res, G)


def _select_emulated(engines, spec, hb, world, stats=None):
    """The otsdb_sel_* protocol with the collectives emulated in-process
    (one context per rank)."""
    import torch
    G = hb.n_groups
    sels = [odist.ShardedSelect(engines[r], spec,
                                odist.to_device(odist.shard_host_batch(hb, world, r)),
                                G) for r in range(world)]
    cs, es, ks = zip(*[s.prepare() for s in sels])
    counts = torch.stack(cs).sum(0)
    emit = torch.stack(es).max(0).values
    krange = torch.stack(ks).min(0).values
    for s in sels:
        s.counts.copy_(counts)
        s.emit.copy_(emit)
        s.krange.copy_(krange)
    p = 0
    while True:
        more = [s.hist_pass(p) for s in sels]
        assert len(set(more)) == 1, "ranks planned different passes"
        if not more[0]:
            break
        h = torch.stack([s.hist for s in sels]).sum(0)
        for s in sels:
            s.hist.copy_(h.to(torch.int32))
        p += 1
        assert p <= odist.MAX_SEL_PASSES
    picks = torch.stack([s.pick().clone() for s in sels]).sum(0)
    for s in sels:
        s.picks.copy_(picks)
    outs = [_host(s.finish(), G) for s in sels]
    for o in outs[1:]:  # every rank ends with the same result
        for a, b in zip(outs[0], o):
            assert np.array_equal(a.ts, b.ts) and np.array_equal(a.bits, b.bits)
    if stats is not None:
        for e in engines[:world]:
            c = e.counters()
            stats.append((c["sel_key_reads"], c["sel_passes"]))
    return outs[0]


AGGS = ["sum", "zimsum", "avg", "dev", "min", "max", "mimmin", "mimmax",
        "count", "first", "last", "diff", "mult", "squareSum", "pfsum"]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("agg", AGGS)
def test_partials_across_ranks(engines, agg, world):
    """Per-(group, bucket) partials merged in rank (= series) order:
    order-free aggregators bit-exact, sums within 1e-12."""
    hb = datasets.random_batch(201, n_series=40, n_groups=3, nan_frac=0.02)
    for ds, fill in (("avg", "none"), ("max", "nan"), ("sum", "zero")):
        spec = _spec(agg, ds, fill)
        ref = pyoracle.group_by(spec, hb)
        got = _partials_emulated(engines, spec, hb, world)
        # downsample avg/sum reduce buckets in a wave tree (1e-12)
        compare(got, ref, agg in ORDER_FREE and ds == "max",
                where="w%d/%s/%s/%s" % (world, agg, ds, fill))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("agg", ["median", "p50", "p90", "p99", "p999",
                                 "ep95r3", "ep50r7"])
def test_percentiles_across_ranks(engines, agg, world):
    """The otsdb_sel_* protocol: exact selection with all-reduced counts and
    histograms — bit-identical to the single-GPU oracle result."""
    hb = datasets.random_batch(203, n_series=90, n_groups=2, nan_frac=0.05,
                               span_ms=3600 * 1000, cadence_ms=20000)
    for ds, fill in (("avg", "none"), ("max", "nan")):
        spec = _spec(agg, ds, fill, end=datasets.T0 + 3600 * 1000)
        ref = pyoracle.group_by(spec, hb)
        got = _select_emulated(engines, spec, hb, world)
        compare(got, ref, ds == "max",
                where="w%d/%s/%s" % (world, agg, fill))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("agg", ["p99", "median", "ep95r3"])
def test_percentiles_across_ranks_fills_rate_calendar(engines, agg, world):
    """The protocol under the other paths into the key matrix: fill zero /
    null (the transpose applies the fill and counts the keys), counter rates
    (the rate-fused bucketize rows), `all`, and a calendar grid."""
    import copy
    from opentsdb_amd import core as ocore, jcalendar
    hb = datasets.random_batch(211, n_series=70, n_groups=2, nan_frac=0.03,
                               span_ms=3 * 3600 * 1000, cadence_ms=20000)
    cases = [("sum", "zero", False, "1m"), ("avg", "null", False, "1m"),
             ("max", "none", False, "30m"), ("avg", "none", False, "0all")]
    for ds, fill, rate, iv in cases:
        spec = _spec(agg, ds, fill, rate=rate, interval=iv)
        ref = pyoracle.group_by(spec, hb)
        got = _select_emulated(engines, spec, hb, world)
        compare(got, ref, ds == "max", where="w%d/%s/%s-%s-%s" % (
            world, agg, iv, ds, fill))
    hc = datasets.random_batch(213, n_series=60, n_groups=2, counter=True,
                               span_ms=3 * 3600 * 1000, cadence_ms=20000)
    ro = ocore.RateOptions(True, 2**63 - 1, 0)
    spec = _spec(agg, "sum", "none", rate=True, ro=ro)
    ref = pyoracle.group_by(spec, hc)
    got = _select_emulated(engines, spec, hc, world)
    compare(got, ref, False, where="w%d/%s/rate" % (world, agg))


def _edge_values(kind, rng, m):
    """Bucket values that stress the cross-rank selection's planning."""
    if kind == "ties":  # one distinct key: resolved from the key range alone
        return np.full(m, 42.0)
    if kind == "clustered":  # the offset digit puts ~all keys in one bin
        v = 1.0 + rng.random(m) * 1e-12
        v[rng.random(m) < 0.005] = 1e6
        return v
    if kind == "signed":  # both signs, +-0.0, subnormals, wide exponents
        v = rng.standard_normal(m) * 10.0 ** rng.integers(-300, 300, m)
        z = rng.random(m)
        v[z < 0.05] = 0.0
        v[(z >= 0.05) & (z < 0.1)] = -0.0
        v[(z >= 0.1) & (z < 0.12)] = 5e-324
        return v
    if kind == "dups":  # few distinct values: bins of many equal keys
        return rng.integers(0, 5, m).astype(np.float64) * 0.25
    raise ValueError(kind)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind", ["ties", "clustered", "signed", "dups"])
def test_selection_protocol_edges(engines, kind, world):
    """The otsdb_sel_* planning on adversarial keys: bit-identical to the
    oracle, every rank planning the same passes, at most two passes over a
    rank's local keys (otsdb_ctx_counters) and MAX_SEL_PASSES histogram
    passes."""
    hb = datasets.random_batch(207, n_series=160, n_groups=2, nan_frac=0.0,
                               span_ms=3600 * 1000, cadence_ms=20000)
    rng = np.random.default_rng(11)
    hb.val = np.ascontiguousarray(
        _edge_values(kind, rng, len(hb.val)).view(np.int64))
    hb.is_float = np.ones(len(hb.val), np.uint8)
    for agg in ("p99", "median", "ep50r7", "p999"):
        spec = _spec(agg, "max", "none", end=datasets.T0 + 3600 * 1000)
        ref = pyoracle.group_by(spec, hb)
        stats = []
        got = _select_emulated(engines, spec, hb, world, stats)
        compare(got, ref, True, where="w%d/%s/%s" % (world, kind, agg))
        for reads, passes in stats:
            assert reads <= 2 and passes <= odist.MAX_SEL_PASSES, (
                kind, agg, reads, passes)
        if kind == "ties":
            assert all(r == 0 and p == 0 for r, p in stats), stats


@pytest.mark.parametrize("agg", ["p99", "median"])
def test_selection_with_an_empty_rank(engines, agg):
    """Three ranks over two series: one rank holds no series at all (empty
    key matrix, every segment's local range empty) and still plans the same
    passes and ends with the full result."""
    hb = datasets.random_batch(209, n_series=2, n_groups=1, nan_frac=0.0,
                               empty_frac=0.0, span_ms=3600 * 1000,
                               cadence_ms=20000)
    spec = _spec(agg, "avg", "none", end=datasets.T0 + 3600 * 1000)
    ref = pyoracle.group_by(spec, hb)
    got = _select_emulated(engines, spec, hb, 3)
    compare(got, ref, False, where="empty-rank/%s" % agg)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


QUERIES = [("sum", "avg", "none"), ("dev", "max", "nan"), ("p99", "avg", "nan"),
           ("median", "max", "none"),
           # raw (non-downsampled) group-by: shared groups run as replicas
           ("sum", None, None), ("max", None, None)]


def _qspec(agg, ds, fill):
    if ds is None:
        t0, t1 = datasets.T0, datasets.T0 + 3 * 3600 * 1000
        return core.make_spec(t0, t1, core.Aggregators.get(agg), None, t0, t1)
    return _spec(agg, ds, fill)


def _rank_main(rank, world, port, q):
    import torch
    import torch.distributed as tdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    e = Engine(0)
    hb = datasets.random_batch(205, n_series=50, n_groups=3, nan_frac=0.02)
    out = []
    for agg, ds, fill in QUERIES:
        spec = _qspec(agg, ds, fill)
        db = odist.to_device(odist.shard_host_batch(hb, world, rank))
        res = odist.run_sharded_any(e, spec, db, hb.n_groups)
        torch.cuda.synchronize()
        # each rank holds its own groups and the shared ones
        out.append({g: tuple(a.copy() for a in v)
                    for g, v in res.host_groups().items()})
    q.put((rank, out))
    tdist.barrier()
    tdist.destroy_process_group()
    e.close()


def test_two_processes_gloo():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, q))
          for r in range(world)]
    for p in ps:
        p.start()
    import queue
    import time
    outs = []
    deadline = time.time() + 240
    while len(outs) < world:  # stop early if a rank died
        assert time.time() < deadline, "ranks did not report"
        try:
            outs.append(q.get(timeout=5))
        except queue.Empty:
            assert all(p.is_alive() or p.exitcode == 0 for p in ps), \
                [p.exitcode for p in ps]
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    hb = datasets.random_batch(205, n_series=50, n_groups=3, nan_frac=0.02)
    for k, (agg, ds, fill) in enumerate(QUERIES):
        ref = pyoracle.group_by(_qspec(agg, ds, fill), hb)
        merged = {}
        for _, out in outs:
            merged.update(out[k])
        assert sorted(merged) == list(range(hb.n_groups))
        got = [DataPoints(*merged[g]) for g in range(hb.n_groups)]
        # raw: the replica runs the whole group in span order (exact); dev:
        # the ranks hand one chain on (dist.hand_on_partials, exact)
        compare(got, ref, (ds == "max" and agg != "sum") or ds is None,
                where="gloo/%s/%s" % (agg, ds))


def _rccl_main(port, q):
    """World size 1 over RCCL: the device-tensor collectives of the sharded
    path (classify_groups' MIN all-reduce, the partial all-gather, the
    selection protocol's count / histogram all-reduces) run through
    ProcessGroupNCCL = RCCL, exactly as bench.py's node launch calls them."""
    import torch
    import torch.distributed as tdist
    torch.cuda.set_device(0)
    tdist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port,
                             rank=0, world_size=1,
                             device_id=torch.device("cuda", 0))
    assert tdist.get_backend() == "nccl"
    e = Engine(0)
    hb = datasets.random_batch(207, n_series=50, n_groups=3, nan_frac=0.02)
    out = []
    for agg, ds, fill in QUERIES:
        spec = _qspec(agg, ds, fill)
        db = odist.to_device(hb)
        # rank-local groups (classification all-reduce on device)
        res = odist.run_sharded_any(e, spec, db, hb.n_groups)
        torch.cuda.synchronize()
        local = {g: tuple(a.copy() for a in v)
                 for g, v in res.host_groups().items()}
        # every group through the shared-group exchange: partials
        # all-gathered over RCCL, merged by otsdb_agg_finalize_device
        shared = None
        if agg not in ("p99", "median"):
            real = odist.classify_groups
            odist.classify_groups = lambda goff, group=None, device=None: (
                np.zeros(0, np.int64), np.nonzero(np.diff(goff) > 0)[0])
            try:
                db2 = odist.to_device(hb)
                # partial exchange, or (raw) the replica gather
                r2 = odist.run_sharded_any(e, spec, db2, hb.n_groups)
            finally:
                odist.classify_groups = real
            torch.cuda.synchronize()
            assert len(r2.shared_ids) == hb.n_groups
            shared = {g: tuple(a.copy() for a in v)
                      for g, v in r2.host_groups().items()}
        out.append((local, shared))
    tdist.barrier()
    tdist.destroy_process_group()
    e.close()
    q.put(out)


def test_rccl_world_size_one():
    import queue
    import time
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_main, args=(_free_port(), q))
    p.start()
    deadline = time.time() + 100
    out = None
    while out is None:
        assert time.time() < deadline, "the RCCL rank did not report"
        try:
            out = q.get(timeout=5)
        except queue.Empty:
            assert p.is_alive() or p.exitcode == 0, p.exitcode
    p.join(timeout=60)
    assert p.exitcode == 0
    hb = datasets.random_batch(207, n_series=50, n_groups=3, nan_frac=0.02)
    for (agg, ds, fill), (local, shared) in zip(QUERIES, out):
        ref = pyoracle.group_by(_qspec(agg, ds, fill), hb)
        exact = (ds == "max" and agg != "sum") or ds is None
        for name, res in (("local", local), ("shared", shared)):
            if res is None:
                continue
            assert sorted(res) == list(range(hb.n_groups))
            got = [DataPoints(*res[g]) for g in range(hb.n_groups)]
            compare(got, ref, exact, where="rccl/%s/%s" % (name, agg))
