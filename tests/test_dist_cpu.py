"""Multi-rank path on CPU (gloo, world size 2): sharding, cross-rank group
detection and the partial exchange protocol (all-gather, rank-major layout,
merge in rank = series order)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from opentsdb_amd import dist as odist
from opentsdb_amd import workload


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_ranges_cover_series_in_order():
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            rs = [odist.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c and a <= b
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


def test_shared_groups_by_config():
    n = 1000
    host = workload.group_ids("C2", 0, n)
    assert len(odist.shared_groups(host, 2)) == 0      # {host=*}: rank-local
    assert len(odist.shared_groups(host, 8)) <= 7      # at most one per cut
    dc = workload.group_ids("C3", 0, n)
    assert len(odist.shared_groups(dc, 2)) == 16       # {dc=*}: spans ranks
    one = workload.group_ids("C5", 0, n)
    assert list(odist.shared_groups(one, 4)) == [0]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(100 + rank)
    GB = 37
    s = rng.random(GB) * 10
    n = rng.integers(0, 5, GB)
    parts = np.zeros((GB, 4), np.int64)
    parts[:, 0] = s.view(np.int64)
    parts[:, 3] = n
    emit = (n > 0).astype(np.uint8)
    gp, ge = odist.all_gather_partials(torch.from_numpy(parts),
                                       torch.from_numpy(emit))
    if rank == 0:
        q.put((gp.numpy(), ge.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_partial_exchange_gloo_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q))
          for r in range(world)]
    for p in ps:
        p.start()
    gp, ge = q.get(timeout=120)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert gp.shape == (2, 37, 4) and ge.shape == (2, 37)
    # rank-major: slice r is exactly what rank r contributed
    for r in range(world):
        rng = np.random.default_rng(100 + r)
        s = rng.random(37) * 10
        n = rng.integers(0, 5, 37)
        assert np.array_equal(gp[r, :, 0].view(np.float64), s)
        assert np.array_equal(gp[r, :, 3], n)
        assert np.array_equal(ge[r], (n > 0).astype(np.uint8))
    s, n = odist.merge_partials_reference(gp)
    exp_s = gp[0, :, 0].view(np.float64) + gp[1, :, 0].view(np.float64)
    assert np.array_equal(s, exp_s)


def test_shard_host_batch_partitions_series_and_groups():
    """Each rank's shard keeps its contiguous series range, its points, and
    group offsets over every global group; together the shards rebuild the
    batch (members in SpanCmp order)."""
    from tests import datasets
    hb = datasets.random_batch(7, n_series=23, n_groups=4)
    for world in (1, 2, 3, 5):
        members = [[] for _ in range(hb.n_groups)]
        pts = []
        for r in range(world):
            sh = odist.shard_host_batch(hb, world, r)
            a, b = odist.shard_range(hb.n_series, world, r, hb.offsets)
            assert sh.n_series == b - a and sh.n_groups == hb.n_groups
            assert sh.offsets[0] == 0
            pts.append(sh.ts)
            for g in range(hb.n_groups):
                loc = sh.group_members[sh.group_offsets[g]:sh.group_offsets[g + 1]]
                members[g].extend((loc + a).tolist())
        assert np.array_equal(np.concatenate(pts), hb.ts)
        for g in range(hb.n_groups):
            exp = hb.group_members[hb.group_offsets[g]:hb.group_offsets[g + 1]]
            assert members[g] == exp.tolist()


def test_shard_range_balances_points():
    """Point-balanced contiguous shards: every rank's share of
    the points is within one series of total / world, and the ranges tile
    the series."""
    rng = np.random.default_rng(3)
    counts = rng.integers(0, 5000, 997)
    counts[:50] = 40000  # heavy series at the front
    off = np.concatenate([[0], np.cumsum(counts)])
    for world in (1, 2, 3, 8):
        cuts = [odist.shard_range(len(counts), world, r, off)
                for r in range(world)]
        assert cuts[0][0] == 0 and cuts[-1][1] == len(counts)
        for (a0, b0), (a1, b1) in zip(cuts, cuts[1:]):
            assert b0 == a1
        share = off[-1] / world
        for a, b in cuts:
            assert abs((off[b] - off[a]) - share) <= counts.max()


def _classify_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # 6 groups over 2 ranks: 0,1 only on rank 0; 2 on both; 3 only on rank 1;
    # 4 on both; 5 on nobody
    counts = {0: [3, 2, 1, 0, 4, 0], 1: [0, 0, 2, 5, 1, 0]}[rank]
    goff = np.concatenate([[0], np.cumsum(counts)])
    local, shared = odist.classify_groups(goff)
    q.put((rank, local.tolist(), shared.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_classify_groups_gloo_world2():
    """Only groups with members on several ranks are exchanged; the rest
    finish where they live (no data-path collective for them)."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_classify_worker, args=(r, world, port, q))
          for r in range(world)]
    for p in ps:
        p.start()
    got = dict((r, (l, s)) for r, l, s in (q.get(timeout=120)
                                          for _ in range(world)))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got[0] == ([0, 1], [2, 4])
    assert got[1] == ([3], [2, 4])


def test_bench_spawns_ranks_dry_run():
    """bench.py --gpus 2 outside a torch.distributed launch starts the two
    ranks itself (torch.distributed.run, 127.0.0.1) and relays rank 0's line;
    the dry run exercises the launcher, the process group and the
    max-over-ranks timing without the HIP engine."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"),
                        "--gpus", "2", "--config", "C3", "--steps", "3",
                        "--warmup", "1", "--dry-run"], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["steps"] == 3


def _gather_worker(rank, world, port, q):
    import torch.distributed as dist
    from tests import datasets
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hb = datasets.random_batch(31, n_series=29, n_groups=4, value_kind="mixed")
    db = odist.to_device(odist.shard_host_batch(hb, world, rank), "cpu")
    sb = odist.gather_shared_series(db, np.array([0, 2, 3]))
    q.put((rank, sb.offsets.numpy().copy(), sb.ts.numpy().copy(),
           sb.val.numpy().copy(), sb.is_float.numpy().copy(),
           sb.group_offsets.numpy().copy(), sb.group_members.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_raw_replica_gather_gloo_world2():
    """Raw group-by across ranks runs the shared groups as replicas: every
    rank gathers the same batch of those groups' members, in series
    (SpanCmp) order, points and value types intact."""
    from tests import datasets
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, q))
          for r in range(world)]
    for p in ps:
        p.start()
    got = dict((x[0], x[1:]) for x in (q.get(timeout=120) for _ in range(world)))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    for a, b in zip(got[0], got[1]):
        assert np.array_equal(a, b)  # identical on every rank
    offs, ts, val, isf, goff, mem = got[0]
    hb = datasets.random_batch(31, n_series=29, n_groups=4, value_kind="mixed")
    for k, g in enumerate([0, 2, 3]):
        exp = hb.group_members[hb.group_offsets[g]:hb.group_offsets[g + 1]]
        got_m = mem[goff[k]:goff[k + 1]]
        assert len(got_m) == len(exp)
        for sg, s in zip(got_m, exp):
            a, b = hb.offsets[s], hb.offsets[s + 1]
            assert np.array_equal(ts[offs[sg]:offs[sg + 1]], hb.ts[a:b])
            assert np.array_equal(val[offs[sg]:offs[sg + 1]], hb.val[a:b])
            assert np.array_equal(isf[offs[sg]:offs[sg + 1]], hb.is_float[a:b])


def _welford_push(state, x):
    """StdDev.runDouble's loop body (Aggregators.java:553-560) on an
    (n, mean, M2) state."""
    n, mean, m2 = state
    if n == 0:
        return (1, x, 0.0)
    n += 1
    nm = mean + (x - mean) / n
    return (n, nm, m2 + (x - mean) * (x - nm))


def _hand_on_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    GB = 5
    # this rank's members' values per slot: offset data (~3e9 +- 1e4), where
    # merging per-rank Welford states lands ~1e-11 from one pass
    rng = np.random.default_rng(500 + rank)
    vals = 3.0e9 + rng.random((GB, 40 + 7 * rank)) * 1e4
    parts = torch.zeros((GB, 4), dtype=torch.int64)
    emit = torch.zeros(GB, dtype=torch.uint8)

    def step(init_p, init_e):
        for k in range(GB):
            if init_p is None:
                st = (0, 0.0, 0.0)
            else:
                w = init_p[k].numpy()
                st = (int(w[3]), float(w[0:1].view(np.float64)[0]),
                      float(w[1:2].view(np.float64)[0]))
            for x in vals[k]:
                st = _welford_push(st, float(x))
            parts[k, 0] = int(np.float64(st[1]).view(np.int64))
            parts[k, 1] = int(np.float64(st[2]).view(np.int64))
            parts[k, 3] = st[0]
            emit[k] = 1
    odist.hand_on_partials(step, parts, emit)
    q.put((rank, parts.numpy().copy(), emit.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_hand_on_partials_gloo_world3():
    """The chained exchange of dev states (dist.hand_on_partials): rank r
    continues rank r - 1's Welford states, so every rank ends with exactly
    the state of ONE sequential pass over all ranks' members in rank order —
    bit for bit, where a merge of per-rank states misses it."""
    world = 3
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_hand_on_worker, args=(r, world, port, q))
          for r in range(world)]
    for p in ps:
        p.start()
    got = dict((r, (pp, ee)) for r, pp, ee in (q.get(timeout=120)
                                              for _ in range(world)))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(1, world):  # broadcast: every rank holds the last's states
        assert np.array_equal(got[r][0], got[0][0])
    vals = [3.0e9 + np.random.default_rng(500 + r).random((5, 40 + 7 * r)) * 1e4
            for r in range(world)]
    for k in range(5):
        st = (0, 0.0, 0.0)
        for r in range(world):
            for x in vals[r][k]:
                st = _welford_push(st, float(x))
        w = got[0][0][k]
        assert int(w[3]) == st[0]
        assert w[0] == np.float64(st[1]).view(np.int64)
        assert w[1] == np.float64(st[2]).view(np.int64)
