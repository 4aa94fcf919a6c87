"""Series-sharded multi-GPU execution.

One process per GPU.  Rank r owns a contiguous range of the SpanCmp-ordered
series.  Groups whose members all live on one rank finish on that rank with
no data-path collective.  Groups that span ranks are reduced to 32-byte
per-(group, bucket) partials on every rank (otsdb_agg_partials_device),
all-gathered over RCCL (torch.distributed, backend "nccl"; "gloo" in CPU
tests) and merged in rank order, which is series order, by
otsdb_agg_finalize_device.
"""
import numpy as np

PARTIAL_WORDS = 4  # otsdb_partial = 3 doubles + int64


def shard_range(n_series, world, rank):
    """Contiguous, balanced series range of `rank`."""
    per = n_series // world
    rem = n_series % world
    a = rank * per + min(rank, rem)
    return a, a + per + (1 if rank < rem else 0)


def shared_groups(group_of_series, world):
    """Global group ids whose members span more than one rank (group ids in
    ByteMap order, one per series)."""
    gid = np.asarray(group_of_series, np.int64)
    n = len(gid)
    owner = np.empty(n, np.int64)
    for r in range(world):
        a, b = shard_range(n, world, r)
        owner[a:b] = r
    G = int(gid.max()) + 1 if n else 0
    lo = np.full(G, world, np.int64)
    hi = np.full(G, -1, np.int64)
    np.minimum.at(lo, gid, owner)
    np.maximum.at(hi, gid, owner)
    return np.nonzero((hi > lo) & (hi >= 0))[0]


def all_gather_partials(partials, emit, group=None):
    """partials: [GB, 4] int64 tensor (raw otsdb_partial words), emit: [GB]
    uint8.  Returns rank-major [world, GB, 4] / [world, GB] tensors — the
    layout otsdb_agg_finalize_device merges in rank order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    gp = [torch.empty_like(partials) for _ in range(world)]
    ge = [torch.empty_like(emit) for _ in range(world)]
    dist.all_gather(gp, partials.contiguous(), group=group)
    dist.all_gather(ge, emit.contiguous(), group=group)
    return torch.stack(gp), torch.stack(ge)


def run_sharded(engine, spec, dbatch, n_groups_global, torch_mod=None,
                group=None):
    """Runs one query over a rank's DeviceBatch whose group_offsets span all
    `n_groups_global` groups (empty for groups with no local members).
    Returns (offsets, ts, val, is_int) device tensors of the final result on
    every rank."""
    import ctypes as C
    import torch
    import torch.distributed as dist
    from . import abi
    from .engine import DeviceResult

    sz = engine.plan(spec, dbatch)
    nb = int(sz.n_buckets)
    GB = n_groups_global * nb
    dev = dbatch.ts.device
    parts = torch.zeros((max(GB, 1), PARTIAL_WORDS), dtype=torch.int64,
                        device=dev)
    emit = torch.zeros(max(GB, 1), dtype=torch.uint8, device=dev)
    b = dbatch.as_abi()
    engine._check(engine.lib.otsdb_agg_partials_device(
        engine.ctx, C.byref(spec), C.byref(b), parts.data_ptr(),
        emit.data_ptr(), None))
    torch.cuda.synchronize()
    gp, ge = all_gather_partials(parts[:GB], emit[:GB], group)
    world = dist.get_world_size(group)
    res = DeviceResult(torch, n_groups_global, GB, dev)
    r = res.as_abi()
    engine._check(engine.lib.otsdb_agg_finalize_device(
        engine.ctx, C.byref(spec), n_groups_global, nb, world,
        gp.contiguous().data_ptr(), ge.contiguous().data_ptr(), C.byref(r),
        None))
    return res


def merge_partials_reference(parts_rank_major, kind="sum"):
    """Host restatement of the rank-order merge for a sum-like state
    (x = sum, w = count), used by the CPU tests of the exchange protocol."""
    p = np.asarray(parts_rank_major)
    s = np.zeros(p.shape[1])
    n = np.zeros(p.shape[1], np.int64)
    for r in range(p.shape[0]):
        s = s + p[r, :, 0].view(np.float64)
        n = n + p[r, :, 3]
    return s, n
