"""Series-sharded multi-GPU execution.

One process per GPU.  Rank r owns a contiguous range of the SpanCmp-ordered
series.  Groups whose members all live on one rank finish on that rank with
no data-path collective.  Groups that span ranks are reduced to 32-byte
per-(group, bucket) partials on every rank (otsdb_agg_partials_device),
all-gathered over RCCL (torch.distributed, backend "nccl"; "gloo" in CPU
tests) and merged in rank order, which is series order, by
otsdb_agg_finalize_device.  Median / percentiles across ranks run the
otsdb_sel_* protocol instead: all-reduced contribution counts and key
ranges, then digit passes whose 2,048-bin histograms are all-reduced until
every order statistic is resolved (exact; two passes over the local keys at
most, see select.hip).
Order-sensitive aggregators (`dev`: StdDev.runDouble is one sequential
Welford loop, Aggregators.java:547-568, whose result on offset data depends
on its order at ~1e-11) hand their states on instead of merging them: rank 0
reduces its members, each later rank continues from its predecessor's states
(otsdb_agg_partials_chained_device, point-to-point in rank = series order),
and the last rank's states are broadcast (hand_on_partials).  Raw
(non-downsampled) queries, whose union-timestamp merge needs every member's
points, run the groups spanning ranks as replicas over all-gathered member
series (gather_shared_series).
"""
import numpy as np

from . import abi

PARTIAL_WORDS = 4  # otsdb_partial = 3 doubles + int64
# aggregators whose partial states are handed on across ranks, not merged
# (monoids.h kOrdered)
ORDERED_AGGS = ("dev",)
# groups up to this many members (over all ranks) are handed on as one
# chain (the engine's kOrderedChunk); larger ones merge per-rank partials
CHAIN_MAX_MEMBERS = 65536


def shard_range(n_series, world, rank, offsets=None):
    """Contiguous series range [a, b) of `rank`.  With the batch's point
    offsets (CSR, S+1) the ranges are balanced by POINT count:
    rank r starts at the first series whose first point is at or past
    r/world of the points; otherwise by series count."""
    if offsets is not None and n_series > 0:
        off = np.asarray(offsets, np.int64)
        total = int(off[-1])

        def cut(r):
            if r <= 0:
                return 0
            if r >= world:
                return n_series
            return int(np.searchsorted(off[:-1], (total * r + world - 1) // world,
                                       side="left"))
        return cut(rank), max(cut(rank), cut(rank + 1))
    per = n_series // world
    rem = n_series % world
    a = rank * per + min(rank, rem)
    return a, a + per + (1 if rank < rem else 0)


def shared_groups(group_of_series, world, offsets=None):
    """Global group ids whose members span more than one rank (group ids in
    ByteMap order, one per series; shards as shard_range cuts them)."""
    gid = np.asarray(group_of_series, np.int64)
    n = len(gid)
    owner = np.empty(n, np.int64)
    for r in range(world):
        a, b = shard_range(n, world, r, offsets)
        owner[a:b] = r
    G = int(gid.max()) + 1 if n else 0
    lo = np.full(G, world, np.int64)
    hi = np.full(G, -1, np.int64)
    np.minimum.at(lo, gid, owner)
    np.maximum.at(hi, gid, owner)
    return np.nonzero((hi > lo) & (hi >= 0))[0]


def _staged(group):
    """gloo collectives run on host tensors; RCCL on device tensors."""
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo"


def all_reduce(t, op="sum", group=None):
    """In-place all-reduce of a device tensor (staged through the host for
    gloo)."""
    import torch.distributed as dist
    o = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
         "min": dist.ReduceOp.MIN}[op]
    if _staged(group):
        h = t.cpu()
        dist.all_reduce(h, op=o, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=o, group=group)
    return t


def all_gather_partials(partials, emit, group=None):
    """partials: [GB, 4] int64 tensor (raw otsdb_partial words), emit: [GB]
    uint8.  Returns rank-major [world, GB, 4] / [world, GB] tensors — the
    layout otsdb_agg_finalize_device merges in rank order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = partials.device
    if dev.type != "cpu" and _staged(group):
        partials, emit = partials.cpu(), emit.cpu()
    gp = [torch.empty_like(partials) for _ in range(world)]
    ge = [torch.empty_like(emit) for _ in range(world)]
    dist.all_gather(gp, partials.contiguous(), group=group)
    dist.all_gather(ge, emit.contiguous(), group=group)
    return torch.stack(gp).to(dev), torch.stack(ge).to(dev)


def hand_on_partials(local_step, partials, emit, group=None):
    """The chained exchange of an order-sensitive aggregator's states.

    local_step(init_p, init_e) fills `partials` [GB, 4] / `emit` [GB] with
    this rank's states: from empty states on rank 0 (init None), from the
    previous rank's output on every later one.  Rank r waits for rank r - 1
    (a point-to-point send / recv in rank = series order), so the last
    rank's states are those of ONE pass over every member; they are
    broadcast and returned (the tensors passed in, overwritten) on every
    rank.  local_step is the whole chained partials call (downsampling
    included), so the ranks run it one after another: a chained group costs
    about world x one rank's step (only shared groups of an order-sensitive
    aggregator take this path; every other group runs in parallel)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    staged = partials.device.type != "cpu" and _staged(group)

    def peer(r):
        return dist.get_global_rank(group, r) if group is not None else r

    def xfer(op, t, r):
        if staged:
            h = t.cpu() if op is dist.send else t.new_empty(t.shape,
                                                             device="cpu")
            op(h, peer(r), group=group)
            if op is dist.recv:
                t.copy_(h)
        else:
            op(t.contiguous(), peer(r), group=group)

    if rank == 0:
        local_step(None, None)
    else:
        init_p, init_e = partials.clone(), emit.clone()
        xfer(dist.recv, init_p, rank - 1)
        xfer(dist.recv, init_e, rank - 1)
        local_step(init_p, init_e)
    if rank + 1 < world:
        xfer(dist.send, partials, rank + 1)
        xfer(dist.send, emit, rank + 1)
    for t in (partials, emit):
        if staged:
            h = t.cpu()
            dist.broadcast(h, peer(world - 1), group=group)
            t.copy_(h)
        else:
            dist.broadcast(t, peer(world - 1), group=group)
    return partials, emit


def classify_groups(group_offsets, group=None, device=None):
    """(local, shared) global group ids: groups whose members this rank holds
    alone, and groups with members on more than one rank.  One MIN
    all-reduce of 2 x G int64 (the lowest rank holding a member, minus the
    highest)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    present = np.diff(np.asarray(group_offsets, np.int64)) > 0
    mm = torch.from_numpy(np.stack([np.where(present, rank, world),
                                    np.where(present, -rank, 1)]
                                   ).astype(np.int64))
    if device is not None:
        mm = mm.to(device)
    dist.all_reduce(mm, op=dist.ReduceOp.MIN, group=group)
    mm = mm.cpu().numpy()
    shared = mm[0] < -mm[1]
    return np.nonzero(present & ~shared)[0], np.nonzero(shared)[0]


class ShardPlan:
    """Which of the G global groups this rank holds alone and which span
    ranks, and the two sub-batches (same series arrays, restricted group
    CSRs) the step runs: rank-local groups finish with otsdb_agg_run_device,
    shared groups exchange 32-byte partials.  Built once per batch with one
    all-reduce of 2 x G ints (min / max rank holding a member)."""

    def __init__(self, engine, spec, dbatch, n_groups_global, group=None):
        import torch
        import torch.distributed as dist
        from .engine import DeviceBatch
        world = dist.get_world_size(group)
        goff = dbatch.group_offsets.cpu().numpy()
        mem = dbatch.group_members.cpu().numpy()
        dev = dbatch.ts.device
        self.local, self.shared = classify_groups(
            goff, group, None if _staged(group) else dev)

        def sub(ids):
            off = [0]
            m = []
            for g in ids:
                seg = mem[goff[g]:goff[g + 1]]
                m.extend(seg.tolist())
                off.append(len(m))
            return DeviceBatch(dbatch.offsets, dbatch.ts, dbatch.val,
                               torch.tensor(off, dtype=torch.int64, device=dev),
                               torch.tensor(m if m else [0], dtype=torch.int64,
                                            device=dev)[:len(m)],
                               dbatch.is_float, dbatch.series_float)
        self.local_batch = sub(self.local)
        # order-sensitive aggregators: shared groups small enough to be one
        # chain over all ranks are handed on (hand_on_partials), the rest
        # merge per-rank partials like every other aggregator
        self.chain = np.zeros(0, np.int64)
        self.merge = self.shared
        if _agg_name(spec) in ORDERED_AGGS and len(self.shared):
            sizes = torch.from_numpy(
                (goff[self.shared + 1] - goff[self.shared]).astype(np.int64))
            if not _staged(group):
                sizes = sizes.to(dev)
            all_reduce(sizes, "sum", group)
            small = sizes.cpu().numpy() <= CHAIN_MAX_MEMBERS
            if spec.flags & abi.SPEC_EXACT_ORDER:
                small[:] = True  # every shared group one chain over the ranks
            self.chain, self.merge = self.shared[small], self.shared[~small]
        self.chain_batch = sub(self.chain)
        self.shared_batch = sub(self.merge)
        sz = engine.plan(spec, self.local_batch)
        self.nb = int(sz.n_buckets)
        from .engine import DeviceResult
        self.local_res = DeviceResult(torch, len(self.local),
                                      int(sz.max_out_points), dev)
        self.world = world


class ShardedResult:
    """Per-rank result of a sharded query: the groups this rank holds alone
    (`local_ids`, `local`) and every group spanning ranks (`shared_ids`,
    identical on every rank: merged partials, `shared`, and groups whose
    states were handed on, `chained`); DeviceResult tensors."""

    def __init__(self, local_ids, local, shared_ids, shared, chain_ids=(),
                 chained=None):
        self.local_ids, self.local = local_ids, local
        self.merge_ids, self.shared = shared_ids, shared
        self.chain_ids, self.chained = np.asarray(chain_ids, np.int64), chained
        self.shared_ids = np.concatenate([np.asarray(shared_ids, np.int64),
                                          self.chain_ids])

    def _parts(self):
        return [(ids, res) for ids, res in
                ((self.local_ids, self.local), (self.merge_ids, self.shared),
                 (self.chain_ids, self.chained)) if len(ids)]

    def n_points(self):
        return sum(int(res.offsets[-1].item()) for _, res in self._parts())

    def host_groups(self):
        """{global group id: (ts, value bits, is_int)} numpy arrays of the
        groups this rank holds the result of (its own and the shared ones)."""
        out = {}
        for ids, res in self._parts():
            out.update(_host_slices(ids, res))
        return out


def _host_slices(ids, res):
    offs = res.offsets.cpu().numpy()
    ts, val, ii = (res.ts.cpu().numpy(), res.val.cpu().numpy(),
                   res.is_int.cpu().numpy())
    return {int(g): (ts[offs[k]:offs[k + 1]], val[offs[k]:offs[k + 1]],
                     ii[offs[k]:offs[k + 1]]) for k, g in enumerate(ids)}


def _agg_name(spec):
    from . import core
    return core.Aggregators.by_id(spec.agg_id).registry_name


def run_sharded(engine, spec, dbatch, n_groups_global, torch_mod=None,
                group=None, plan=None):
    """Runs one query over a rank's DeviceBatch whose group_offsets span all
    `n_groups_global` groups (empty for groups with no local members).
    Groups held by this rank alone finish locally (no collective); only the
    groups whose members span ranks exchange partials: 32 B per (shared
    group, bucket), all-gathered over RCCL and merged in rank (= series)
    order.  Returns a ShardedResult."""
    import ctypes as C
    import torch
    from .engine import DeviceResult, run_device

    if plan is None:
        # cached on the batch itself (an id()-keyed cache can hand a freed
        # batch's plan to a new one on one rank only, which then skips the
        # classification all-reduce the other ranks wait in)
        plans = getattr(dbatch, "_shard_plans", None)
        if plans is None:
            plans = dbatch._shard_plans = {}
        key = (id(engine), bytes(memoryview(spec).cast("B")), n_groups_global)
        plan = plans.get(key)
        if plan is None:
            plan = plans[key] = ShardPlan(engine, spec, dbatch,
                                          n_groups_global, group)
    if len(plan.local):
        run_device(engine, spec, plan.local_batch, plan.local_res)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    dev = dbatch.ts.device
    nb = plan.nb

    def exchange(ids, sub, chained):
        GB = len(ids) * nb
        parts = torch.zeros((max(GB, 1), PARTIAL_WORDS), dtype=torch.int64,
                            device=dev)
        emit = torch.zeros(max(GB, 1), dtype=torch.uint8, device=dev)
        b = sub.as_abi()
        if chained:
            # every rank continues its predecessor's states; rank 0 from
            # empty ones (the dev state's zero bits)
            def step(init_p, init_e):
                if init_p is None:
                    init_p, init_e = torch.zeros_like(parts), torch.zeros_like(emit)
                engine._check(engine.lib.otsdb_agg_partials_chained_device(
                    engine.ctx, C.byref(spec), C.byref(b), init_p.data_ptr(),
                    init_e.data_ptr(), parts.data_ptr(), emit.data_ptr(),
                    stream))
            hand_on_partials(step, parts, emit, group)
            gp, ge, n_ranks = parts[:GB], emit[:GB], 1
        else:
            engine._check(engine.lib.otsdb_agg_partials_device(
                engine.ctx, C.byref(spec), C.byref(b), parts.data_ptr(),
                emit.data_ptr(), stream))
            gp, ge = all_gather_partials(parts[:GB], emit[:GB], group)
            n_ranks = plan.world
        res = DeviceResult(torch, len(ids), max(GB, 1), dev)
        r = res.as_abi()
        engine._check(engine.lib.otsdb_agg_finalize_device(
            engine.ctx, C.byref(spec), len(ids), nb, n_ranks,
            gp.contiguous().data_ptr(), ge.contiguous().data_ptr(),
            C.byref(r), stream))
        return res

    merged = exchange(plan.merge, plan.shared_batch, False) \
        if len(plan.merge) else None
    chained = exchange(plan.chain, plan.chain_batch, True) \
        if len(plan.chain) else None
    return ShardedResult(plan.local, plan.local_res, plan.merge, merged,
                         plan.chain, chained)


class ShardedSelect:
    """One rank's side of the otsdb_sel_* protocol (include/otsdb_agg.h):
    prepare -> counts / emit / key range; hist_pass(p) while it reports
    more; pick; finish.  The collectives between the steps are the caller's
    (run_sharded_select, or an in-process emulation in the GPU tests)."""

    BINS = 2048  # OTSDB_SEL_BINS: u32 per (group, bucket) and pass

    @staticmethod
    def _stream():
        """torch's current stream: the protocol's kernels queue behind the
        tensor copies/collectives that feed them (the context's own stream
        may be non-blocking)."""
        import ctypes as C
        import torch
        return C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def __init__(self, engine, spec, dbatch, n_groups_global):
        import torch
        self.engine, self.spec, self.dbatch = engine, spec, dbatch
        self.G = n_groups_global
        sz = engine.plan(spec, dbatch)
        self.nb = int(sz.n_buckets)
        self.GB = self.G * self.nb
        self.dev = dbatch.ts.device
        n = max(self.GB, 1)
        self.counts = torch.zeros(n, dtype=torch.int64, device=self.dev)
        self.emit = torch.zeros(n, dtype=torch.uint8, device=self.dev)
        self.krange = torch.zeros(2 * n, dtype=torch.int64, device=self.dev)
        self.hist = torch.zeros(n * self.BINS, dtype=torch.int32,
                                device=self.dev)
        self.picks = torch.zeros(2 * n, dtype=torch.int64, device=self.dev)

    def prepare(self):
        import ctypes as C
        b = self.dbatch.as_abi()
        self.engine._check(self.engine.lib.otsdb_sel_prepare_device(
            self.engine.ctx, C.byref(self.spec), C.byref(b),
            self.counts.data_ptr(), self.emit.data_ptr(),
            self.krange.data_ptr(), self._stream()))
        return self.counts, self.emit, self.krange

    def hist_pass(self, p):
        """Pass p: applies self.hist (for p > 0 it must hold the all-reduced
        histogram of pass p - 1) and, when a pass is planned, overwrites it
        with this rank's histogram of pass p.  Returns whether it did."""
        import ctypes as C
        more = C.c_int32(0)
        self.engine._check(self.engine.lib.otsdb_sel_hist_device(
            self.engine.ctx, int(p), self.counts.data_ptr(),
            self.emit.data_ptr(), self.krange.data_ptr(),
            self.hist.data_ptr(), self.hist.data_ptr(), C.byref(more),
            self._stream()))
        return bool(more.value)

    def wait(self):
        """The histogram / pick kernels are done (otsdb_sel_hist_wait): for
        a host-staged collective that does not read through torch's current
        stream."""
        self.engine._check(self.engine.lib.otsdb_sel_hist_wait(
            self.engine.ctx, self._stream()))

    def pick(self):
        self.engine._check(self.engine.lib.otsdb_sel_pick_device(
            self.engine.ctx, self.picks.data_ptr(), self._stream()))
        return self.picks

    def finish(self):
        import ctypes as C
        import torch
        from .engine import DeviceResult
        res = DeviceResult(torch, self.G, max(self.GB, 1), self.dev)
        r = res.as_abi()
        self.engine._check(self.engine.lib.otsdb_sel_finish_device(
            self.engine.ctx, self.picks.data_ptr(), C.byref(r),
            self._stream()))
        return res


# passes the protocol can plan: the offset digit resolves >= 10 of a key's
# 64 bits, every later pass >= 10 more
MAX_SEL_PASSES = 7


def run_sharded_select(engine, spec, dbatch, n_groups_global, group=None):
    """Median / percentile over series-sharded groups: exact selection with
    all-reduces of the counts, key ranges, each pass's histograms and the
    picked keys."""
    sel = ShardedSelect(engine, spec, dbatch, n_groups_global)
    counts, emit, krange = sel.prepare()
    all_reduce(counts, "sum", group)
    all_reduce(emit, "max", group)
    all_reduce(krange, "min", group)
    p = 0
    while sel.hist_pass(p):
        if p >= MAX_SEL_PASSES:
            raise RuntimeError("selection: pass %d planned" % p)
        if _staged(group):
            sel.wait()  # the host copy below reads the histogram
        all_reduce(sel.hist, "sum", group)
        p += 1
    picks = sel.pick()
    if _staged(group):
        sel.wait()
    all_reduce(picks, "sum", group)
    return sel.finish()


def shard_host_batch(hb, world, rank, by_points=True):
    """Rank `rank`'s contiguous series range of a HostBatch (balanced by
    point count), with group offsets over every global group (members
    renumbered locally)."""
    from .batch import HostBatch
    a, b = shard_range(hb.n_series, world, rank,
                       hb.offsets if by_points else None)
    offs = hb.offsets[a:b + 1] - hb.offsets[a]
    p0, p1 = hb.offsets[a], hb.offsets[b]
    g_off = [0]
    members = []
    for g in range(hb.n_groups):
        m = hb.group_members[hb.group_offsets[g]:hb.group_offsets[g + 1]]
        loc = m[(m >= a) & (m < b)] - a
        members.extend(loc.tolist())
        g_off.append(len(members))
    return HostBatch(offs, hb.ts[p0:p1], hb.val[p0:p1],
                     None if hb.is_float is None else hb.is_float[p0:p1],
                     None if hb.series_float is None else hb.series_float[a:b],
                     np.array(g_off, np.int64), np.array(members, np.int64))


def to_device(hb, device="cuda"):
    """HostBatch -> DeviceBatch (HBM-resident torch tensors)."""
    import torch
    from .engine import DeviceBatch

    def t(x):
        if x is None:
            return None
        y = torch.from_numpy(np.ascontiguousarray(x)).to(device)
        return y
    ts = torch.zeros(max(len(hb.ts), 2), dtype=torch.int64, device=device)
    val = torch.zeros_like(ts)
    if len(hb.ts):
        ts[:len(hb.ts)] = t(hb.ts)
        val[:len(hb.ts)] = t(hb.val)
    db = DeviceBatch(t(hb.offsets), ts[:len(hb.ts)], val[:len(hb.ts)],
                     t(hb.group_offsets), t(hb.group_members),
                     t(hb.is_float), t(hb.series_float))
    db.n_points_total = len(hb.ts)
    return db


class _SelResult:
    def __init__(self, res):
        self.res = res
        self.offsets = res.offsets

    def n_points(self):
        return int(self.res.offsets[-1].item())

    def host_groups(self):
        return _host_slices(range(len(self.res.offsets) - 1), self.res)


def _all_gather_var(t, group=None):
    """All-gather of a 1-D tensor whose length differs per rank: lengths
    first, then the tensors padded to the longest.  Returns the per-rank
    tensors in rank order (on t's device)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = t.device
    staged = _staged(group)
    n = torch.tensor([t.numel()], dtype=torch.int64,
                     device="cpu" if staged else dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    L = max(max(ns), 1)
    src = t.cpu() if staged else t
    pad = torch.zeros(L, dtype=t.dtype, device=src.device)
    pad[:t.numel()] = src
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return [o[:k].to(dev) for o, k in zip(outs, ns)]


def gather_shared_series(dbatch, shared_ids, group=None):
    """Raw (non-downsampled) group-by over groups that span ranks: the
    union-timestamp merge (AggregationIterator.next, AggregationIterator.java:
    514-567) needs every member's points, so those groups run as replicas
    (SURVEY §8e): each rank contributes its members of the shared groups
    (points in SpanCmp order) and every rank gathers all of them, rank order
    being series order.  Returns a DeviceBatch over the shared groups only
    (group i = shared_ids[i]) on dbatch's device."""
    import torch
    from .engine import DeviceBatch
    dev = dbatch.ts.device
    goff = dbatch.group_offsets.cpu().numpy()
    mem = dbatch.group_members.cpu().numpy()
    offs = dbatch.offsets.cpu().numpy()
    series, gids = [], []
    for k, g in enumerate(shared_ids):
        for s in mem[goff[g]:goff[g + 1]]:
            series.append(int(s))
            gids.append(k)
    sidx = torch.tensor(series or [0], dtype=torch.int64, device=dev)[:len(series)]
    lens = torch.tensor([offs[s + 1] - offs[s] for s in series] or [0],
                        dtype=torch.int64, device=dev)[:len(series)]
    pts = (torch.cat([torch.arange(int(offs[s]), int(offs[s + 1]),
                                   dtype=torch.int64, device=dev)
                      for s in series])
           if series else torch.zeros(0, dtype=torch.int64, device=dev))
    ts = dbatch.ts[pts]
    val = dbatch.val[pts]
    if dbatch.is_float is not None:
        isf = dbatch.is_float[pts]
    elif dbatch.series_float is not None:
        isf = torch.repeat_interleave(dbatch.series_float[sidx].to(torch.uint8),
                                      lens)
    else:
        isf = torch.ones(len(pts), dtype=torch.uint8, device=dev)
    gl = torch.tensor(gids or [0], dtype=torch.int64, device=dev)[:len(gids)]
    parts = [_all_gather_var(x, group) for x in (lens, gl, ts, val, isf)]
    lens_all = torch.cat(parts[0])
    g_all = torch.cat(parts[1])
    # members of each shared group: rank-major = series order
    order = torch.argsort(g_all, stable=True)
    n_sh = len(shared_ids)
    counts = torch.bincount(g_all, minlength=n_sh) if g_all.numel() else \
        torch.zeros(n_sh, dtype=torch.int64, device=dev)
    g_off = torch.zeros(n_sh + 1, dtype=torch.int64, device=dev)
    g_off[1:] = torch.cumsum(counts, 0)
    offsets = torch.zeros(lens_all.numel() + 1, dtype=torch.int64, device=dev)
    offsets[1:] = torch.cumsum(lens_all, 0)
    cat = lambda xs: torch.cat(xs) if xs else xs  # noqa: E731
    ts_all, val_all, isf_all = cat(parts[2]), cat(parts[3]), cat(parts[4])
    # 16-byte aligned columns for the engine's streaming loads
    n = ts_all.numel()
    tsb = torch.zeros(max(n, 2), dtype=torch.int64, device=dev)
    vb = torch.zeros_like(tsb)
    tsb[:n] = ts_all
    vb[:n] = val_all
    db = DeviceBatch(offsets, tsb[:n], vb[:n], g_off, order.contiguous(),
                     isf_all.contiguous(), None)
    db.n_points_total = n
    return db


def run_sharded_raw(engine, spec, dbatch, n_groups_global, group=None):
    """Raw group-by over series-sharded ranks: groups a rank holds alone run
    locally; groups spanning ranks run as replicas over their gathered
    members (gather_shared_series), identical on every rank."""
    import torch
    from .engine import DeviceResult, run_device
    plans = getattr(dbatch, "_shard_plans", None)
    if plans is None:
        plans = dbatch._shard_plans = {}
    key = (id(engine), bytes(memoryview(spec).cast("B")), n_groups_global,
           "raw")
    plan = plans.get(key)
    if plan is None:
        plan = plans[key] = ShardPlan(engine, spec, dbatch, n_groups_global,
                                      group)
    if len(plan.local):
        run_device(engine, spec, plan.local_batch, plan.local_res)
    shared_res = None
    if len(plan.shared):
        sb = gather_shared_series(dbatch, plan.shared, group)
        cap = int(engine.plan(spec, sb).max_out_points)
        shared_res = DeviceResult(torch, len(plan.shared), max(cap, 1),
                                  dbatch.ts.device)
        run_device(engine, spec, sb, shared_res)
    return ShardedResult(plan.local, plan.local_res, plan.shared, shared_res)


def run_sharded_any(engine, spec, dbatch, n_groups_global, group=None):
    """Dispatch: selection aggregators take the histogram protocol, raw
    (non-downsampled) queries the replica exchange, every other aggregator
    the shared-group partial exchange.  The result has n_points()."""
    raw = not (spec.ds_interval_ms > 0 or spec.run_all)
    if raw:
        return run_sharded_raw(engine, spec, dbatch, n_groups_global, group)
    if spec.agg_id == 5 or spec.agg_id >= 17:  # median, p*, ep*
        return _SelResult(run_sharded_select(engine, spec, dbatch,
                                             n_groups_global, group))
    return run_sharded(engine, spec, dbatch, n_groups_global, group=group)


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
