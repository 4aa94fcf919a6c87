"""CPU model of the cross-rank selection protocol's plan (otsdb_sel_*,
opentsdb_amd/csrc/select.hip k_xsel_*): the same offset digit, digit widths,
candidate pool and pick rule, run over the keys of one (group, bucket)
segment split across ranks.  It counts each rank's passes over its local
keys on adversarial key sets (the protocol promises two at most) and checks
the order statistics against a sort.  The kernels' own counters are checked
on the GPU (test_gpu_sharded.py::test_selection_protocol_edges)."""
import numpy as np
import pytest

from opentsdb_amd import dist as odist

BINS = 2048


def _bitlen(x):
    return int(x).bit_length()


class _Target:
    def __init__(self, rank, n):
        self.prefix, self.shift, self.rank, self.cnt = 0, 64, rank, n
        self.done, self.w = 0, 0

    def match(self, k):
        if self.shift >= 64:
            return np.ones(len(k), bool)
        s = np.uint64(self.shift)
        return (k >> s) == np.uint64(self.prefix >> self.shift)

    def digit(self, k):
        return ((k >> np.uint64(self.shift - self.w)) &
                np.uint64((1 << self.w) - 1)).astype(np.int64)


def _apply(t, h, offset=None):
    """k_xsel_apply for one target over its bins h."""
    cum = np.cumsum(h)
    d = int(np.searchsorted(cum, t.rank, side="right"))
    assert d < len(h), "rank past the bins"
    below = int(cum[d - 1]) if d else 0
    t.rank -= below
    t.cnt = int(h[d])
    if offset is not None:
        s1, base = offset
        t.prefix, t.shift = (base + d) << s1, s1
    else:
        t.shift -= t.w
        t.prefix |= d << t.shift
    t.w = 0
    if t.shift == 0:
        t.done = 1
    elif t.cnt == 1:
        t.done = 2


def select(rank_keys, ranks):
    """rank_keys: per rank the uint64 keys of the segment; ranks: the one or
    two order statistics.  Returns (keys, reads per rank, histogram passes,
    pool sizes per rank)."""
    R = len(rank_keys)
    reads = [0] * R
    n = sum(len(k) for k in rank_keys)
    ts = [_Target(r, n) for r in ranks]
    nonempty = [k for k in rank_keys if len(k)]
    mn = min(int(k.min()) for k in nonempty)
    mx = max(int(k.max()) for k in nonempty)
    if mn == mx:
        return [mn] * len(ts), reads, 0, [0] * R
    # pass 0: the offset digit, one histogram the targets share
    s1 = max(_bitlen(mx - mn) - 11, 0)
    while (mx >> s1) - (mn >> s1) >= BINS:
        s1 += 1
    base = mn >> s1
    h = np.zeros(BINS, np.int64)
    for r, k in enumerate(rank_keys):
        reads[r] += 1
        h += np.bincount(((k >> np.uint64(s1)) - np.uint64(base)).astype(np.int64),
                         minlength=BINS)
    for t in ts:
        _apply(t, h, (s1, base))
    passes, pools = 1, None
    while True:
        # xs_plan
        op = [t for t in ts if t.done == 0]
        if not op:
            break
        same = len(op) == 2 and op[0].prefix == op[1].prefix and \
            op[0].shift == op[1].shift
        split = len(op) == 2 and not same
        wmax = 10 if split else 11
        for t in op:
            t.w = min(wmax, t.shift)
        if pools is None:  # pass 1 reads the keys and builds the pool
            keep = lambda k: np.logical_or.reduce(
                [t.match(k) for t in ts if t.done != 1])
            pools = []
            for r, k in enumerate(rank_keys):
                reads[r] += 1
                pools.append(k[keep(k)] if len(k) else k)
        src = pools
        hs = [np.zeros(1024 if split else BINS, np.int64) for _ in op]
        for k in src:
            for i, t in enumerate(op):
                m = t.match(k)
                hs[i] += np.bincount(t.digit(k[m]), minlength=len(hs[i]))
        for i, t in enumerate(op):
            _apply(t, hs[0] if same else hs[i])
        passes += 1
    out = []
    for t in ts:
        if t.done == 1:
            out.append(t.prefix)
            continue
        # the pick: the one key of the bin, from the pool (else the keys)
        src = pools
        if src is None:
            src = rank_keys
            for r in range(R):
                reads[r] += 1
        hit = [k[t.match(k)] for k in src]
        got = np.concatenate(hit)
        assert len(got) == 1, len(got)
        out.append(int(got[0]))
    psz = [len(p) for p in pools] if pools is not None else [0] * R
    return out, reads, passes, psz


def _keys_of(v):
    u = np.asarray(v, np.float64).view(np.uint64)
    neg = (u >> np.uint64(63)) == np.uint64(1)
    return np.where(neg, ~u, u | np.uint64(1 << 63))


def _cases(rng):
    yield "uniform", _keys_of(rng.random(50000) * 100.0)
    yield "signed", _keys_of(rng.standard_normal(30000) *
                             10.0 ** rng.integers(-300, 300, 30000))
    yield "dense", np.uint64(1 << 62) + np.arange(100000, dtype=np.uint64)
    yield "bits", np.array([1 << i for i in range(64)] * 50, np.uint64)
    yield "outlier", np.concatenate([np.arange(1 << 18, dtype=np.uint64),
                                     np.array([(1 << 64) - 2], np.uint64)])
    yield "ties", np.full(5000, 12345, np.uint64)
    yield "two", np.array([7] * 3000 + [9] * 2, np.uint64)
    yield "clustered", _keys_of(np.where(rng.random(40000) < 0.005, 1e6,
                                         1.0 + rng.random(40000) * 1e-12))


@pytest.mark.parametrize("world", [1, 2, 8])
def test_selection_plan_reads_keys_at_most_twice(world):
    rng = np.random.default_rng(5)
    for name, keys in _cases(rng):
        rng.shuffle(keys)
        cuts = np.sort(rng.integers(0, len(keys), world - 1))
        parts = np.split(keys, cuts)
        srt = np.sort(keys)
        n = len(keys)
        for ranks in ([n // 2], [0], [n - 1], [int(0.99 * n) - 1, int(0.99 * n)],
                      [n - 2, n - 1]):
            got, reads, passes, psz = select(parts, ranks)
            assert got == [int(srt[r]) for r in ranks], (name, ranks)
            assert max(reads) <= 2, (name, ranks, reads)
            assert passes <= odist.MAX_SEL_PASSES, (name, ranks, passes)
            assert all(p <= len(k) for p, k in zip(psz, parts))
