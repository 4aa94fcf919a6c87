"""Self-tests of the parity comparator (CPU only): the sweeps' comparator
must reject results that differ from the reference's in exactly the rules
the rate path implements.  A mutated oracle (its junk first rate scaled by
1 + 1e-6, RateSpan.java:109-115, held by AggregationIterator.java:448-459
until a span's first real rate) stands in for a wrong GPU result; the
comparator run with the sweeps' own floor must flag it wherever the
mutation reaches the output beyond the comparator's own bound.  (The
round-2 floor, 1e-12 x 2,000 x max|raw counter|, about 8.6 absolute, let 15
of the 17 visibly mutated rate queries pass; the contribution floor
catches all 17.)"""
import numpy as np
import pytest

from oracle import pyoracle
from tests.test_gpu_parity import compare, contribution_floor
from tests.test_gpu_sweep import _case, _rate_case


class _Res:
    """An oracle group result in the engine's result shape."""

    def __init__(self, pts):
        self.ts, self.bits, self.is_int = pts["ts"], pts["bits"], pts["is_int"]


def _mutated(spec, b, scale):
    with pyoracle.junk_rate_scaled(scale):
        return pyoracle.group_by(spec, b)


def _visible(mut, ref, floor):
    """The mutation changes some output point by more than ten times the
    comparator's own bound there (a 1e-6 change of one term among many, or
    under another term's propagated rounding, is below what any comparator
    at this precision can see)."""
    from tests.test_gpu_parity import _vals
    for g, (x, y) in enumerate(zip(mut, ref)):
        if len(x) != len(y):
            return True
        a, r = _vals(x["bits"], x["is_int"]), _vals(y["bits"], y["is_int"])
        if not (np.isnan(a) == np.isnan(r)).all():
            return True
        ok = ~np.isnan(r)
        tol = 1e-12 * np.abs(r[ok]) + np.asarray(floor[g])[ok]
        if (np.abs(a - r)[ok] > 10 * tol).any():
            return True
    return False


def test_comparator_catches_a_perturbed_junk_rate():
    caught = reached = 0
    for seed in range(60):
        b, spec, exact, where = _rate_case(seed)
        try:
            ref = pyoracle.group_by(spec, b)
        except pyoracle.OracleError:
            continue
        mut = _mutated(spec, b, 1.0 + 1e-6)
        fl = contribution_floor(spec, b, ref)
        if not _visible(mut, ref, fl):
            continue  # the junk rate does not reach this query's output
        reached += 1
        with pytest.raises(AssertionError):
            compare([_Res(p) for p in mut], ref, exact, where, fl)
        caught += 1
    # the generator puts junk rates into most rate queries' output
    assert reached >= 15, reached
    assert caught == reached


def test_contribution_floor_is_zero_for_same_signed_contributions():
    """All-positive float data (U[0,100)): nothing can cancel, so the
    comparator is the pure 1e-12 relative bound everywhere."""
    from opentsdb_amd import core
    from tests import datasets
    b = datasets.random_batch(11, n_series=30, n_groups=3)
    spec = core.make_spec(datasets.T0, datasets.T0 + 3 * 3600 * 1000,
                          core.Aggregators.get("sum"),
                          core.DownsamplingSpecification("1m-avg"),
                          datasets.T0, datasets.T0 + 3 * 3600 * 1000)
    ref = pyoracle.group_by(spec, b)
    fl = contribution_floor(spec, b, ref)
    assert sum(len(f) for f in fl) > 0
    assert all((f == 0).all() for f in fl)


def test_contribution_floor_is_set_where_signs_meet():
    """Mixed-sign integer data (U[-50,100)): the floor is nonzero only where
    both signs meet, finite, and far below the old raw-value floor
    (1e-12 x 2,000 x max|raw|)."""
    n_nonzero = n_points = 0
    for seed in range(40):
        b, spec, exact, where = _case(seed)
        if spec.interp in (2, 3) or spec.rate:  # +-MAX_VALUE fill-ins
            continue
        try:
            ref = pyoracle.group_by(spec, b)
        except pyoracle.OracleError:
            continue
        for f in contribution_floor(spec, b, ref):
            assert (f >= 0).all() and np.isfinite(f).all()
            n_nonzero += int((f > 0).sum())
            n_points += len(f)
    assert 0 < n_nonzero < n_points


def _tree_dev(xs, run=8):
    """A bucket's population sigma from Welford runs of `run` consecutive
    points merged with Chan's formula (the lane tree the engine no longer
    uses for dev)."""
    n, mean, m2 = 0, 0.0, 0.0
    for i in range(0, len(xs), run):
        c = xs[i:i + run]
        cn, cm, cm2 = 1, c[0], 0.0
        for x in c[1:]:
            cn += 1
            nm = cm + (x - cm) / cn
            cm2 += (x - cm) * (x - nm)
            cm = nm
        if n == 0:
            n, mean, m2 = cn, cm, cm2
            continue
        d = cm - mean
        tot = n + cn
        mean = mean + d * (cn / tot)
        m2 = m2 + cm2 + d * d * (n * cn / tot)
        n = tot
    return 0.0 if n < 2 else float(np.sqrt(m2 / n))


def test_comparator_rejects_a_reordered_welford():
    """dev downsampling replayed in another order (runs of 8 merged with
    Chan's formula) over counters near 2^32: the comparator, run with the
    sweeps' floor, rejects it (the round-3 floor of n x max|raw| per dev
    bucket let exactly this through: sweep seed 5266)."""
    from opentsdb_amd import core
    from opentsdb_amd.batch import groups_from_ids
    from tests import datasets
    b = datasets.random_batch(5266, n_series=6, n_groups=6, counter=True,
                              empty_frac=0.0, outside=False)
    g_off, members = groups_from_ids(np.arange(6), 6)  # a group per series
    b.group_offsets, b.group_members = g_off, members
    t0, t1 = datasets.T0, datasets.T0 + 3 * 3600 * 1000
    spec = core.make_spec(t0, t1, core.Aggregators.get("sum"),
                          core.DownsamplingSpecification("5m-dev"), t0, t1)
    ref = pyoracle.group_by(spec, b)
    fl = contribution_floor(spec, b, ref)
    mut = []
    for g, r in enumerate(ref):
        s = int(members[g])
        ts = b.ts[b.offsets[s]:b.offsets[s + 1]]
        v = b.val[b.offsets[s]:b.offsets[s + 1]].astype(np.float64)
        m = r.copy()
        for k, bt in enumerate(r["ts"]):
            sel = (ts >= bt) & (ts < bt + 300000)
            m["bits"][k] = np.float64(_tree_dev(list(v[sel]))).view(np.int64)
        mut.append(m)
    assert any((m["bits"] != r["bits"]).any() for m, r in zip(mut, ref))
    with pytest.raises(AssertionError):
        compare([_Res(p) for p in mut], ref, False, "reordered-dev", fl)


def _sweep_cases():
    """The general sweep's first 120 seeds and sweep_many.py's 5000-5399 (the
    seeds whose MAX / MIN fill-ins gave round 4's comparator floors of
    ~1e296 or infinity: 5007, 5184, 5255, 5397)."""
    for seed in list(range(120)) + list(range(5000, 5400)):
        b, spec, exact, where = _case(seed)
        try:
            ref = pyoracle.group_by(spec, b)
        except pyoracle.OracleError:
            continue
        yield b, spec, exact, where, ref


def test_contribution_floors_are_finite_and_bounded():
    """No floor of the sweep comparator is infinite or lets a MAX_VALUE
    fill-in in: every floor is at most 2e-12 x the sum over the group's
    members of the largest scale of the member's own view stream — a bound
    computed from the real contributions only, whatever the interpolation
    (AggregationIterator.java:711-719, :781-787)."""
    from tests.test_gpu_parity import _member_scales
    n_fill = 0
    for b, spec, exact, where, ref in _sweep_cases():
        views = _member_scales(spec, b)
        fl = contribution_floor(spec, b, ref, views)
        n_fill += spec.interp in (2, 3)
        for g, (f, gv) in enumerate(zip(fl, views)):
            assert np.isfinite(f).all(), where
            bound = 2e-12 * sum(float(sc.max()) for _, _, sc in gv if len(sc))
            assert (f <= bound).all(), "%s/g%d: floor %g > %g" % (
                where, g, f.max(), bound)
    assert n_fill >= 40, n_fill  # the generator's MAX / MIN overrides


def test_comparator_sees_perturbed_fill_in_results():
    """Every sweep query with a MAX / MIN fill-in (mimmin / mimmax, whose
    default interpolation it is, and the i2 / i3 overrides): a 1e-9 relative
    change of any nonzero output point is outside the comparator's bound at
    all but a handful of points (where the result is a near-cancellation of
    real contributions).  Round 4's floors took the fill-ins' MAX_VALUE as a
    scale and were blind at 910 of these 26,302 points; now 4."""
    from tests.test_gpu_parity import _vals
    n = blind = 0
    for b, spec, exact, where, ref in _sweep_cases():
        agg = where.split(":")[1]
        if spec.rate or not (spec.interp in (2, 3) or
                             agg in ("mimmin", "mimmax")):
            continue
        for r, f in zip(ref, contribution_floor(spec, b, ref)):
            v = _vals(r["bits"], r["is_int"])
            sel = np.isfinite(v) & (v != 0) & (np.abs(v) < 1e300)
            tol = 1e-12 * np.abs(v[sel]) + np.asarray(f)[sel]
            n += int(sel.sum())
            blind += int((1e-9 * np.abs(v[sel]) <= tol).sum())
    assert n > 20000, n
    assert blind <= n // 1000, (blind, n)
