"""Parity of the HIP engine (through the C-ABI) with the CPU oracle and with
the reference's transcribed known answers.  Needs an MI355X.

Bar (north star): timestamps, emission, counts, min/max/first/last and
anything computed from order-insensitive inputs are bit-exact; double
sum/avg/dev/mult/squareSum within 1e-12 relative where the reduction order
differs (downsample buckets are reduced in a wavefront tree, chunks of 256
series and ranks merge their partials in order; inside a chunk the
cross-series aggregator is fed in the reference's SpanCmp order).

The tolerance is relative: |got - ref| <= 1e-12 * max(|got|, |ref|).  An
absolute term is added only where the compared value is a sum of terms of
both signs that can cancel (mixed-sign integer data, `diff` downsampling,
rates of counters); it is the forward-error bound of such a sum,
1e-12 * (number of terms) * max|term| (cancel_floor), and each use names why.
"""
import math

import numpy as np
import pytest

from opentsdb_amd import core
from opentsdb_amd.engine import Engine
from oracle import pyoracle
from tests import datasets, kat

pytestmark = pytest.mark.gpu

ORDER_FREE = {"min", "max", "mimmin", "mimmax", "first", "last", "count",
              "diff"}
# cross-series aggregators whose result moves by at most the largest error
# of one contribution: selections, percentiles (between two selections),
# population sigma, last - first
LIPSCHITZ_AGG = ({"dev", "diff", "min", "max", "mimmin", "mimmax", "first",
                  "last", "median"} |
                 {"p%s" % q for q in ("999", "99", "95", "90", "75", "50")} |
                 {"ep%sr%d" % (q, k) for q in ("999", "99", "95", "90", "75",
                                              "50") for k in (3, 7)})


@pytest.fixture(scope="module")
def engine():
    from opentsdb_amd import build
    build.build()
    e = Engine(0)
    yield e
    e.close()


def _vals(bits, is_int):
    b = np.asarray(bits, np.int64)
    f = b.view(np.float64).copy()
    ii = np.asarray(is_int).astype(bool)
    f[ii] = b[ii].astype(np.float64)
    return f


def cancel_floor(batch, terms):
    """Absolute error bound of a sum of `terms` values of both signs drawn
    from the batch (|sum error| <= 1e-12 * terms * max|x|)."""
    b = np.asarray(batch.val, np.int64)
    if len(b) == 0:
        return 0.0
    f = b.view(np.float64)
    isf = (np.ones(len(b), bool) if batch.is_float is None
           else np.asarray(batch.is_float).astype(bool))
    mags = np.where(isf, np.abs(np.nan_to_num(f, nan=0.0, posinf=0.0,
                                             neginf=0.0)),
                    np.abs(b.astype(np.float64)))
    return 1e-12 * terms * float(mags.max())


# downsampling functions the engine computes bit-identically to the
# reference: order-free ones, and dev (one sequential Welford pass per
# bucket in point order, Aggregators.java:547-568) and diff (one subtraction)
ORDER_FREE_DS = {"min", "max", "mimmin", "mimmax", "first", "last", "count",
                 "median", "p50", "p75", "p90", "p95", "p99", "p999",
                 "dev", "diff"}


def _spec_variant(spec, **kw):
    """A copy of a query spec with some fields changed (the calendar tables
    stay the original spec's: keep it alive)."""
    s2 = type(spec).from_buffer_copy(spec)
    for k, v in kw.items():
        setattr(s2, k, v)
    return s2


def _member_scales(spec, batch):
    """Per group, per member SpanGroup.add keeps (SpanGroup.java:295-339):
    (ts, value, scale) of its view stream (Downsampler / RateSpan output,
    seeked to the window start like AggregationIterator.java:421-437) — the
    value the aggregator is fed and the magnitude its rounding is relative
    to.  A downsampled value's scale is |value|, or n x max|raw value| of
    its bucket when it is a sum over raw values of both signs (dev and diff
    buckets are bit-exact: no scale beyond |value|); a rate's is
    (scale(v0) + scale(v1)) / dt of the two bucket values it differences
    (counterMax added at a counter wrap, RateSpan.java:121-180)."""
    from opentsdb_amd import core as _core
    offs = np.asarray(batch.offsets, np.int64)
    ts = np.asarray(batch.ts, np.int64)
    val = np.asarray(batch.val, np.int64)
    isf = (np.ones(len(val), np.uint8) if batch.is_float is None
           else np.asarray(batch.is_float, np.uint8))
    g_off = np.asarray(batch.group_offsets, np.int64)
    members = np.asarray(batch.group_members, np.int64)
    ds = spec.ds_interval_ms > 0 or spec.run_all
    ds_name = _core.Aggregators.by_id(spec.ds_agg_id).registry_name if ds \
        else None
    plain = _spec_variant(spec, rate=0)
    if ds:
        # bucket min / max / count of the raw values (same grid)
        v_min = _spec_variant(spec, rate=0, ds_agg_id=_core.Aggregators.MIN.id)
        v_max = _spec_variant(spec, rate=0, ds_agg_id=_core.Aggregators.MAX.id)
        v_cnt = _spec_variant(spec, rate=0,
                              ds_agg_id=_core.Aggregators.COUNT.id)
    out = []
    for g in range(len(g_off) - 1):
        views = []
        for sid in members[g_off[g]:g_off[g + 1]]:
            p0, p1 = int(offs[sid]), int(offs[sid + 1])
            if p1 <= p0 or not (ts[p0] <= spec.end_ms and
                                ts[p1 - 1] >= spec.start_ms):
                continue
            sl = (ts[p0:p1], val[p0:p1], isf[p0:p1])

            def view(sp):
                v = pyoracle.view_stream(sp, *sl, seek=spec.start_ms)
                return v["ts"], _vals(v["bits"], v["is_int"])
            dts, dv = view(plain)
            scale = np.abs(np.nan_to_num(dv, nan=0.0))
            # a bucket value computed exactly rounds nowhere: order-free
            # functions, and sums / averages of longs below 2^53
            exact = np.full(len(dv), ds_name in ORDER_FREE_DS)
            if ds_name in ("sum", "zimsum", "pfsum", "avg") and \
                    not sl[2].any() and (np.abs(dv) < 2.0 ** 52).all():
                exact[:] = True
            if ds and ds_name not in ORDER_FREE_DS:
                _, mn = view(v_min)
                _, mx = view(v_max)
                _, n = view(v_cnt)
                mn, mx, n = np.nan_to_num(mn), np.nan_to_num(mx), np.nan_to_num(n)
                raw = np.maximum(np.abs(mn), np.abs(mx)) * np.maximum(n, 1)
                cancels = (mn < 0) & (mx > 0)
                scale = np.where(cancels, np.maximum(scale, raw), scale)
            if not spec.rate:
                views.append((dts, dv, scale))
                continue
            rts, rv = view(spec)
            # each rate's bucket pair: the ds point at its ts and the one
            # before it (the (0, 0) reset point for the junk rate); only an
            # inexact bucket value carries rounding into the difference
            err = np.where(exact, 0.0, scale)
            k = np.searchsorted(dts, rts)
            s1 = err[k]
            s0 = np.where(k > 0, err[np.maximum(k - 1, 0)], 0.0)
            t0 = np.where(k > 0, dts[np.maximum(k - 1, 0)], 0)
            v0 = np.where(k > 0, dv[np.maximum(k - 1, 0)], 0.0)
            wrap = bool(spec.counter) & (dv[k] < v0)
            s0 = s0 + np.where(wrap & ~exact[k], float(spec.counter_max), 0.0)
            dt = np.maximum((rts - t0) / 1000.0, 1e-3)
            rscale = (s0 + s1) / dt
            views.append((rts, rv, rscale + np.abs(np.nan_to_num(rv))))
        out.append(views)
    return out


def contribution_floor(spec, batch, ref, views=None):
    """Per emitted point, the absolute floor 1e-12 x sum of the scales of
    the values the cross-series aggregator is fed at that timestamp
    (AggregationIterator.java:682-797) — each member's real value, or its
    interpolated / held one bounded by its neighbours — from the oracle's
    per-member view streams (_member_scales: |value|, or the raw magnitude
    a downsampled value or a rate was computed from when that computation
    subtracts).  Nonzero only where rounding can be amplified: the
    contributions have both signs, the aggregator subtracts (dev, diff), or
    a contribution's own computation does (rates; sums over raw values of
    both signs).  Elsewhere the comparator is the
    pure 1e-12 relative bound (a sum of same-signed terms keeps its relative
    error).

    A member filled in with Long/Double MAX_VALUE or -MAX_VALUE (MAX / MIN
    interpolation, AggregationIterator.java:711-719, :781-787) contributes
    an exact constant: it carries no rounding and takes no part in the floor
    (scale 0, no sign), so every floor is at most 1e-12 x the sum of the
    real contributions' scales (tests/test_comparator_cpu.py checks that
    over the sweep generator).  Aggregators whose result moves by at most
    one contribution's error (LIPSCHITZ_AGG: selections, percentiles, dev,
    diff) take 2e-12 x the largest scale instead of the sum, avg the sum's
    floor / the number of contributions."""
    interp = spec.interp
    if interp < 0:
        interp = core.Aggregators.by_id(spec.agg_id).interpolationMethod()
    interp = int(interp)
    agg = core.Aggregators.by_id(spec.agg_id).registry_name
    floors = []
    if views is None:
        views = _member_scales(spec, batch)
    for gviews, r in zip(views, ref):
        x = np.asarray(r["ts"], np.int64)
        mag = np.zeros(len(x))
        mag_max = np.zeros(len(x))
        n_live = np.zeros(len(x), np.int64)
        pos = np.zeros(len(x), bool)
        neg = np.zeros(len(x), bool)
        amp = np.zeros(len(x), bool)  # a contribution's own subtraction
        for vts, vv, sc in gviews:
            if len(vts) == 0:
                continue
            v = np.nan_to_num(vv, nan=0.0)
            i = np.searchsorted(vts, x, "left")
            last = len(vts) - 1
            exact_pt = (i <= last) & (vts[np.minimum(i, last)] == x)
            y1, s1 = v[np.minimum(i, last)], sc[np.minimum(i, last)]
            y0, s0 = v[np.maximum(i - 1, 0)], sc[np.maximum(i - 1, 0)]
            if spec.rate:
                # every kept span contributes from the first emitted ts with
                # its latest rate at or before x, the junk rate included
                # (AggregationIterator.java:448-459, :744-753)
                live = x <= vts[-1]
                held = np.where(i > 0, y0, v[0])
                hs = np.where(i > 0, s0, sc[0])
                lo = hi = np.where(exact_pt, y1, held)
                m = np.where(exact_pt, s1, hs)
            else:
                live = (x >= vts[0]) & (x <= vts[-1])
                if interp == 0:    # LERP: between its neighbours
                    lo, hi, m = y0, y1, np.maximum(s0, s1)
                elif interp == 1:  # ZIM
                    lo = hi = m = np.zeros(len(x))
                elif interp in (2, 3):  # MAX / MIN: an exact constant
                    live = live & exact_pt
                    lo = hi = m = np.zeros(len(x))
                else:              # PREV
                    lo = hi = y0
                    m = s0
                lo = np.where(exact_pt, y1, lo)
                hi = np.where(exact_pt, y1, hi)
                m = np.where(exact_pt, s1, m)
            mag += np.where(live, m, 0.0)
            mag_max = np.maximum(mag_max, np.where(live, m, 0.0))
            n_live += live
            pos |= live & ((lo > 0) | (hi > 0))
            neg |= live & ((lo < 0) | (hi < 0))
            amp |= live & (m > np.maximum(np.abs(lo), np.abs(hi)))
        need = (pos & neg) | amp | (agg in ("dev", "diff"))
        if agg in LIPSCHITZ_AGG:
            # |f(x + d) - f(x)| <= max|d_i| (population sigma, last - first,
            # a selection or an interpolation between two selections): the
            # largest contribution error bounds the result's, whatever the
            # group size
            fl = 2e-12 * mag_max
        elif agg == "avg":
            fl = 1e-12 * mag / np.maximum(n_live, 1)
        else:
            fl = 1e-12 * mag
        floors.append(np.where(need, fl, 0.0))
    return floors


def compare(got, ref, exact, where="", floor=0.0):
    """floor: a scalar, or one per-point array per group
    (contribution_floor)."""
    assert len(got) == len(ref), "%s: %d groups vs %d" % (where, len(got), len(ref))
    for g, (a, r) in enumerate(zip(got, ref)):
        w = "%s/g%d" % (where, g)
        assert len(a.ts) == len(r), "%s: %d points vs oracle %d" % (w, len(a.ts), len(r))
        if len(r) == 0:
            continue
        assert np.array_equal(np.asarray(a.ts), r["ts"]), w + ": timestamps"
        assert np.array_equal(np.asarray(a.is_int).astype(bool),
                              r["is_int"].astype(bool)), w + ": is_int"
        va, vr = _vals(a.bits, a.is_int), _vals(r["bits"], r["is_int"])
        na, nr = np.isnan(va), np.isnan(vr)
        assert np.array_equal(na, nr), w + ": NaN pattern %s vs %s" % (
            va[na != nr][:4], vr[na != nr][:4])
        if exact:
            bad = (np.asarray(a.bits) != r["bits"]) & ~na
            assert not bad.any(), "%s: not bit-exact at %s: %r vs %r" % (
                w, np.nonzero(bad)[0][:5], va[bad][:5], vr[bad][:5])
        else:
            fl = floor if np.isscalar(floor) else np.asarray(floor[g])[~na]
            d = np.abs(va - vr)[~na]
            tol = 1e-12 * np.maximum(np.abs(va), np.abs(vr))[~na] + fl
            inf = ~np.isfinite(va[~na]) | ~np.isfinite(vr[~na])
            assert np.array_equal(va[~na][inf], vr[~na][inf]), w + ": inf"
            ok = (d <= tol) | inf
            assert ok.all(), "%s: |err| %g at %r vs %r (tol %g)" % (
                w, d[~ok].max(), va[~na][~ok][:3], vr[~na][~ok][:3],
                tol[~ok][0])


def run_both(engine, spec, batch):
    try:
        ref = pyoracle.group_by(spec, batch)
        ref_err = None
    except pyoracle.OracleError as e:
        ref, ref_err = None, e.status
    try:
        got = engine.run(spec, batch)
        got_err = None
    except core.OpenTSDBException as e:
        got, got_err = None, e.status
    assert got_err == ref_err, "engine status %s vs oracle %s" % (got_err, ref_err)
    return got, ref


def check(engine, spec, batch, exact, where="", floor=0.0):
    """run_both + compare; a query both sides reject is parity too.
    floor="contributions": contribution_floor of the oracle's result."""
    got, ref = run_both(engine, spec, batch)
    if ref is not None:
        if isinstance(floor, str):
            assert floor == "contributions"
            floor = contribution_floor(spec, batch, ref)
        compare(got, ref, exact, where, floor)
    return got, ref


# ------------------------------------------------------------------ KATs
def _points(dps):
    pts = np.zeros(len(dps.ts), pyoracle.POINT)
    pts["ts"], pts["bits"], pts["is_int"] = dps.ts, dps.bits, dps.is_int
    return pts


@pytest.mark.parametrize("c", kat.load_cases("group_by"), ids=lambda c: c["name"])
def test_reference_kat(engine, c):
    spec = kat.spec_from_case(c["spec"])
    batch = kat.batch_from_case(c)
    got = engine.run(spec, batch)
    for g, exp in enumerate(c["expect"]):
        pts = _points(got[g])
        if c.get("post"):
            # a Downsampler over the aggregate (TestAggregationIterator
            # testDownsample_afterAggregation): the engine again, over the
            # aggregate as one span
            from opentsdb_amd.batch import HostBatch
            agg1 = HostBatch.from_groups([[[
                (int(p["ts"]), kat.point_value(p["bits"], p["is_int"]),
                 0 if p["is_int"] else 1) for p in pts]]])
            iv = c["post"]["ds_interval_ms"]
            t0 = int(pts["ts"][0]) if len(pts) else 0
            d = dict(c["post"], agg="sum", start_ms=t0 - t0 % iv,
                     end_ms=int(pts["ts"][-1]) if len(pts) else 1)
            pts = _points(engine.run(kat.spec_from_case(d), agg1)[0])
        kat.check_points(pts, exp, c["tol"], "%s/g%d" % (c["name"], g))


@pytest.mark.parametrize("c", [c for c in kat.load_cases("view") if "error" not in c],
                         ids=lambda c: c["name"])
def test_reference_view_kat(engine, c):
    """The reference's Downsampler / FillingDownsampler / RateSpan KATs as
    the one-span query the engine runs (kat.view_as_query): where that query
    yields the view's own points (the oracle's group_by reproduces the KAT),
    the engine must yield the KAT's points; elsewhere (a junk first rate, a
    filling grid past the iterator's end) it must equal the oracle's query."""
    spec, batch = kat.view_as_query(c)
    ref = pyoracle.group_by(spec, batch)[0]
    got = _points(engine.run(spec, batch)[0])
    exp = c["expect"]
    try:
        kat.check_points(ref[:len(exp)] if c.get("prefix") else ref, exp,
                         c["tol"], c["name"])
        same = True
    except AssertionError:
        same = False
    if same:
        kat.check_points(got[:len(exp)] if c.get("prefix") else got, exp,
                         c["tol"], c["name"])
    else:
        from opentsdb_amd.engine import DataPoints
        compare([DataPoints(got["ts"], got["bits"], got["is_int"])], [ref],
                False, where=c["name"])


# ------------------------------------------------------- parity matrix
def _spec(agg, ds, fill="none", start=None, end=None, rate=False, ro=None,
          interp=None, interval="1m"):
    d = core.DownsamplingSpecification("%s-%s-%s" % (interval, ds, fill))
    s0 = datasets.T0 if start is None else start
    e0 = datasets.T0 + 3 * 3600 * 1000 if end is None else end
    return core.make_spec(s0, e0, core.Aggregators.get(agg), d, s0, e0, rate,
                          ro, interp)


AGGS = ["sum", "zimsum", "pfsum", "avg", "min", "max", "mimmin", "mimmax",
        "dev", "count", "first", "last", "diff", "mult", "squareSum",
        "median", "p50", "p90", "p99", "p999", "ep95r3", "ep75r7"]
DS = ["avg", "sum", "min", "max", "count", "first", "last", "dev", "diff",
      "mult", "squareSum", "zimsum", "mimmax"]


@pytest.mark.parametrize("agg", AGGS)
def test_cross_series_aggregators(engine, agg):
    b = datasets.random_batch(11, n_series=60, n_groups=6)
    for ds in ("avg", "max"):
        spec = _spec(agg, ds)
        # max buckets are exact, and the fold feeds the aggregator in
        # SpanCmp order: bit-exact.  avg buckets are tree-reduced (1e-12);
        # diff subtracts two such values (cancellation)
        exact = ds == "max"
        fl = cancel_floor(b, 2) if agg == "diff" else 0.0
        check(engine, spec, b, exact, where="%s:%s" % (agg, ds), floor=fl)


@pytest.mark.parametrize("ds", DS)
def test_downsample_functions(engine, ds):
    for kind in ("float", "int", "mixed"):
        b = datasets.random_batch(23, n_series=30, n_groups=3, value_kind=kind,
                                  nan_frac=0.05 if kind == "float" else 0)
        for agg in ("sum", "min"):
            spec = _spec(agg, ds, interval="5m")
            # dev / diff buckets are bit-exact (dev: one Welford pass in
            # point order) and the fold feeds them in SpanCmp order
            exact = ds in ORDER_FREE or ds in ("dev", "diff") or (
                kind == "int" and ds != "mult")
            # diff buckets and integer data (-50..100) make mixed-sign sums:
            # 30 points per 5 m bucket x 10 series per group
            fl = (cancel_floor(b, 300) if (ds == "diff" or kind == "int")
                  else 0.0)
            check(engine, spec, b, exact, where="%s/%s/%s" % (ds, agg, kind),
                  floor=fl)


SEL_DS = ["median", "p50", "p75", "p95", "p99", "p999", "ep90r3", "ep50r7"]


@pytest.mark.parametrize("ds", SEL_DS)
def test_selection_downsampling(engine, ds):
    """median / percentile as the downsampling function: per-bucket
    selection (LDS sort for small buckets, wave radix select for large)."""
    for kind, nan in (("float", 0.1), ("int", 0.0), ("mixed", 0.0)):
        b = datasets.random_batch(27, n_series=24, n_groups=3, value_kind=kind,
                                  nan_frac=nan)
        for interval in ("1m", "1h"):  # 6 and 360 points per bucket
            for agg, fill in (("sum", "none"), ("max", "nan"), ("p90", "zero")):
                spec = _spec(agg, ds, fill, interval=interval)
                # selected buckets are exact and fed in order: bit-exact
                check(engine, spec, b, True,
                      where="%s/%s/%s/%s" % (ds, kind, interval, agg))
    b = datasets.random_batch(29, n_series=12, n_groups=2, counter=True)
    spec = _spec("sum", ds, rate=True, ro=RATES[1], interval="5m")
    check(engine, spec, b, True, where="%s/rate" % ds)
    d = core.DownsamplingSpecification("0all-" + ds)
    spec = core.make_spec(datasets.T0, datasets.T0 + 4 * 3600 * 1000,
                          core.Aggregators.get("max"), d,
                          datasets.T0 + 600000, datasets.T0 + 7200000)
    check(engine, spec, b, True, where="%s/all" % ds)


@pytest.mark.parametrize("fill", ["none", "nan", "zero", "null"])
@pytest.mark.parametrize("aligned", [True, False])
def test_fill_policies_and_window(engine, fill, aligned):
    b = datasets.random_batch(31, n_series=25, n_groups=4, nan_frac=0.02)
    start = datasets.T0 + (0 if aligned else 37000)
    end = datasets.T0 + 2 * 3600 * 1000 + (0 if aligned else 11000)
    for agg in ("sum", "avg", "count", "last", "mimmin"):
        spec = _spec(agg, "max", fill, start, end)
        check(engine, spec, b, True, where="%s/%s/%s" % (fill, agg, aligned))


@pytest.mark.parametrize("interp", list(core.Interpolation))
def test_interpolation_methods(engine, interp):
    b = datasets.random_batch(41, n_series=30, n_groups=3)
    for agg in ("sum", "max", "first"):
        spec = _spec(agg, "min", interp=interp, interval="10s")
        check(engine, spec, b, True, where="%s/%s" % (interp.name, agg))


RATES = [
    core.RateOptions(),
    core.RateOptions(True, 2**63 - 1, 0),
    core.RateOptions(True, 2**63 - 1, 50),
    core.RateOptions(True, 10**12, 0, True),
]


@pytest.mark.parametrize("ri", range(len(RATES)))
@pytest.mark.parametrize("fill", ["none", "nan", "zero"])
def test_rate(engine, ri, fill):
    b = datasets.random_batch(51 + ri, n_series=30, n_groups=3, counter=True)
    for agg, ds in (("sum", "max"), ("dev", "sum"), ("avg", "last"),
                    ("count", "min")):
        for aligned in (True, False):
            start = datasets.T0 + (0 if aligned else 61000)
            spec = _spec(agg, ds, fill, start=start, rate=True, ro=RATES[ri])
            # dev over a group of 10: one chain per bucket (bit-exact)
            check(engine, spec, b, True,
                  where="rate%d/%s/%s/%s" % (ri, fill, agg, aligned))


def test_run_all(engine):
    b = datasets.random_batch(61, n_series=20, n_groups=4)
    qs, qe = datasets.T0 + 600000, datasets.T0 + 7200000
    for agg in ("sum", "max", "count"):
        d = core.DownsamplingSpecification("0all-max")
        spec = core.make_spec(datasets.T0, datasets.T0 + 4 * 3600 * 1000,
                              core.Aggregators.get(agg), d, qs, qe)
        check(engine, spec, b, True, where="all/" + agg)


def test_big_groups_chunked(engine):
    """Groups larger than one 256-series chunk: chunk partials merged in
    order (exact for order-free aggregators, 1e-12 otherwise; dev reduces
    the 700 members in one chain per bucket: exact)."""
    b = datasets.random_batch(71, n_series=700, big_group=True,
                              span_ms=3600 * 1000, cadence_ms=30000)
    for agg in ("sum", "avg", "dev", "min", "count", "first", "last", "diff"):
        spec = _spec(agg, "max", end=datasets.T0 + 3600 * 1000)
        # chunk partials merge in order (1e-12); diff: cancellation
        fl = cancel_floor(b, 2) if agg == "diff" else 0.0
        check(engine, spec, b, agg in ORDER_FREE or agg == "dev",
              where="big/" + agg, floor=fl)


def test_huge_group_two_level_combine(engine):
    """One group of > 128 chunks (36k series): the ordered two-level chunk
    combine (k_combine_l1 + k_combine) — exact for order-free aggregators,
    1e-12 otherwise."""
    b = datasets.random_batch(73, n_series=36000, big_group=True,
                              span_ms=600 * 1000, cadence_ms=30000,
                              empty_frac=0.01)
    for agg in ("sum", "zimsum", "avg", "dev", "min", "mimmax", "count",
                "first", "last", "diff", "none"):
        spec = _spec(agg, "max", end=datasets.T0 + 600 * 1000)
        fl = cancel_floor(b, 2) if agg == "diff" else 0.0
        check(engine, spec, b, agg in ORDER_FREE, where="huge/" + agg,
              floor=fl)


@pytest.mark.parametrize("n_series,kind", [(45, "float"), (300, "float"),
                                           (5000, "float"), (5000, "int")])
def test_percentiles_large_groups(engine, n_series, kind):
    """median / percentiles over groups above the LDS-sort limit: per-segment
    select over transposed keys — direct gather below SS_CAP candidates,
    11-bit digit passes above it, ties from integer data (exact: selection
    + the reference's estimator arithmetic)."""
    b = datasets.random_batch(77, n_series=n_series, big_group=True,
                              span_ms=3600 * 1000, cadence_ms=30000,
                              nan_frac=0.05 if kind == "float" else 0.0,
                              value_kind=kind)
    for agg in ("median", "p50", "p75", "p99", "p999", "ep95r3", "ep50r7"):
        for fill in ("none", "nan"):
            spec = _spec(agg, "max", fill, end=datasets.T0 + 3600 * 1000)
            check(engine, spec, b, True, where="sel%d/%s/%s" % (
                n_series, agg, fill))


def test_percentiles_fill_several_large_groups(engine):
    """Fill-mode percentiles with every group large: the keys transpose
    applies the FillingDownsampler fill and counts the non-NaN keys per
    (bucket, 64-member tile), with group boundaries inside tiles and a group
    whose series are all empty (not kept: it emits nothing)."""
    import numpy as np
    from opentsdb_amd.batch import HostBatch
    b = datasets.random_batch(79, n_series=300, n_groups=3,
                              span_ms=3600 * 1000, cadence_ms=30000,
                              nan_frac=0.05, empty_frac=0.1)
    n_empty = 40
    offs = np.concatenate([b.offsets, np.full(n_empty, b.offsets[-1])])
    g_off = np.concatenate([b.group_offsets, [b.group_offsets[-1] + n_empty]])
    members = np.concatenate([b.group_members,
                              300 + np.arange(n_empty, dtype=np.int64)])
    b2 = HostBatch(offs.astype(np.int64), b.ts, b.val, b.is_float, None,
                   g_off.astype(np.int64), members.astype(np.int64))
    for agg in ("median", "p50", "p99", "p999", "ep95r3"):
        for fill in ("nan", "null", "zero"):
            spec = _spec(agg, "avg", fill, end=datasets.T0 + 3600 * 1000)
            check(engine, spec, b2, True, where="selfill/%s/%s" % (agg, fill))


@pytest.mark.parametrize("n_series,n_groups", [(150, 2), (333, 5)])
def test_percentiles_fill_keys_fold_windows(engine, n_series, n_groups):
    """Fill-mode percentiles with every group large over wide grids (6 h of
    1 m / 10 s buckets: 360 / 2,160 of them) — the keys transpose's fill and
    counts per (bucket, 64-member tile) with group boundaries inside tiles,
    series that start late or end early (the fill before / after them), NaN
    values, empty series (not kept): bit-exact with the oracle."""
    b = datasets.random_batch(83 + n_series, n_series=n_series,
                              n_groups=n_groups, span_ms=6 * 3600 * 1000,
                              cadence_ms=20000, nan_frac=0.03,
                              empty_frac=0.05)
    end = datasets.T0 + 6 * 3600 * 1000
    # order-free downsamplers: bit-exact; avg over 3 points a bucket: the
    # downsample's lane-tree sums, within 1e-12
    for agg, interval, ds in (("p99", "1m", "max"), ("median", "1m", "min"),
                              ("p50", "10s", "first"), ("ep95r3", "1m", "max"),
                              ("p99", "1m", "avg")):
        for fill in ("nan", "zero"):
            spec = _spec(agg, ds, fill, end=end, interval=interval)
            check(engine, spec, b, ds != "avg", where="kfold%d/%s/%s/%s/%s" % (
                n_series, agg, interval, ds, fill))


def test_got_infinity(engine):
    """AggregationIterator.doubleValue throws on +-Infinity
    (AggregationIterator.java:640-643)."""
    from opentsdb_amd.batch import HostBatch
    big = 1.5e308
    groups = [[[(datasets.T0 + 1000 * i, big, 1) for i in range(5)]] * 3]
    b = HostBatch.from_groups(groups)
    spec = _spec("sum", "max", end=datasets.T0 + 60000)
    run_both(engine, spec, b)
    with pytest.raises(core.IllegalStateException):
        engine.run(spec, b)


def test_none_more_than_one_value(engine):
    """`none` fed by more than one span -> IllegalDataException
    (Aggregators.java:446-449)."""
    b = datasets.random_batch(81, n_series=6, n_groups=2, outside=False,
                              empty_frac=0)
    spec = _spec("none", "avg")
    run_both(engine, spec, b)
    with pytest.raises(core.IllegalDataException):
        engine.run(spec, b)


def test_empty_and_degenerate(engine):
    from opentsdb_amd.batch import HostBatch
    # no series at all / empty spans only / window before all data
    b = HostBatch.from_groups([[[], []], []])
    got, ref = run_both(engine, _spec("sum", "avg"), b)
    compare(got, ref, True, where="empty")
    b = datasets.random_batch(91, n_series=10, n_groups=2)
    spec = _spec("sum", "avg", start=datasets.T0 - 10 * 3600 * 1000,
                 end=datasets.T0 - 9 * 3600 * 1000)
    check(engine, spec, b, True, where="before")


# ------------------------------------------------- raw (no downsampling)
def _raw(agg, start=None, end=None, rate=False, ro=None, interp=None):
    s0 = datasets.T0 if start is None else start
    e0 = datasets.T0 + 3 * 3600 * 1000 if end is None else end
    return core.make_spec(s0, e0, core.Aggregators.get(agg), None, s0, e0,
                          rate, ro, interp)


RAW_AGGS = AGGS + ["none"]


@pytest.mark.parametrize("kind", ["float", "int", "mixed", "nan"])
@pytest.mark.parametrize("agg", RAW_AGGS)
def test_raw_group_by(engine, agg, kind):
    """AggregationIterator over the spans' own points: union emission,
    contribution window, isInteger over current+next slots, runLong with
    Java long arithmetic — sequential in span order, so bit-exact."""
    b = datasets.random_batch(101, n_series=24, n_groups=4,
                              value_kind="float" if kind == "nan" else kind,
                              nan_frac=0.05 if kind == "nan" else 0.0,
                              cadence_ms=37000)
    check(engine, _raw(agg), b, True, where="raw/%s/%s" % (agg, kind))


@pytest.mark.parametrize("interp", list(core.Interpolation))
def test_raw_interpolation(engine, interp):
    for kind in ("float", "int"):
        b = datasets.random_batch(103, n_series=20, n_groups=3,
                                  value_kind=kind, cadence_ms=23000)
        for agg in ("sum", "max", "avg"):
            check(engine, _raw(agg, interp=interp), b, True,
                  where="raw/%s/%s/%s" % (interp.name, agg, kind))


@pytest.mark.parametrize("ri", range(len(RATES)))
def test_raw_rate(engine, ri):
    b = datasets.random_batch(107 + ri, n_series=20, n_groups=3, counter=True,
                              cadence_ms=31000)
    for agg in ("sum", "avg", "max", "count", "p95", "median"):
        for start in (datasets.T0, datasets.T0 + 61000):
            spec = _raw(agg, start=start, rate=True, ro=RATES[ri])
            check(engine, spec, b, True, where="rawrate%d/%s" % (ri, agg))


def test_raw_windows_and_big_groups(engine):
    """Unaligned / narrow windows, spans outside the window, and groups of
    hundreds of spans (the selection path with > 64 contributions)."""
    b = datasets.random_batch(109, n_series=12, n_groups=3, cadence_ms=13000)
    for s, e in ((datasets.T0 + 12345, datasets.T0 + 2 * 3600 * 1000 + 999),
                 (datasets.T0 + 3600 * 1000, datasets.T0 + 3600 * 1000),
                 (datasets.T0 - 10 * 3600 * 1000, datasets.T0 - 9 * 3600 * 1000)):
        for agg in ("sum", "last", "p99", "dev"):
            check(engine, _raw(agg, s, e), b, True, where="rawwin/%s" % agg)
    b = datasets.random_batch(111, n_series=300, big_group=True,
                              span_ms=1800 * 1000, cadence_ms=60000,
                              value_kind="mixed")
    for agg in ("sum", "avg", "median", "p50", "p999", "ep95r3", "ep75r7",
                "count", "mimmax"):
        check(engine, _raw(agg, end=datasets.T0 + 1800 * 1000), b, True,
              where="rawbig/" + agg)


def _dup_batch(seed, kind, n_series=16, n_groups=3):
    """random_batch with repeated timestamps: runs of 2-4 copies of a point
    (new values) inside spans, at span ends and at the window's edges."""
    from opentsdb_amd.batch import HostBatch
    b = datasets.random_batch(seed, n_series=n_series, n_groups=n_groups,
                              value_kind=kind, cadence_ms=37000)
    rng = np.random.default_rng(seed)
    offs, ts, val, isf = [0], [], [], []
    for s in range(b.n_series):
        t = b.ts[b.offsets[s]:b.offsets[s + 1]]
        v = b.val[b.offsets[s]:b.offsets[s + 1]]
        f = b.is_float[b.offsets[s]:b.offsets[s + 1]]
        reps = np.ones(len(t), np.int64)
        if len(t):
            pick = rng.random(len(t)) < 0.08
            if rng.random() < 0.5:
                pick[-1] = True  # copies of the span's last point
            reps[pick] = rng.integers(2, 5, int(pick.sum()))
        idx = np.repeat(np.arange(len(t)), reps)
        t2, f2 = t[idx], f[idx]
        v2 = v[idx].copy()
        first = np.r_[True, idx[1:] != idx[:-1]] if len(idx) else idx
        newv = (rng.random(len(idx)) * 100.0).view(np.int64) if kind != "int" \
            else rng.integers(-50, 100, len(idx)).astype(np.int64)
        v2[~first] = np.where(f2[~first] == 1, newv[~first],
                              rng.integers(0, 100, len(idx))[~first])
        ts.append(t2)
        val.append(v2)
        isf.append(f2)
        offs.append(offs[-1] + len(t2))
    return HostBatch(np.array(offs, np.int64), np.concatenate(ts),
                     np.concatenate(val), np.concatenate(isf), None,
                     b.group_offsets, b.group_members)


@pytest.mark.parametrize("kind", ["float", "int", "mixed"])
def test_raw_repeated_timestamps(engine, kind):
    """A span holding a timestamp k times: the iterator emits it k times,
    the m-th emission taking that span's m-th copy while the other spans
    hold theirs (or interpolate), and a span whose last point is repeated
    expires after its last copy (AggregationIterator.java:514-588) —
    against the oracle's line-by-line iterator, bit-exact."""
    b = _dup_batch(113, kind)
    assert (np.diff(b.ts)[np.diff(b.ts) == 0]).size > 0
    for agg in ("sum", "avg", "max", "dev", "count", "first", "last", "diff",
                "mimmin", "p90", "median"):
        for interp in (None, core.Interpolation.PREV):
            spec = _raw(agg, start=datasets.T0 + 37000 * 3, interp=interp)
            check(engine, spec, b, True,
                  where="rawdup/%s/%s/%s" % (kind, agg, interp))
    # downsampled: repeated timestamps fall into one bucket, in order
    check(engine, _spec("sum", "dev", interval="5m"), b, True,
          where="dsdup/%s" % kind)


# ------------------------------------------------------------ generator
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_device_generator_matches_oracle(engine, kind):
    import torch
    from opentsdb_amd import abi, workload
    g = abi.GenSpec(42, 1356998400000, 86400000, 10000, kind, 0)
    db = workload.generate_device(engine, g, series0=1000, n_series=64,
                                  group_size=10)
    offs = db.offsets.cpu().numpy()
    ts = db.ts.cpu().numpy()
    val = db.val.cpu().numpy()
    for i in range(64):
        t, v = pyoracle.gen_series(g, 1000 + i)
        assert np.array_equal(ts[offs[i]:offs[i + 1]], t), i
        assert np.array_equal(val[offs[i]:offs[i + 1]], v), i


def test_device_path_matches_host_path(engine):
    """otsdb_agg_run_device on HBM-resident tensors == otsdb_agg_run."""
    import torch
    from opentsdb_amd import abi, workload
    from opentsdb_amd.engine import DeviceResult, run_device
    g = abi.GenSpec(42, 1356998400000, 86400000, 10000, 0, 0)
    db = workload.generate_device(engine, g, series0=0, n_series=200,
                                  group_size=10)
    spec = workload.query_spec("C1", 0)
    sz = engine.plan(spec, db)
    res = DeviceResult(torch, db.n_groups, int(sz.max_out_points), "cuda")
    run_device(engine, spec, db, res)
    torch.cuda.synchronize()
    hb = pyoracle.gen_batch(g, 0, 200, lambda s: s // 10)
    ref = pyoracle.group_by(spec, hb)
    host = engine.run(spec, hb)
    offs = res.offsets.cpu().numpy()
    from opentsdb_amd.engine import DataPoints
    got = [DataPoints(res.ts[offs[i]:offs[i + 1]].cpu().numpy(),
                      res.val[offs[i]:offs[i + 1]].cpu().numpy(),
                      res.is_int[offs[i]:offs[i + 1]].cpu().numpy())
           for i in range(db.n_groups)]
    compare(got, ref, False, where="device")
    compare(host, ref, False, where="host")
    for a, h in zip(got, host):
        assert np.array_equal(a.bits, h.bits)


@pytest.mark.parametrize("ri", range(len(RATES)))
def test_rate_long_gaps(engine, ri):
    """Rate rows whose 512-point steps straddle gaps wider than the fused
    kernel's 1,024-bucket ring (the series is handed back to k_bucketize +
    k_transform) next to series that stay fused; 2 days of 1 m buckets."""
    from opentsdb_amd.batch import HostBatch
    rng = np.random.default_rng(70 + ri)
    T0 = datasets.T0
    offs, tss, vals = [0], [], []
    for s in range(24):
        parts = []
        t = T0 + int(rng.integers(0, 10000))
        for blk in range(int(rng.integers(1, 5))):
            n = int(rng.integers(5, 200))
            parts.append(t + 10000 * np.arange(n, dtype=np.int64))
            # gaps from minutes to a day: > 1,024 buckets for some
            t = int(parts[-1][-1]) + int(rng.choice([60000, 3600000, 20 * 3600000,
                                                     26 * 3600000]))
        ts = np.concatenate(parts)
        ts = ts[ts < T0 + 2 * 86400000]
        v = np.cumsum(rng.integers(0, 1000, len(ts))).astype(np.int64)
        v[rng.random(len(ts)) < 0.03] = 0  # counter resets
        tss.append(ts)
        vals.append(v)
        offs.append(offs[-1] + len(ts))
    ts, val = np.concatenate(tss), np.concatenate(vals)
    hb = HostBatch(np.array(offs, np.int64), ts, val,
                   np.zeros(len(ts), np.uint8), None,
                   np.array([0, 8, 16, 24], np.int64),
                   np.arange(24, dtype=np.int64))
    for agg, ds in (("sum", "sum"), ("max", "last"), ("dev", "max")):
        spec = _spec(agg, ds, start=T0, end=T0 + 2 * 86400000 - 1000,
                     rate=True, ro=RATES[ri])
        check(engine, spec, hb, agg == "max",
              where="rategap%d/%s/%s" % (ri, agg, ds))


# ------------------------------------------------ fold order / determinism
def _cancel_batch(n_series, reps=180, cadence_ms=60000):
    """n_series series on a one-point-per-minute grid (1m buckets hold one
    point: the downsample is exact) whose values cancel: 1e17, 1, -1e17,
    1, 1e17, ... — a sum's result depends on the order of the adds
    (1e17 + 1 == 1e17)."""
    from opentsdb_amd.batch import HostBatch, groups_from_ids
    pattern = np.array([1e17, 1.0, -1e17, 1.0])
    t = datasets.T0 + cadence_ms * np.arange(reps, dtype=np.int64)
    ts = np.tile(t, n_series)
    v = np.repeat(pattern[np.arange(n_series) % 4], reps)
    offs = np.arange(n_series + 1, dtype=np.int64) * reps
    g_off, members = groups_from_ids(np.zeros(n_series, np.int64), 1)
    return HostBatch(offs, ts, v.view(np.int64), np.ones(len(ts), np.uint8),
                     None, g_off, members)


@pytest.mark.parametrize("agg", ["sum", "zimsum", "avg", "dev"])
def test_fold_order_cancellation(engine, agg):
    """The ordered group fold feeds the aggregator in SpanCmp order
    (Aggregators.java:246-258 Sum.runDouble adds in span order): on values
    whose sum depends on the order of the adds, a group inside one fold
    tile is bit-exact with the reference's order, and every group —
    several tiles merged in order included — gives bit-identical results
    run after run."""
    spec = _spec(agg, "avg")
    one_tile = _cancel_batch(7)
    check(engine, spec, one_tile, exact=True, where="cancel/%s/1tile" % agg)
    many = _cancel_batch(203)  # six 32-member tiles + a partial one
    if agg == "dev":  # one 256-member tile: the reference's order
        check(engine, spec, many, exact=True, where="cancel/dev/203")
    first = engine.run(spec, many)
    for _ in range(2):
        again = engine.run(spec, many)
        for a, b in zip(first, again):
            assert np.array_equal(np.asarray(a.ts), np.asarray(b.ts))
            assert np.array_equal(np.asarray(a.bits), np.asarray(b.bits)), (
                "%s: run-to-run difference" % agg)


def _outage_batch(reset_after=False):
    """Two counter series of one group: A reports every 10 s; B's outage
    covers the whole query window, with points before it and after its end
    (inside the scan range).  reset_after: B's counter resets right after
    the window (dropResets then drops the first rate past it)."""
    from opentsdb_amd.batch import HostBatch, groups_from_ids
    t = datasets.T0 + 10000 * np.arange(6 * 360, dtype=np.int64)  # 6 h
    a = 1000 + 37 * np.arange(len(t), dtype=np.int64)
    keep = (t < datasets.T0 + 3600000) | (t >= datasets.T0 + 4 * 3600000)
    tb = t[keep]
    vb = 5_000_000 + 11 * np.arange(len(tb), dtype=np.int64)
    if reset_after:
        after = tb >= datasets.T0 + 4 * 3600000
        vb[after] = 3 * np.arange(after.sum(), dtype=np.int64)
    ts = np.concatenate([t, tb])
    val = np.concatenate([a, vb])
    offs = np.array([0, len(t), len(t) + len(tb)], np.int64)
    g_off, members = groups_from_ids(np.zeros(2, np.int64), 1)
    return HostBatch(offs, ts, val, np.zeros(len(ts), np.uint8), None, g_off,
                     members)


@pytest.mark.parametrize("ds", ["1m-sum", "1m-p90", "1m-median", "2m-avg",
                                "30s-p50"])
@pytest.mark.parametrize("drop", [False, True])
@pytest.mark.parametrize("agg", ["min", "sum", "max"])
def test_rate_series_whose_rates_all_lie_past_the_window(engine, agg, drop,
                                                         ds):
    """Rate mode pre-consumes each span's first (junk) rate and keeps the
    span contributing while it has a second (AggregationIterator.java:
    448-459): a series whose outage covers the whole window still
    contributes its junk rate, held over the window, when its rates lie
    past the window's end (found by the random sweep, seed 48)."""
    b = _outage_batch(reset_after=drop)
    t0, t1 = datasets.T0 + 3600000 + 120000, datasets.T0 + 3 * 3600000
    ro = core.RateOptions(True, core.LONG_MAX, 0, drop)
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification(ds), t0, t1, True, ro)
    check(engine, spec, b, exact=agg in ("min", "max"),
          where="outage/%s/%s/drop=%s" % (agg, ds, drop))


def _empty_member_batch(after):
    """A reports every 10 s over 6 h; B is kept (its points straddle the
    window, or end inside the scan range when after=False) but has none
    inside the window, and its first index past the window is odd (the fold
    steps from an even base).  B is the batch's last series."""
    from opentsdb_amd.batch import HostBatch, groups_from_ids
    t = datasets.T0 + 10000 * np.arange(6 * 360, dtype=np.int64)
    a = (t // 1000) % 97
    # B's last point lies in [start, first bucket): kept, nothing in the grid
    tb = (datasets.T0 + 3600000 + 127000
          - 10000 * np.arange(100, -1, -1, dtype=np.int64))
    if after:
        tb = np.concatenate([tb, datasets.T0 + 4 * 3600000
                             + 10000 * np.arange(40, dtype=np.int64)])
    assert (len(t) + 101) % 2 == 1
    vb = np.arange(len(tb), dtype=np.int64) % 13
    ts = np.concatenate([t, tb])
    val = np.concatenate([a, vb]).astype(np.int64)
    offs = np.array([0, len(t), len(t) + len(tb)], np.int64)
    g_off, members = groups_from_ids(np.zeros(2, np.int64), 1)
    return HostBatch(offs, ts, val, np.zeros(len(ts), np.uint8), None, g_off,
                     members)


@pytest.mark.parametrize("after", [False, True])
@pytest.mark.parametrize("fill", ["zero", "null", "nan", "none"])
@pytest.mark.parametrize("ds", ["1m-sum", "30s-min", "2m-count"])
def test_fold_member_without_window_points(engine, ds, fill, after):
    """A kept member with no point inside the window (SpanGroup.add keeps
    it; FillingDownsampler still fills its every bucket) must stream
    nothing: found by the random sweep (seeds 850, 865, 1103), where such a
    member at an odd point index pushed fills past the window's LDS states.
    The 30s grid (236 buckets) runs as two narrowed fold windows."""
    b = _empty_member_batch(after)
    t0 = datasets.T0 + 3600000 + 125000
    t1 = datasets.T0 + 3 * 3600000
    spec = _spec("sum", ds.split("-")[1], fill, t0, t1,
                 interval=ds.split("-")[0])
    check(engine, spec, b, exact=False,
          where="empty-member/%s/%s/after=%s" % (ds, fill, after))
    # B alone: its group is fill values only (or absent)
    from opentsdb_amd.batch import HostBatch
    o = int(b.offsets[1])
    bb = HostBatch(np.array([0, len(b.ts) - o], np.int64), b.ts[o:], b.val[o:],
                   b.is_float[o:], None, np.array([0, 1], np.int64),
                   np.array([0], np.int64))
    check(engine, spec, bb, exact=True,
          where="empty-member-alone/%s/%s/after=%s" % (ds, fill, after))
