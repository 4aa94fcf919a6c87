"""Calendar downsampling on the host and in the oracle (CPU only): the
supported / unsupported boundary of the edge table and an independent
bucketing cross-check of the oracle's calendar Downsampler."""
import numpy as np
import pytest

from opentsdb_amd import core, jcalendar
from oracle import pyoracle
from tests import datasets

DAY = 86400000
T_SPRING = 1362614400000  # 2013-03-07 00:00 UTC, before the US DST start


def _spec(agg, ds, tz, start, end, batch=None):
    d = core.DownsamplingSpecification(ds)
    if tz:
        d.setTimezone(tz)
    cover = int(batch.ts.max()) if batch is not None else None
    return core.make_spec(start, end, core.Aggregators.get(agg), d, start,
                          end, cal_cover_ms=cover)


def test_grid_dependent_specs_carry_anchors():
    """'7mc' re-anchors at every local midnight and 1440 % 7 != 0, '2wc'
    at every Sunday, '6hc' steps 6 hours from local midnight across the
    23-hour DST day: the grid depends on where a series starts, so the spec
    carries per-anchor chains (otsdb_query_spec.cal_anchors) instead of one
    edge table."""
    for ds, tz, days in (("7mc-sum", None, 3), ("2wc-sum", None, 30),
                         ("6hc-sum", "America/Denver", 6)):
        with pytest.raises(core.UnsupportedOperationException):
            n, unit = core.DownsamplingSpecification(ds).calendar_interval()
            jcalendar.calendar_edges(T_SPRING, T_SPRING + days * DAY, n, unit,
                                     tz)
        s = _spec("sum", ds, tz, T_SPRING, T_SPRING + days * DAY)
        assert s.n_cal_anchors > 0
    # whole days stay one table
    s = _spec("sum", "1dc-sum", "America/Denver", T_SPRING, T_SPRING + 6 * DAY)
    assert s.n_cal_anchors == 0
    e = np.ctypeslib.as_array(s._cal_edges_ref)
    d = np.diff(e) // 3600000
    assert sorted(set(d.tolist())) == [23, 24]  # the spring-forward day


@pytest.mark.parametrize("n,unit,tz,days", [
    (7, "m", None, 3), (2, "w", None, 40), (6, "h", "America/Denver", 6),
    (13, "s", "Asia/Kabul", 1), (5, "h", "Pacific/Chatham", 4),
    (2, "d", "America/Denver", 400), (3, "n", "America/Denver", 400)])
def test_anchor_tables_match_previous_interval(n, unit, tz, days):
    """The largest anchor <= t is DateTime.previousInterval(t) for every t of
    the window, and its chain continues the way the Downsampler steps it
    (Downsampler.java:330-345, :383-397)."""
    start = T_SPRING + 1234567
    end = start + days * DAY
    tables = jcalendar.calendar_anchor_tables(start, end, n, unit, tz)
    edges = tables[0]
    rng = np.random.default_rng(n * 1000 + days)
    ts = np.concatenate([rng.integers(start, end, 300),
                         np.asarray(tables[1][:50]) + 0,
                         np.asarray(tables[1][:50]) - 1])
    for t in ts.tolist():
        if t < start:
            continue
        k = jcalendar.anchored_previous_interval(tables, t)
        a = jcalendar.previous_interval(t, n, unit, tz)
        assert edges[k] == a, (t, edges[k], a)
        # the chain from the anchor is Calendar.add-stepped past t
        c = a
        for j in range(1, 4):
            c = jcalendar.step(c, n, unit, jcalendar.get_timezone(tz))
            if edges[k + j] == jcalendar.SENTINEL:
                break
            assert edges[k + j] == c


def test_dst_day_lengths_fall_back():
    e = jcalendar.calendar_edges(1383177600000, 1383177600000 + 6 * DAY, 1,
                                 "d", "America/Denver")
    assert 25 in (np.diff(e) // 3600000).tolist()


@pytest.mark.parametrize("ds,tz", [("1dc-sum", "America/Denver"),
                                   ("1hc-sum", "Asia/Kabul"),
                                   ("1wc-sum", "Pacific/Fiji")])
def test_oracle_calendar_vs_naive_bucketing(ds, tz):
    """zimsum over calendar buckets with NONE fill and no gaps inside a
    bucket equals a plain per-bucket sum over the edge table."""
    b = datasets.random_batch(3, n_series=6, n_groups=1, span_ms=20 * DAY,
                              cadence_ms=3600000, outside=False,
                              empty_frac=0.0, t0=T_SPRING, big_group=True)
    start, end = T_SPRING, T_SPRING + 19 * DAY
    spec = _spec("zimsum", ds, tz, start, end, b)
    got = pyoracle.group_by(spec, b)[0]
    edges = np.asarray(spec._cal_edges_ref)
    seek = edges[np.searchsorted(edges, start)]
    vals = b.val.view(np.float64)
    sums = {}
    for s in range(len(b.offsets) - 1):
        per = {}
        for i in range(b.offsets[s], b.offsets[s + 1]):
            t = int(b.ts[i])
            if t < seek:
                continue
            # a bucket is emitted iff its timestamp is <= end; it holds all
            # of its points, also those past end (Downsampler buckets)
            k = int(np.searchsorted(edges, t, side="right") - 1)
            if edges[k] > end:
                continue
            per.setdefault(int(edges[k]), []).append(vals[i])
        for k, v in per.items():
            # sum downsampler: sequential double sum in time order
            acc = 0.0
            for x in v:
                acc += x
            sums[k] = sums.get(k, 0.0) + acc
    exp_ts = sorted(sums)
    assert got["ts"].tolist() == exp_ts
    np.testing.assert_allclose(got["bits"].view(np.float64),
                               [sums[t] for t in exp_ts], rtol=1e-12)


@pytest.mark.parametrize("ds,tz,days,cad", [("7mc-sum", None, 3, 60000),
                                            ("6hc-sum", "America/Denver", 6,
                                             600000),
                                            ("2wc-sum", None, 45, 3600000)])
def test_oracle_per_series_grids_vs_naive(ds, tz, days, cad):
    """zimsum over per-series calendar grids (each series anchored at
    previousInterval(its first point after the seek), jcalendar's
    bucket_edges_for_series) equals, at each union timestamp, the sum of the
    series' own buckets starting there (ZIM: a series without a bucket
    there adds nothing)."""
    b = datasets.random_batch(11, n_series=12, n_groups=1,
                              span_ms=days * DAY, cadence_ms=cad,
                              outside=False, empty_frac=0.0, t0=T_SPRING,
                              big_group=True)
    start, end = T_SPRING + 3600000, T_SPRING + (days - 1) * DAY
    spec = _spec("zimsum", ds, tz, start, end, b)
    assert spec.n_cal_anchors > 0
    got = pyoracle.group_by(spec, b)[0]
    n, unit = core.DownsamplingSpecification(ds).calendar_interval()
    tzz = jcalendar.get_timezone(tz)
    a0 = jcalendar.previous_interval(start, n, unit, tzz)
    seek = a0 if a0 >= start else jcalendar.step(a0, n, unit, tzz)
    vals = b.val.view(np.float64)
    sums = {}
    for s in range(len(b.offsets) - 1):
        t = b.ts[b.offsets[s]:b.offsets[s + 1]]
        v = vals[b.offsets[s]:b.offsets[s + 1]]
        keep = t >= seek
        t, v = t[keep], v[keep]
        if not len(t):
            continue
        edges = jcalendar.bucket_edges_for_series(int(t[0]), int(t[-1]), n,
                                                  unit, tzz)
        per = {}
        for x, y in zip(t.tolist(), v.tolist()):
            k = jcalendar.edge_index(edges, x)
            if edges[k] > end:
                continue
            per.setdefault(edges[k], []).append(y)
        for k, ys in per.items():
            acc = 0.0
            for y in ys:
                acc += y
            sums[k] = sums.get(k, 0.0) + acc
    exp_ts = sorted(sums)
    assert got["ts"].tolist() == exp_ts
    np.testing.assert_allclose(got["bits"].view(np.float64),
                               [sums[t] for t in exp_ts], rtol=1e-12)
