"""Calendar downsampling ("<n><unit>c-<agg>", timezones) on the GPU against
the oracle: the host computes the query's bucket-edge table
(opentsdb_amd/jcalendar.py, pinned by TestDateTime/TestDownsampler KATs in
tests/test_oracle_kat.py), the engine buckets every series on it.

Windows cross DST transitions (America/Denver 2013-03-10, 2013-11-03),
odd offsets (Asia/Kabul +4:30, Pacific/Chatham +12:45/+13:45) and month
boundaries.  Bar as in test_gpu_parity.py: bit-exact for order-free
functions, 1e-12 relative otherwise.
"""
import pytest

from opentsdb_amd import core
from tests import datasets
from tests.test_gpu_parity import check, engine  # noqa: F401

pytestmark = pytest.mark.gpu

DAY = 86400000
# 2013-03-07 00:00 UTC: the window below spans the US spring-forward
T_SPRING = 1362614400000
# 2013-10-31 00:00 UTC: spans the US fall-back
T_FALL = 1383177600000


def _cal_spec(agg, ds, tz, start, end, rate=False, ro=None, batch=None):
    d = core.DownsamplingSpecification(ds)
    if tz:
        d.setTimezone(tz)
    cover = int(batch.ts.max()) if batch is not None and len(batch.ts) else None
    return core.make_spec(start, end, core.Aggregators.get(agg), d, start,
                          end, rate, ro, cal_cover_ms=cover)


CASES = [
    # (downsampler, tz, t0, days, cadence)
    ("1dc-sum", "America/Denver", T_SPRING, 7, 600000),
    ("1dc-avg", "America/Denver", T_FALL, 7, 600000),
    ("1hc-max", "Asia/Kabul", T_SPRING, 3, 120000),
    ("4hc-min", "Asia/Kabul", T_SPRING, 3, 120000),
    ("30mc-sum", "Pacific/Chatham", T_SPRING, 2, 60000),
    ("1wc-sum", None, T_SPRING, 30, 3600000),
    ("1wc-count", "Pacific/Fiji", T_SPRING, 30, 3600000),
    ("1nc-avg", "America/Denver", T_SPRING, 100, 3600000),
    ("1dc-sum-nan", "America/Denver", T_SPRING, 7, 600000),
    ("1dc-sum-zero", "America/Denver", T_FALL, 7, 600000),
    ("6hc-last", "America/Denver", T_SPRING, 4, 300000),
    # grids anchored at each series' first point (otsdb_query_spec.
    # cal_anchors): union of the series' own bucket starts
    ("7mc-sum", None, T_SPRING, 3, 60000),
    ("7mc-avg", "America/Denver", T_SPRING + 2 * DAY, 3, 45000),
    ("2wc-max", None, T_SPRING, 45, 3600000),
    ("6hc-avg", "America/Denver", T_SPRING, 5, 300000),
    ("6hc-dev", "America/Denver", T_FALL, 5, 300000),
    ("13mc-p90", "Asia/Kabul", T_SPRING, 2, 60000),
]


@pytest.mark.parametrize("ds,tz,t0,days,cad", CASES,
                         ids=["%s@%s" % (c[0], c[1]) for c in CASES])
@pytest.mark.parametrize("agg", ["sum", "zimsum", "max", "count", "p90"])
def test_calendar_group_by(engine, ds, tz, t0, days, cad, agg):  # noqa: F811
    b = datasets.random_batch(97, n_series=24, n_groups=3,
                              span_ms=days * DAY, cadence_ms=cad, t0=t0)
    start, end = t0 + 3600000, t0 + (days - 1) * DAY
    try:
        spec = _cal_spec(agg, ds, tz, start, end, batch=b)
    except core.UnsupportedOperationException:
        pytest.skip("grid depends on the series' first point")
    fn = ds.split("-")[1]
    exact = fn in ("min", "max", "count", "last") and agg in (
        "max", "count", "p90")
    check(engine, spec, b, exact, where="%s/%s/%s" % (ds, tz, agg))


@pytest.mark.parametrize("ds,tz", [("1hc-sum", "Asia/Kabul"),
                                   ("1dc-sum-zero", "America/Denver"),
                                   ("7mc-sum", None),
                                   ("6hc-max", "America/Denver")])
def test_calendar_rate(engine, ds, tz):  # noqa: F811
    b = datasets.random_batch(5, n_series=20, n_groups=2, span_ms=5 * DAY,
                              cadence_ms=300000, counter=True, t0=T_SPRING)
    ro = core.RateOptions(True, core.LONG_MAX, 1000000)
    spec = _cal_spec("sum", ds, tz, T_SPRING, T_SPRING + 4 * DAY, True, ro,
                     batch=b)
    check(engine, spec, b, False, where=ds)


FILL_CASES = [
    # FillingDownsampler over grids anchored at each series' first point
    ("7mc-avg-nan", None, T_SPRING, 3, 60000),
    ("7mc-sum-zero", "America/Denver", T_SPRING + 2 * DAY, 3, 45000),
    ("2wc-sum-zero", None, T_SPRING, 45, 3600000),
    ("6hc-max-null", "America/Denver", T_SPRING, 5, 300000),
    ("6hc-dev-nan", "America/Denver", T_FALL, 5, 300000),
    ("13mc-count-zero", "Asia/Kabul", T_SPRING, 2, 60000),
]


@pytest.mark.parametrize("ds,tz,t0,days,cad", FILL_CASES,
                         ids=["%s@%s" % (c[0], c[1]) for c in FILL_CASES])
@pytest.mark.parametrize("agg", ["sum", "max", "count", "avg", "p90"])
def test_per_series_grids_with_fill(engine, ds, tz, t0, days, cad, agg):  # noqa: F811
    """FillingDownsampler over per-series grids: its own grid is anchored at
    previousInterval(start) (FillingDownsampler.java:113-135), each series'
    buckets at previousInterval(its first point); a series bucket is emitted
    only where its start is on the filling grid, every other expected
    timestamp is filled (:175-272).  Windows across DST changes, series that
    start late (their own anchors differ from the filling grid's)."""
    b = datasets.random_batch(197, n_series=24, n_groups=3,
                              span_ms=days * DAY, cadence_ms=cad, t0=t0)
    for start, end in ((t0 + 3600000, t0 + (days - 1) * DAY),
                       (t0 + 3600000 + 123000, t0 + (days - 1) * DAY - 7000)):
        spec = _cal_spec(agg, ds, tz, start, end, batch=b)
        # (6hc across DST: per-series anchors or one table, as the window
        # decides; both take the filling pipeline)
        assert spec.n_cal_anchors > 0 or ds.startswith("6hc")
        fn = ds.split("-")[1]
        exact = fn in ("max", "count", "dev") and agg in ("max", "count",
                                                          "p90")
        check(engine, spec, b, exact, where="%s/%s/%s" % (ds, tz, agg))


def test_per_series_grids_with_fill_rate(engine):  # noqa: F811
    b = datasets.random_batch(5, n_series=20, n_groups=2, span_ms=5 * DAY,
                              cadence_ms=300000, counter=True, t0=T_SPRING)
    ro = core.RateOptions(True, core.LONG_MAX, 1000000)
    for ds in ("7mc-sum-nan", "6hc-max-zero"):
        spec = _cal_spec("sum", ds, "America/Denver", T_SPRING + 3600000,
                         T_SPRING + 4 * DAY, True, ro, batch=b)
        check(engine, spec, b, False, where="rate/" + ds)


def test_per_series_grids_points_past_the_chains(engine):  # noqa: F811
    """Points far past the window (past every chain's last edge, the tables
    built without cal_cover_ms): a non-rate query reads only the first bucket
    past the window, so the engine runs it — and gives the result the oracle
    gives with tables that cover every point (java.util.Calendar has no
    end); a series whose first point past the window lies beyond its chain
    still needs the Java path (E_UNSUPPORTED)."""
    from oracle import pyoracle
    from tests.test_gpu_parity import compare
    import numpy as np
    from opentsdb_amd.batch import HostBatch
    from opentsdb_amd.batch import groups_from_ids
    rng = np.random.default_rng(17)
    n_series, n = 12, 2 * DAY // 60000
    # every series reports each minute (a phase of its own) for two days
    ts = np.concatenate([T_SPRING + int(rng.integers(0, 60000)) +
                         60000 * np.arange(n, dtype=np.int64)
                         for _ in range(n_series)])
    vals = (rng.random(len(ts)) * 100.0).view(np.int64)
    g_off, members = groups_from_ids(np.arange(n_series) % 2, 2)
    b = HostBatch(np.arange(n_series + 1, dtype=np.int64) * n, ts, vals,
                  np.ones(len(ts), np.uint8), None, g_off, members)
    start, end = T_SPRING + 3600000, T_SPRING + DAY
    for ds in ("7mc-avg", "7mc-avg-nan"):
        d = core.DownsamplingSpecification(ds)
        spec = core.make_spec(start, end, core.Aggregators.get("sum"), d,
                              start, end)
        assert spec.n_cal_anchors > 0
        full = _cal_spec("sum", ds, None, start, end, batch=b)
        compare(engine.run(spec, b), pyoracle.group_by(full, b), False,
                where="far/" + ds)
    # one series with nothing between the window and a point 1 day later
    ts, val = [], []
    offs = [0]
    for s in range(b.n_series):
        t = b.ts[b.offsets[s]:b.offsets[s + 1]]
        v = b.val[b.offsets[s]:b.offsets[s + 1]]
        if s == 0:
            keep = (t <= end)
            t = np.concatenate([t[keep], [end + DAY]])
            v = np.concatenate([v[keep], v[:1]])
        ts.append(t)
        val.append(v)
        offs.append(offs[-1] + len(t))
    b2 = HostBatch(np.array(offs, np.int64), np.concatenate(ts),
                   np.concatenate(val), np.ones(offs[-1], np.uint8), None,
                   b.group_offsets, b.group_members)
    d = core.DownsamplingSpecification("7mc-avg")
    spec = core.make_spec(start, end, core.Aggregators.get("sum"), d, start,
                          end)
    with pytest.raises(core.UnsupportedOperationException):
        engine.run(spec, b2)


@pytest.mark.parametrize("ds", ["7mc-avg", "7mc-avg-nan"])
def test_per_series_grids_from_cells(engine, ds):  # noqa: F811
    """The same per-series grids from compacted cells
    (otsdb_agg_run_cells_device: decoded, then the anchored pipeline)."""
    import numpy as np
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult
    from oracle import pyoracle
    from tests.test_gpu_decode import _device_batch, _result_points
    from tests.test_gpu_parity import compare
    hb = datasets.random_batch(13, n_series=16, n_groups=2, span_ms=3 * DAY,
                               cadence_ms=60000, t0=T_SPRING)
    hb.ts[:] = hb.ts - hb.ts % 1000
    hb.is_float = np.ones(len(hb.ts), np.uint8)
    db = _device_batch(hb, "float")
    cells_d = workload.encode_cells_device(engine, db)
    spec = _cal_spec("sum", ds, None, T_SPRING + 3600000,
                     T_SPRING + 2 * DAY, batch=hb)
    assert spec.n_cal_anchors > 0
    ref = pyoracle.group_by(spec, hb)
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    workload.run_cells_device(engine, spec, cells_d, db, res)
    compare(_result_points(res, db.n_groups), ref, False, where="cells/" + ds)


def test_per_series_grids_with_fill_chain_ends_inside_the_window(engine):  # noqa: F811
    """FillingDownsampler over per-series grids whose caller-supplied chains
    end inside the window: every series anchored off the filling grid's own
    chain (7mc grids restart each day: a series first seen on day 2 steps
    its own chain) gets a chain that ends three edges past its anchor.  Its
    later points lie in buckets the table cannot place — on the filling grid
    (emitted) or not (dropped) — so the engine must not drop them (and fill
    their buckets) silently: E_UNSUPPORTED, the Java path's query (advisor,
    round 4)."""
    import numpy as np
    b = datasets.random_batch(197, n_series=24, n_groups=3, span_ms=3 * DAY,
                              cadence_ms=60000, t0=T_SPRING)
    start, end = T_SPRING + 3600000, T_SPRING + 2 * DAY
    spec = _cal_spec("sum", "7mc-avg-nan", None, start, end, batch=b)
    assert spec.n_cal_anchors > 0
    edges = spec._cal_edges_ref.copy()
    anchors, aedge = (np.array(x) for x in spec._cal_anchor_refs)
    big = np.iinfo(np.int64).max
    terms = np.nonzero(edges == big)[0]
    j = int(np.searchsorted(anchors, start, "right")) - 1
    fd_chain = int(np.searchsorted(terms, aedge[j]))
    cut = 0
    for s in range(b.n_series):
        ts = b.ts[b.offsets[s]:b.offsets[s + 1]]
        ts = ts[ts >= start]
        if not len(ts):
            continue
        k = int(np.searchsorted(anchors, ts[0], "right")) - 1
        e = int(aedge[k])
        if int(np.searchsorted(terms, e)) != fd_chain and \
                edges[e + 3] != big and ts[-1] > edges[e + 3]:
            edges[e + 3] = big  # the series' chain: 3 edges
            cut += 1
    assert cut > 0
    keep = edges[aedge] == anchors
    anchors, aedge = anchors[keep], aedge[keep]
    spec._cal_edges_ref, spec._cal_anchor_refs = edges, (anchors, aedge)
    spec.cal_edges = edges.ctypes.data
    spec.n_cal_edges = len(edges)
    spec.cal_anchors = anchors.ctypes.data
    spec.cal_anchor_edge = aedge.ctypes.data
    spec.n_cal_anchors = len(anchors)
    with pytest.raises(core.UnsupportedOperationException):
        engine.run(spec, b)
