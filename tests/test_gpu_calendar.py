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
                                   ("1dc-sum-zero", "America/Denver")])
def test_calendar_rate(engine, ds, tz):  # noqa: F811
    b = datasets.random_batch(5, n_series=20, n_groups=2, span_ms=5 * DAY,
                              cadence_ms=300000, counter=True, t0=T_SPRING)
    ro = core.RateOptions(True, core.LONG_MAX, 1000000)
    spec = _cal_spec("sum", ds, tz, T_SPRING, T_SPRING + 4 * DAY, True, ro,
                     batch=b)
    check(engine, spec, b, False, where=ds)
