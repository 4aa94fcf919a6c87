"""MAX / MIN fill-ins at the pure 1e-12 bound (Needs an MI355X).

A member with no value at an emitted timestamp contributes, under MAX / MIN
interpolation, Long.MAX_VALUE / Double.MAX_VALUE or their negatives
(AggregationIterator.java:711-719, :781-787): mimmin and mimmax interpolate
that way by default (Aggregators.java:47-119), any aggregator can be told to
by an interpolation override.  Those contributions are exact constants, so
nothing here is compared with an absolute floor: positive float data (no
cancellation) against the oracle at 1e-12 relative, and integer data —
every downsampled value exact, so every selection bit-exact — bit for bit.
Round 4's sweep comparator took the fill-ins' MAX_VALUE as a rounding scale
and accepted any value at such points; tests/test_comparator_cpu.py pins
the fixed comparator."""
import pytest

from opentsdb_amd import core
from tests import datasets
from tests.test_gpu_parity import check

pytestmark = pytest.mark.gpu

LERP, ZIM, MAX, MIN, PREV = range(5)


@pytest.fixture(scope="module")
def engine():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def _spec(agg, ds, interp=None, fill="none", interval="1m", hours=3):
    d = core.DownsamplingSpecification("%s-%s-%s" % (interval, ds, fill))
    t0, t1 = datasets.T0, datasets.T0 + hours * 3600 * 1000
    return core.make_spec(t0, t1, core.Aggregators.get(agg), d, t0, t1,
                          False, None, interp)


# (aggregator, interpolation override): the two fill-in aggregators with
# their own interpolation and every other one; sum / avg / dev / p50 / min /
# max made to take the fill-ins
CASES = ([("mimmin", None), ("mimmax", None)] +
         [("mimmin", i) for i in (LERP, ZIM, MIN, PREV)] +
         [("mimmax", i) for i in (LERP, ZIM, MAX, PREV)] +
         [(a, i) for a in ("sum", "avg", "p50", "p99", "min", "max", "dev")
          for i in (MAX, MIN)])


@pytest.mark.parametrize("ds", ["sum", "avg", "zimsum"])
@pytest.mark.parametrize("agg,interp", CASES)
def test_fill_ins_positive_floats(engine, agg, interp, ds):
    """U[0, 100) floats with outages, late starts and early ends (members
    missing at many emitted timestamps): 60 series in 6 groups (fold
    tiles), and one 400-series group (the row path)."""
    for seed, kw in ((71, dict(n_series=60, n_groups=6)),
                     (72, dict(n_series=400, big_group=True,
                               span_ms=3600 * 1000))):
        b = datasets.random_batch(seed, cadence_ms=15000, **kw)
        hours = 3 if seed == 71 else 1
        for fill in ("none", "nan"):
            spec = _spec(agg, ds, interp, fill, interval="2m", hours=hours)
            check(engine, spec, b, False,
                  where="%s:i%s:%s-%s/%d" % (agg, interp, ds, fill, seed),
                  floor=0.0)


SELECT = [("mimmin", None), ("mimmax", None), ("mimmin", LERP),
          ("mimmax", PREV), ("min", MAX), ("max", MIN), ("p50", MAX),
          ("p99", MIN), ("median", MAX)]


@pytest.mark.parametrize("ds", ["sum", "avg", "zimsum", "max"])
@pytest.mark.parametrize("agg,interp", SELECT)
def test_fill_ins_integer_selections_bit_exact(engine, agg, interp, ds):
    """Integer data U[-50, 100): sums and averages of longs are exact, so a
    selection across series (fill-ins included) is bit-exact."""
    b = datasets.random_batch(73, n_series=80, n_groups=4, value_kind="int",
                              cadence_ms=20000)
    for interval in ("1m", "5m"):
        spec = _spec(agg, ds, interp, interval=interval)
        check(engine, spec, b, True,
              where="%s:i%s:%s-%s" % (agg, interp, interval, ds))
