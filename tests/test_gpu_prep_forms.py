"""k_prep + k_fold_prep as one launch (k_prep_fold) or two (Needs an MI355X).

Small queries run the fused kernel (every (series, window boundary) thread
finds its series' bounds itself); queries with more than
OTSDB_PREP_FOLD_MAX (series, boundary) pairs run the two kernels.  The
environment override lets one process run both forms: each query below runs
both ways, both are compared with the oracle and with each other bit for
bit (the fold is deterministic, so the two forms must agree exactly)."""
import os

import numpy as np
import pytest

from oracle import pyoracle
from tests import datasets
from tests.test_gpu_parity import _spec, compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def _both(engine, spec, hb):
    out = []
    old = os.environ.get("OTSDB_PREP_FOLD_MAX")
    try:
        for lim in ("0", "1000000"):
            os.environ["OTSDB_PREP_FOLD_MAX"] = lim
            out.append(engine.run(spec, hb))
    finally:
        if old is None:
            os.environ.pop("OTSDB_PREP_FOLD_MAX", None)
        else:
            os.environ["OTSDB_PREP_FOLD_MAX"] = old
    return out


CASES = [  # (aggregator, downsampler, fill, interval) over narrowed windows
    ("sum", "avg", "none", "30s"),
    ("avg", "max", "none", "1m"),
    ("zimsum", "sum", "zero", "30s"),
    ("dev", "avg", "none", "1m"),
    ("count", "count", "nan", "30s"),
    ("max", "last", "none", "10s"),
    ("p90", "avg", "none", "1m"),
]


@pytest.mark.parametrize("agg,ds,fill,interval", CASES)
def test_fused_and_separate_prep_agree(engine, agg, ds, fill, interval):
    hb = datasets.random_batch(401, n_series=40, n_groups=4)
    spec = _spec(agg, ds, fill=fill, interval=interval)
    ref = pyoracle.group_by(spec, hb)
    sep, fused = _both(engine, spec, hb)
    for got, where in ((sep, "separate"), (fused, "fused")):
        compare(got, ref, ds in ("max", "count", "last") and agg != "dev",
                where="%s:%s/%s" % (agg, ds, where))
    for a, b in zip(sep, fused):
        assert np.array_equal(a.ts, b.ts)
        assert np.array_equal(a.bits, b.bits)


def test_fused_prep_seek_and_stop_inside_series(engine):
    """A window that cuts every series on both sides (the seek and stop
    searches run, the point past the window is folded by the series' first
    thread only) and series wholly outside it."""
    hb = datasets.random_batch(402, n_series=30, n_groups=3)
    s0 = datasets.T0 + 1800 * 1000 + 7000
    e0 = datasets.T0 + 2 * 3600 * 1000 - 13000
    for agg, ds in (("sum", "avg"), ("max", "min")):
        spec = _spec(agg, ds, start=s0, end=e0, interval="20s")
        ref = pyoracle.group_by(spec, hb)
        sep, fused = _both(engine, spec, hb)
        compare(sep, ref, False, where="cut-separate")
        compare(fused, ref, False, where="cut-fused")
        for a, b in zip(sep, fused):
            assert np.array_equal(a.bits, b.bits)


@pytest.mark.parametrize("agg", ["dev", "sum", "max"])
def test_wide_windows_without_preloaded_contexts(engine, agg):
    """1,200 single-series groups on a 2,160-bucket grid: enough tiles that
    the fold keeps full 2,048-bucket windows, whose states leave no LDS for
    the preloaded member contexts (ds_tu.hip drops them: each member loads
    its own), next to the small-window queries above that preload them."""
    hb = datasets.random_batch(403, n_series=1200, n_groups=1200,
                               cadence_ms=60000)
    spec = _spec(agg, "avg", interval="5s")
    ref = pyoracle.group_by(spec, hb)
    got = engine.run(spec, hb)
    compare(got, ref, False, where="wide/" + agg)
