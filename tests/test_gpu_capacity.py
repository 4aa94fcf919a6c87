"""OTSDB_E_CAPACITY from the host entries (Needs an MI355X): a result too
small for the query returns the status with result.offsets holding the
whole result's offsets — offsets[n_groups] is the capacity a retry needs
(include/otsdb_agg.h) — and the retry with it equals the plan-sized run."""
import ctypes as C

import numpy as np
import pytest

from opentsdb_amd import abi, core
from tests import datasets

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def _run(engine, spec, b, cap):
    G = b.n_groups
    offs = np.zeros(G + 1, np.int64)
    ts = np.zeros(max(cap, 1), np.int64)
    bits = np.zeros(max(cap, 1), np.int64)
    isint = np.ones(max(cap, 1), np.uint8)
    r = abi.Result(cap, offs.ctypes.data, ts.ctypes.data, bits.ctypes.data,
                   isint.ctypes.data)
    st = engine.lib.otsdb_agg_run(engine.ctx, C.byref(spec),
                                  C.byref(b.as_abi()), C.byref(r))
    return st, offs, ts, bits, isint


@pytest.mark.parametrize("ds,agg", [("1m-avg", "sum"), ("5m-max-nan", "avg"),
                                    ("0all-sum", "zimsum")])
def test_capacity_returns_the_needed_offsets(engine, ds, agg):
    b = datasets.random_batch(71, n_series=40, n_groups=4)
    spec = core.make_spec(datasets.T0, datasets.T0 + 3 * 3600000,
                          core.Aggregators.get(agg),
                          core.DownsamplingSpecification(ds),
                          datasets.T0 + 600000, datasets.T0 + 7200000)
    ref = engine.run(spec, b)
    need = sum(len(g.ts) for g in ref)
    assert need > 2
    st, offs, *_ = _run(engine, spec, b, 2)
    assert st == 7  # OTSDB_E_CAPACITY
    assert int(offs[-1]) == need
    assert np.array_equal(np.diff(offs), [len(g.ts) for g in ref])
    st, offs, ts, bits, isint = _run(engine, spec, b, need)
    assert st == 0
    for g, r in enumerate(ref):
        a, z = offs[g], offs[g + 1]
        assert np.array_equal(ts[a:z], r.ts) and np.array_equal(bits[a:z], r.bits)
        assert not isint[a:z].any()  # downsampled values are doubles
