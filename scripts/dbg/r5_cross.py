"""Debug: one cross-series query, print the engine's error text."""
from opentsdb_amd import core
from opentsdb_amd.engine import Engine
from tests import datasets
from tests.test_gpu_parity import _spec

e = Engine(0)
b = datasets.random_batch(11, n_series=60, n_groups=6)
for agg in ("sum", "avg", "max"):
    for ds in ("avg", "max"):
        spec = _spec(agg, ds)
        try:
            r = e.run(spec, b)
            print(agg, ds, "ok", sum(len(g.ts) for g in r))
        except core.OpenTSDBException as x:
            print(agg, ds, "ERR", x.status, x)
