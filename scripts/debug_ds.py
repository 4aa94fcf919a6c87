"""Debug: single-series downsample parity, growing sizes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from opentsdb_amd import core
from opentsdb_amd.batch import HostBatch
from opentsdb_amd.engine import Engine
from oracle import pyoracle
T0 = 1356998400000
e = Engine(0)
for n in (10, 64, 127, 128, 129, 200, 300, 1000):
    for off in (0, 1):
        ts = T0 + 10000 * np.arange(n, dtype=np.int64) + off * 10000
        v = np.arange(n, dtype=np.float64) + 1.0
        b = HostBatch(np.array([0, n]), ts, v.view(np.int64), np.ones(n, np.uint8))
        d = core.DownsamplingSpecification("1m-sum")
        spec = core.make_spec(T0, T0 + 10000 * (n + 5), core.Aggregators.SUM, d, T0, T0)
        got = e.run(spec, b)[0]
        ref = pyoracle.group_by(spec, b)[0]
        gv = got.bits.view(np.float64); rv = ref["bits"].view(np.float64)
        ok = len(gv) == len(rv) and np.array_equal(got.ts, ref["ts"]) and np.allclose(gv, rv)
        print(n, off, "OK" if ok else "BAD", len(gv), len(rv))
        if not ok:
            m = min(len(gv), len(rv))
            bad = np.nonzero(~np.isclose(gv[:m], rv[:m]))[0][:6]
            print("  ts", got.ts[:8], ref["ts"][:8])
            print("  bad idx", bad, gv[bad], rv[bad])
