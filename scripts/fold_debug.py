"""Debug harness: runs a few small downsampled queries, each in its own
subprocess under a time limit, against the library named by OTSDB_LIB."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = ["kat", "single", "rand"]


def run_case(name):
    import numpy as np
    from opentsdb_amd import core
    from opentsdb_amd.engine import Engine
    from oracle import pyoracle
    from tests import datasets, kat
    eng = Engine(0)
    if name == "kat":
        c = [c for c in kat.load_cases("group_by")
             if c["name"] == "ai_many_spans_downsampled"][0]
        spec, b = kat.spec_from_case(c["spec"]), kat.batch_from_case(c)
    else:
        b = datasets.random_batch(11, n_series=1 if name == "single" else 60,
                                  n_groups=1 if name == "single" else 6)
        d = core.DownsamplingSpecification("1m-avg")
        s0 = datasets.T0
        spec = core.make_spec(s0, s0 + 3 * 3600 * 1000, core.Aggregators.get("sum"),
                              d, s0, s0 + 3 * 3600 * 1000)
    got = eng.run(spec, b)
    ref = pyoracle.group_by(spec, b)
    bad = 0
    for a, r in zip(got, ref):
        if len(a.ts) != len(r) or not np.array_equal(a.ts, r["ts"]):
            bad += 1
            continue
        va, vr = a.bits.view(np.float64), r["bits"].view(np.float64)
        if not np.allclose(va, vr, rtol=1e-12, atol=0, equal_nan=True):
            bad += 1
    print("case %s: %d groups, %d mismatched" % (name, len(got), bad), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run_case(sys.argv[1])
        sys.exit(0)
    for c in CASES:
        try:
            r = subprocess.run([sys.executable, "-u", __file__, c], timeout=60)
            print("case %s rc=%d" % (c, r.returncode), flush=True)
        except subprocess.TimeoutExpired:
            print("case %s TIMEOUT" % c, flush=True)
            sys.exit(3)
