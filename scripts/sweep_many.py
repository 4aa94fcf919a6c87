"""Run the random-query sweeps (tests/test_gpu_sweep.py) over many more
seeds than the test suite does and list every divergence from the oracle.
Usage: python scripts/sweep_many.py [n_general] [n_rate] [first_seed]"""
import os
import sys
import time
import traceback

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from opentsdb_amd.engine import Engine  # noqa: E402
from tests.test_gpu_parity import check  # noqa: E402
from tests.test_gpu_sweep import _case, _rate_case  # noqa: E402


def main():
    ng = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    s0 = int(sys.argv[3]) if len(sys.argv) > 3 else 120
    e = Engine(0)
    bad = 0
    t = time.time()
    for i, seed in enumerate(range(s0, s0 + ng + nr)):
        general = i < ng
        if general:
            b, spec, exact, where = _case(seed)
        else:
            b, spec, exact, where = _rate_case(seed)
        try:
            # the suite's comparator: 1e-12 relative, the contributions'
            # floor only where they have both signs
            check(e, spec, b, exact, where=where, floor="contributions")
        except Exception as ex:  # noqa: BLE001
            bad += 1
            msg = str(ex).splitlines()[0][:300]
            print("FAIL %s %s: %s" % ("gen" if general else "rate", where,
                                      msg), flush=True)
            if bad <= 3:
                traceback.print_exc(limit=2)
        if i % 100 == 99:
            print("%d cases, %d failing, %.0f s" % (i + 1, bad, time.time() - t),
                  flush=True)
    e.close()
    print("done: %d cases, %d failing" % (ng + nr, bad))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
