"""Run the cells / storage-rows sweep (tests/test_gpu_sweep.py
test_random_cells_sweep) over many more seeds and list every divergence.
Usage: python scripts/sweep_cells.py [n] [first_seed]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from opentsdb_amd.engine import Engine  # noqa: E402
from tests.test_gpu_sweep import test_random_cells_sweep  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    s0 = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    e = Engine(0)
    bad = 0
    t = time.time()
    for i, seed in enumerate(range(s0, s0 + n)):
        try:
            test_random_cells_sweep(e, seed)
        except Exception as ex:  # noqa: BLE001
            bad += 1
            print("FAIL seed %d: %s" % (seed, str(ex).splitlines()[0][:300]),
                  flush=True)
        if i % 50 == 49:
            print("%d cases, %d failing, %.0f s" % (i + 1, bad, time.time() - t),
                  flush=True)
    print("done: %d cases, %d failing" % (n, bad))
    e.close()


if __name__ == "__main__":
    main()
