"""Times the fused cells query (k_bucketize_cells) on a C2-shaped workload:
generate in HBM, encode to compacted cells, run otsdb_agg_run_cells_device.
For PMC passes and quick A/B of the fused kernel."""
import argparse
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--series", type=int, default=100000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import Engine, DeviceResult
    eng = Engine(0)
    g = workload.gen_spec(a.config)
    g.flags = 1
    db = workload.generate_device(eng, g, 0, a.series, config=a.config)
    n = db.n_points_total
    cells = workload.encode_cells_device(eng, db)
    db.ts = db.val = None
    torch.cuda.empty_cache()
    spec = workload.query_spec(a.config)
    res = DeviceResult(torch, db.n_groups, db.n_groups * 2100, "cuda")
    workload.run_cells_device(eng, spec, cells, db, res)
    eng.lib.otsdb_prof_enable(eng.ctx, 1)
    eng.lib.otsdb_prof_read(eng.ctx, None, None, 0, 1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        workload.run_cells_device(eng, spec, cells, db, res)
    torch.cuda.synchronize()
    dq = (time.perf_counter() - t) / a.reps
    ms = (C.c_double * 8)()
    nn = (C.c_int64 * 8)()
    eng.lib.otsdb_prof_read(eng.ctx, ms, nn, 8, 1)
    kb = ms[0] / max(nn[0], 1) / 1e3
    cb = cells.n_bytes
    print("cells: %d pts %.3f GB compacted; query %.2f ms (%.1f Gpts/s); "
          "k_bucketize_cells %.2f ms = %.0f GB/s compacted"
          % (n, cb / 1e9, dq * 1e3, n / dq / 1e9, kb * 1e3, cb / kb / 1e9))


if __name__ == "__main__":
    main()
