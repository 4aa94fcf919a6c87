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
    ap.add_argument("--named", action="store_true",
                    help="the metric's named query sum:1m-avg (LERP) instead "
                         "of the config's")
    ap.add_argument("--variants", default="",
                    help="comma list of OTSDB_CELLS_VARIANT values (variants "
                         "build), timed interleaved")
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
    if a.named:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import bench  # noqa: E402
        spec = bench.named_spec(a.config)
    else:
        spec = workload.query_spec(a.config)
    nbk = 10200 if a.named else 2100
    res = DeviceResult(torch, db.n_groups, db.n_groups * nbk, "cuda")
    cb = cells.n_bytes
    vs = [v for v in a.variants.split(",") if v] or [None]
    ref = None
    times = {v: [] for v in vs}
    for rnd in range(3 if len(vs) > 1 else 1):
        for v in vs:
            if v is not None:
                os.environ["OTSDB_CELLS_VARIANT"] = v
            workload.run_cells_device(eng, spec, cells, db, res)
            torch.cuda.synchronize()
            out = res.val[:int(res.offsets[-1])].clone()
            if ref is None:
                ref = out
            same = out.numel() == ref.numel() and bool(
                ((out.view(torch.float64) - ref.view(torch.float64)).abs()
                 <= 1e-9 * ref.view(torch.float64).abs().clamp(min=1)).all())
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
            eng.lib.otsdb_prof_enable(eng.ctx, 0)
            kb = ms[0] / max(nn[0], 1) / 1e3
            print("stages ms:", [round(ms[i] / max(nn[i], 1), 3) for i in range(8)],
                  flush=True)
            times[v].append(kb)
            print("variant %s round %d: %d pts %.3f GB compacted; query %.2f ms "
                  "(%.1f Gpts/s); k_bucketize_cells %.2f ms = %.0f GB/s "
                  "compacted; same as first: %s"
                  % (v, rnd, n, cb / 1e9, dq * 1e3, n / dq / 1e9, kb * 1e3,
                     cb / kb / 1e9, same), flush=True)
    for v in vs:
        print("variant %s: k_bucketize_cells min %.2f ms" % (v, min(times[v]) * 1e3))

if __name__ == "__main__":
    main()
