"""Times the C2 query from storage rows (otsdb_agg_run_raw_device:
query-time compaction, span assembly, the cells fold) and, with --mixed, the
generic decode of rows mixing 2- and 4-byte qualifiers.  Stage times per
rep; for rocprofv3 --kernel-trace --stats runs of those paths."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--series", type=int, default=100000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mixed", action="store_true")
    a = ap.parse_args()
    import torch
    from opentsdb_amd import storage, workload
    from opentsdb_amd.engine import DeviceResult, Engine
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import bench  # noqa: E402  (stage names / reader)
    eng = Engine(0)
    g = workload.gen_spec(a.config)
    g.flags = 0 if a.mixed else 1
    db = workload.generate_device(eng, g, 0, a.series, config=a.config)
    n = db.n_points_total
    if a.mixed:
        even = db.ts[0::2]
        even -= torch.remainder(even, 1000)
        del even
    cells = workload.encode_cells_device(eng, db)
    db.ts = db.val = None
    torch.cuda.empty_cache()
    spec = workload.query_spec(a.config)
    res = DeviceResult(torch, db.n_groups, db.n_groups * 2100, "cuda")
    if a.mixed:
        fn = lambda: workload.run_cells_device(eng, spec, cells, db, res)  # noqa
    else:
        raw = storage.raw_rows_from_cells(cells)
        fn = lambda: storage.run_raw_device(eng, spec, raw, db, res)  # noqa
    fn()
    torch.cuda.synchronize()
    read = bench.stage_reader(eng, all_stages=True)
    eng.lib.otsdb_prof_enable(eng.ctx, 1)
    read()
    t = time.perf_counter()
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / a.reps
    st = read()
    print("%s %d pts %.3f GB: %.2f ms/query (%.1f Gpts/s); stages %s" % (
        "mixed cells" if a.mixed else "storage rows", n, cells.n_bytes / 1e9,
        dt * 1e3, n / dt / 1e9,
        {k: round(v, 3) for k, v in zip(bench.STAGES, st) if v}), flush=True)


if __name__ == "__main__":
    main()
