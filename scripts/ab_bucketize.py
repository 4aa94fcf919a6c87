"""A/B of k_bucketize variants in ONE process and ONE context (same input
and workspace placement), interleaved rounds (methodology rule:
cdna_hip_programming.md §5.4 r24).  Needs the variants build
(OTSDB_LIB=.../libotsdb_agg_variants.so), which re-reads OTSDB_BUCKETIZE_K
per query."""
import argparse, ctypes as C, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from opentsdb_amd import workload
from opentsdb_amd.engine import DeviceResult, Engine, run_device

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C2")
ap.add_argument("--series", type=int, default=0)
ap.add_argument("--ks", default="2,4,8")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
torch.cuda.set_device(0)
ks = [int(x) for x in a.ks.split(",")]
e0 = Engine(0)
engs = {k: e0 for k in ks}
cfg = workload.CONFIGS[a.config]
n = a.series or cfg["n_series"]
db = workload.generate_device(e0, workload.gen_spec(a.config), 0, n, config=a.config)
spec = workload.query_spec(a.config)
sz = e0.plan(spec, db)
res = {k: DeviceResult(torch, db.n_groups, int(sz.max_out_points), "cuda") for k in ks}
times = {k: [] for k in ks}
for k in ks:
    os.environ["OTSDB_BUCKETIZE_K"] = str(k)
    run_device(engs[k], spec, db, res[k])
torch.cuda.synchronize()
for r in range(a.rounds):
    for k in ks:
        e = engs[k]
        os.environ["OTSDB_BUCKETIZE_K"] = str(k)
        e.lib.otsdb_prof_enable(e.ctx, 1)
        e.lib.otsdb_prof_read(e.ctx, None, None, 0, 1)
        for _ in range(a.reps):
            run_device(e, spec, db, res[k])
        ms = (C.c_double * 8)(); nn = (C.c_int64 * 8)()
        e.lib.otsdb_prof_read(e.ctx, ms, nn, 8, 1)
        e.lib.otsdb_prof_enable(e.ctx, 0)
        times[k].append(ms[0] / nn[0])
N = db.n_points_total
out = {}
for k in ks:
    t = np.median(times[k])
    out[k] = dict(ms_median=t, ms_min=min(times[k]), gbs=16 * N / t / 1e6)
# parity between variants
base = res[ks[0]]
for k in ks[1:]:
    a0 = base.val[:int(base.offsets[-1])].view(torch.float64)
    b0 = res[k].val[:int(res[k].offsets[-1])].view(torch.float64)
    if a0.numel() == b0.numel():
        out[k]["max_rel_diff_vs_k%d" % ks[0]] = float(
            ((a0 - b0).abs() / a0.abs().clamp(min=1)).max())
print(json.dumps({"config": a.config, "series": n, "points": N, "variants": out}))
