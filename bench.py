"""Headline benchmark: data points aggregated per second for a downsample +
group-by query (BASELINE.json metric), on N GPUs of one node.

One process per GPU.  Each rank owns a contiguous shard of series of the
synthetic dataset (weak scaling: `--series` per GPU, default the BASELINE
config's series count), generated straight into HBM.  A step is one
execution of the query (otsdb_agg_run_device: downsample, interpolate,
group-by, compact) over the rank's resident batch; for the host-grouped
workload every group is rank-local, so there is no data-path collective.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2]

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec, MI355X_MICROARCH.md
BYTES_PER_POINT = 16   # int64 ts + 64-bit value, one read


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--series", type=int, default=0,
                    help="series per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decode", action="store_true",
                    help="skip the secondary compacted-cell decode figure")
    return ap.parse_args()


def decode_figure(eng, config, n_series, reps=5):
    """Secondary figure: the compacted-cell decode of the same
    workload's series at whole-second resolution (2-byte qualifiers, 8-byte
    doubles + meta byte per hour row, the format a scan returns): cells are
    encoded in HBM (otsdb_encode_cells_device), then otsdb_decode_cells_device
    (validate/count, scan, write) is timed end to end."""
    import torch
    from opentsdb_amd import workload
    g = workload.gen_spec(config)
    g.flags = 1
    db = workload.generate_device(eng, g, 0, n_series, config=config)
    n = db.n_points_total
    cells = workload.encode_cells_device(eng, db)
    db.ts = db.val = None  # keep the group arrays only
    torch.cuda.empty_cache()
    # output columns allocated once, outside the timed region
    out = (torch.zeros(n_series + 1, dtype=torch.int64, device="cuda"),
           torch.empty(n, dtype=torch.int64, device="cuda"),
           torch.empty(n, dtype=torch.int64, device="cuda"),
           torch.empty(n, dtype=torch.uint8, device="cuda"))
    workload.decode_cells_device(eng, cells, out=out)  # warm-up
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        workload.decode_cells_device(eng, cells, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    cb = cells.n_bytes
    del out
    torch.cuda.empty_cache()
    # the whole query straight from the cells: decode fused into the
    # downsample (otsdb_agg_run_cells_device)
    from opentsdb_amd.engine import DeviceResult
    spec = workload.query_spec(config)
    res = DeviceResult(torch, db.n_groups, db.n_groups * 2100, "cuda")
    workload.run_cells_device(eng, spec, cells, db, res)  # warm-up
    eng.lib.otsdb_prof_enable(eng.ctx, 1)
    eng.lib.otsdb_prof_read(eng.ctx, None, None, 0, 1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        workload.run_cells_device(eng, spec, cells, db, res)
    torch.cuda.synchronize()
    dq = (time.perf_counter() - t) / reps
    import ctypes as C
    ms = (C.c_double * 8)()
    nn = (C.c_int64 * 8)()
    eng.lib.otsdb_prof_read(eng.ctx, ms, nn, 8, 1)
    eng.lib.otsdb_prof_enable(eng.ctx, 0)
    kb = ms[0] / max(nn[0], 1) / 1e3
    del cells, res, db
    torch.cuda.empty_cache()
    return {"kernel": "k_decode (count + scan + write)",
            "points": n, "ms": dt * 1e3, "value": n / dt,
            "unit": "data points/s",
            "compacted_bytes": cb, "compacted_bytes_per_point": cb / n,
            "achieved_GBs": (cb + 17 * n) / dt / 1e9,
            "note": "reads the compacted cells, writes ts/val/is_float "
                    "(17 B/point); not part of the headline value",
            "fused_query": {
                "what": "the same C2 query straight from the cells, decode "
                        "fused into the downsample (k_bucketize_cells)",
                "value": n / dq, "unit": "data points/s",
                "ms_per_query": dq * 1e3,
                "k_bucketize_cells_ms": kb * 1e3,
                "achieved_GBs_compacted": cb / kb / 1e9 if kb else None,
                "frac_of_8TBs": cb / kb / 8e12 if kb else None}}


def cpu_baseline(config, target_s):
    """The oracle (iterator-faithful C restatement of the reference's
    single-threaded per-group evaluation) timed on a bounded sample of the
    same workload: the first whole groups of series of the config."""
    from opentsdb_amd import workload
    from oracle import pyoracle
    g = workload.gen_spec(config)
    spec = workload.query_spec(config)
    gof = lambda s: workload.group_of(config, s)  # noqa: E731
    # calibrate on 10 series, then size the sample to ~target_s
    hb = pyoracle.gen_batch(g, 0, 10, gof)
    t = time.perf_counter()
    pyoracle.group_by(spec, hb)
    dt = max(time.perf_counter() - t, 1e-3)
    n = int(10 * target_s / dt)
    n = max(10, min(n, workload.CONFIGS[config]["n_series"]))
    n -= n % 10
    hb = pyoracle.gen_batch(g, 0, n, gof)
    pts = int(hb.offsets[-1])
    t = time.perf_counter()
    pyoracle.group_by(spec, hb)
    dt = time.perf_counter() - t
    n_groups = len(hb.group_offsets) - 1
    out = {"value": pts / dt, "unit": "data points/s", "cores": 1,
           "kind": "port",
           "sample": "%s query over its first %d series (%d points, %d "
                     "groups), single thread, %.1f s" % (
                         config, n, pts, n_groups, dt)}
    del hb
    # (ii) of SURVEY §8d: the same sample with whole groups sharded over the
    # host threads (ctypes drops the GIL inside the oracle call).  Only for
    # host-grouped configs: the reference evaluates one group on one thread.
    threads = min(16, os.cpu_count() or 1)
    if workload.CONFIGS[config]["group"] == "host" and n >= 10 * threads > 10:
        from concurrent.futures import ThreadPoolExecutor
        cut = [((n // 10) * i // threads) * 10 for i in range(threads + 1)]
        parts = [pyoracle.gen_batch(g, cut[i], cut[i + 1] - cut[i], gof)
                 for i in range(threads)]
        with ThreadPoolExecutor(threads) as ex:
            t = time.perf_counter()
            list(ex.map(lambda b: pyoracle.group_by(spec, b), parts))
            dtm = time.perf_counter() - t
        out["all_cores"] = {"value": pts / dtm, "cores": threads,
                            "seconds": dtm}
    return out


_last = None


def main():
    args = parse()
    import numpy as np
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult, Engine, run_device

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (a multi-rank run on a one-GPU box): every rank on
    # device 0 and gloo instead of RCCL; the driver's runs use neither
    if os.environ.get("OTSDB_BENCH_SAME_DEVICE"):
        local = 0
    backend = os.environ.get("OTSDB_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl",
                                    device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    cfg = workload.CONFIGS[args.config]
    n_series = args.series or workload.default_series_per_gpu(args.config)
    # groups that span ranks ({dc=*}, no group-by) take the cross-rank
    # exchange: partial all-gather, or the histogram protocol for
    # percentiles (opentsdb_amd/dist.py); host groups stay rank-local
    sharded = world > 1 and workload.spans_ranks(args.config)
    G_glob = (workload.n_groups_global(args.config, n_series * world)
              if sharded else None)
    eng = Engine(local)
    g = workload.gen_spec(args.config)
    t_gen = time.perf_counter()
    db = workload.generate_device(eng, g, series0=rank * n_series,
                                  n_series=n_series, config=args.config,
                                  n_groups=G_glob)
    t_gen = time.perf_counter() - t_gen
    n_points = db.n_points_total
    spec = workload.query_spec(args.config)
    sz = eng.plan(spec, db)
    res = DeviceResult(torch, db.n_groups, int(sz.max_out_points), "cuda")
    if sharded:
        from opentsdb_amd import dist as odist

        def step():
            global _last
            _last = odist.run_sharded_any(eng, spec, db, G_glob)
    else:
        def step():
            run_device(eng, spec, db, res)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    import ctypes as C
    eng.lib.otsdb_prof_enable(eng.ctx, 1)
    eng.lib.otsdb_prof_read(eng.ctx, None, None, 0, 1)  # reset

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    ms = (C.c_double * 8)()
    n = (C.c_int64 * 8)()
    eng.lib.otsdb_prof_read(eng.ctx, ms, n, 8, 1)
    eng.lib.otsdb_prof_enable(eng.ctx, 0)
    stage_ms = [ms[i] / max(n[i], 1) for i in range(5)]

    total_points = n_points * world
    out_points = int((_last if sharded else res).offsets[-1].item())
    if dist:
        dev = "cuda" if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tp = torch.tensor([n_points], dtype=torch.int64, device=dev)
        dist.all_reduce(tp)
        total_points = int(tp.item())
    step_s = elapsed / args.steps
    value = total_points / step_s

    # dominant kernel: k_bucketize streams every point once (16 B/point)
    kb_s = stage_ms[0] / 1e3
    achieved = BYTES_PER_POINT * n_points / kb_s / 1e9 if kb_s > 0 else None
    # PMC traffic of this exact workload (scripts/gpu_pmc.sh, default size,
    # one GPU), per k_bucketize launch
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc) and not args.series and world == 1:
        with open(pmc) as f:
            traffic = json.load(f).get("k_bucketize_hbm_bytes_per_launch")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, args.cpu_seconds)

    n_groups, n_buckets = db.n_groups, int(sz.n_buckets)
    decode = None
    if world == 1 and not args.no_decode and args.config == "C2":
        del db, res
        torch.cuda.empty_cache()
        decode = decode_figure(eng, args.config, n_series)

    if rank == 0:
        line = {
            "metric": "data points aggregated/sec (node) for 1m-avg "
                      "downsample + sum group-by, 1/2/4/8 GPU",
            "value": value,
            "unit": "data points/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": step_s * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY §8d generator, seed 42, generated in "
                    "HBM; %d series x %d d @10s per GPU)" % (
                        n_series, cfg["days"]),
            "config": {
                "workload": "%s: %s:%s:sys.cpu.user{%s} over %d series x %d "
                            "days @10s per GPU" % (
                                args.config, cfg["agg"], cfg["ds"],
                                (cfg["group"] or "") + "=*" if cfg["group"]
                                else "", n_series, cfg["days"]),
                "points_per_gpu": n_points,
                "groups_per_gpu": n_groups,
                "buckets": n_buckets,
                "output_points_per_gpu": out_points,
                "parallelism": "series-sharded dp%d%s" % (
                    world, " + RCCL exchange" if sharded else ""),
                "stage_ms": {"bucketize": stage_ms[0],
                             "transform": stage_ms[1],
                             "group": stage_ms[2], "prep": stage_ms[3],
                             "compact": stage_ms[4]},
                "generate_s": t_gen,
            },
            "roofline": {
                "bound": "hbm",
                # the downsample stage's kernel: k_bucketize_group when the
                # group-by folds into it (zimsum over one-chunk groups, C2),
                # k_bucketize_k otherwise
                "kernel": ("k_bucketize_group" if (
                    args.config == "C2" and
                    os.environ.get("OTSDB_GRP_FUSED", "1") != "0")
                    else "k_bucketize_k"),
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": BYTES_PER_POINT * n_points,
            },
            "cpu_baseline": cpu,
            "decode": decode,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
