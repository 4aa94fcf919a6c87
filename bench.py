"""Headline benchmark: data points aggregated per second for a downsample +
group-by query (BASELINE.json metric), on N GPUs of one node.

One process per GPU.  Each rank owns a contiguous shard of series of the
synthetic dataset (weak scaling: `--series` per GPU, default the BASELINE
config's series count), generated straight into HBM.  A step is one
execution of the query over the rank's resident batch: otsdb_agg_run_device
(downsample, interpolate, group-by, compact) for groups that live on one
rank; groups spanning ranks add the partial all-gather over RCCL
(opentsdb_amd/dist.py).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2]

With --gpus N > 1 outside a torch.distributed launch, this process starts
the N ranks itself (torch.distributed.run on 127.0.0.1, one rank per GPU)
without touching the GPU, and relays rank 0's line.  Prints ONE JSON line
(rank 0).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec, MI355X_MICROARCH.md
BYTES_PER_POINT = 16   # int64 ts + 64-bit value, one read
METRIC = ("data points aggregated/sec (node) for 1m-avg downsample + sum "
          "group-by, 1/2/4/8 GPU")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # BASELINE.md protocol: 3 warm-ups, then 10 timed executions
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--series", type=int, default=0,
                    help="series per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decode", action="store_true",
                    help="skip the secondary compacted-cell figures")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the named-query and PCIe-inclusive figures")
    ap.add_argument("--named-query", action="store_true",
                    help="profiling: time BASELINE's sum:1m-avg (LERP) shape "
                         "over the config's series instead of its query")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / collective rehearsal without the HIP "
                         "engine (CPU tests): times a gloo all-reduce")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(args):
    """--gpus N > 1 without WORLD_SIZE: run this script as N ranks under
    torch.distributed.run (one process per GPU) and relay rank 0's JSON
    line.  The parent never initialises the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % args.gpus, "--master-addr=127.0.0.1",
           "--master-port=%d" % _free_port(), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    for ln in p.stdout.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if lines:
        print(lines[-1], flush=True)
    return p.returncode if lines or p.returncode else 1


def timed_reps(fn, warm, reps):
    """median / mean seconds of `reps` synchronous calls after `warm`."""
    import statistics
    import torch
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts), sum(ts) / len(ts)


# otsdb_prof_* stages: 0 downsample / fold, 1 transform, 2 group /
# selection, 3 prep, 4 compact, 5 query-time row compaction, 6 span
# assembly, 7 the generic cells decode
STAGES = ("downsample", "transform", "group", "prep", "compact",
          "row_compaction", "span_assembly", "cells_decode")


def stage_reader(eng, all_stages=False):
    import ctypes as C

    def read(reset=True):
        ms = (C.c_double * 8)()
        n = (C.c_int64 * 8)()
        eng.lib.otsdb_prof_read(eng.ctx, ms, n, 8, 1 if reset else 0)
        return [ms[i] / max(n[i], 1) for i in range(8 if all_stages else 5)]
    return read


def workload_label(config, n_series):
    """The query as /api/query spells it (rate options included)."""
    from opentsdb_amd import workload
    cfg = workload.CONFIGS[config]
    rate = ""
    if cfg["rate"]:
        counter, cmax, reset = cfg["rate"]
        rate = "rate{%s,%d,%d}:" % ("counter" if counter else "", cmax, reset)
    grp = (cfg["group"] + "=*") if cfg["group"] else ""
    return "%s: %s:%s:%ssys.cpu.user{%s} over %d series x %d days @10s per " \
           "GPU" % (config, cfg["agg"], cfg["ds"], rate, grp, n_series,
                    cfg["days"])


def named_spec(config):
    """BASELINE's metric shape, sum:1m-avg{host=*} (LERP), over config's
    window."""
    from opentsdb_amd import core, workload
    c = workload.CONFIGS[config]
    ds = core.DownsamplingSpecification("1m-avg")
    q0 = workload.T0_S
    q1 = q0 + c["days"] * 86400 - 1
    return core.make_spec(core.get_scan_start_time_seconds(q0, ds),
                          core.get_scan_end_time_seconds(q1, ds),
                          core.Aggregators.get("sum"), ds, q0 * 1000,
                          q1 * 1000, normalize=True)


def pmc_traffic(name):
    """HBM bytes per launch of the dominant kernel measured by
    scripts/gpu_pmc.sh for this workload (the latest round's
    profiles/r<N>_pmc_<name>.json)."""
    import glob
    import re
    found = []
    for p in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_%s.json" % name)):
        m = re.match(r"r(\d+)_pmc_", os.path.basename(p))
        if m:
            found.append((int(m.group(1)), p))
    if not found:
        return None
    pmc = max(found)[1]
    with open(pmc) as f:
        d = json.load(f)
    return {"step": d.get("step_hbm_bytes"),
            "dominant_kernel": d.get("hbm_bytes_per_launch",
                                     d.get("k_bucketize_hbm_bytes_per_launch")),
            "source": os.path.relpath(pmc, ROOT)}


def named_query_figure(eng, db, config, warm=3, reps=10):
    """Secondary figure: the metric's own query shape, sum:1m-avg{host=*}
    (LERP interpolation), over the same resident C2 series — the ordered
    group fold with 10,080 one-minute buckets in 5 LDS windows."""
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult, run_device
    import torch
    c = workload.CONFIGS[config]
    spec = named_spec(config)
    sz = eng.plan(spec, db)
    res = DeviceResult(torch, db.n_groups, int(sz.max_out_points), "cuda")
    read = stage_reader(eng)
    eng.lib.otsdb_prof_enable(eng.ctx, 1)
    read()
    med, mean = timed_reps(lambda: run_device(eng, spec, db, res), warm, reps)
    st = read()
    eng.lib.otsdb_prof_enable(eng.ctx, 0)
    n = db.n_points_total
    kf = st[0] / 1e3
    out = {"query": "sum:1m-avg:sys.cpu.user{host=*} (LERP) over the same "
                    "%d series x %d d" % (db.n_series, c["days"]),
           "buckets": int(sz.n_buckets), "value": n / med,
           "unit": "data points/s", "ms_median": med * 1e3,
           "ms_mean": mean * 1e3,
           "stage_ms": {"fold": st[0], "prep": st[3], "compact": st[4]},
           "kernel": "k_fold (+ k_fold_prep)",
           "achieved_GBs": BYTES_PER_POINT * n / kf / 1e9 if kf else None,
           "algorithmic_bytes_per_launch": BYTES_PER_POINT * n,
           # scripts/gpu_pmc.sh with bench.py --named-query
           "traffic": pmc_traffic(config + "_named")}
    out["frac"] = out["achieved_GBs"] / HBM_PEAK_GBS if kf else None
    # over the whole query (median step), like the headline's frac
    out["step_frac"] = BYTES_PER_POINT * n / med / 1e9 / HBM_PEAK_GBS
    del res
    return out


def p999_figure(eng, db, config, warm=2, reps=5):
    """C5 names p99 and p999: the p999 query over the same
    resident series, timed like the headline."""
    from opentsdb_amd import core, workload
    from opentsdb_amd.engine import DeviceResult, run_device
    import torch
    spec = workload.query_spec(config)
    spec.agg_id = core.Aggregators.get("p999").id
    sz = eng.plan(spec, db)
    res = DeviceResult(torch, db.n_groups, int(sz.max_out_points), "cuda")
    read = stage_reader(eng)
    eng.lib.otsdb_prof_enable(eng.ctx, 1)
    read()
    med, mean = timed_reps(lambda: run_device(eng, spec, db, res), warm, reps)
    st = read()
    eng.lib.otsdb_prof_enable(eng.ctx, 0)
    n = db.n_points_total
    del res
    return {"query": "p999:1m-avg-nan over the same series", "value": n / med,
            "unit": "data points/s", "ms_median": med * 1e3,
            "ms_mean": mean * 1e3,
            "stage_ms": {"downsample": st[0], "transform": st[1],
                         "group_select": st[2], "prep": st[3],
                         "compact": st[4]}}


def pcie_figure(eng, config):
    """PCIe-inclusive rate (not the headline): otsdb_agg_run from host
    buffers — H2D of the columns, the query, D2H of the result — at C1 and
    on a 2,000-series subset of the config."""
    from opentsdb_amd import workload
    from oracle import pyoracle  # the data generator only (bench input)
    out = {}
    for name, cfg, n in (("C1", "C1", 1000), (config + "_subset", config, 2000)):
        g = workload.gen_spec(cfg)
        spec = workload.query_spec(cfg)
        hb = pyoracle.gen_batch(g, 0, n,
                                lambda s, c=cfg: workload.group_of(c, s))
        pts = len(hb.ts)
        eng.run(spec, hb)  # warm-up (staging allocation)
        t = time.perf_counter()
        reps = 3
        for _ in range(reps):
            eng.run(spec, hb)
        dt = (time.perf_counter() - t) / reps
        out[name] = {"series": n, "points": pts, "ms": dt * 1e3,
                     "value": pts / dt, "unit": "data points/s",
                     "bytes_h2d": 16 * pts}
        del hb
    return out


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
    dt, _ = timed_reps(lambda: workload.decode_cells_device(eng, cells, out=out),
                       1, reps)
    cb = cells.n_bytes
    del out
    torch.cuda.empty_cache()
    # the whole query straight from the cells: decode fused into the
    # downsample (otsdb_agg_run_cells_device)
    from opentsdb_amd.engine import DeviceResult
    spec = workload.query_spec(config)
    res = DeviceResult(torch, db.n_groups, db.n_groups * 2100, "cuda")
    read = stage_reader(eng)
    eng.lib.otsdb_prof_enable(eng.ctx, 1)
    read()
    dq, _ = timed_reps(
        lambda: workload.run_cells_device(eng, spec, cells, db, res), 1, reps)
    kb = read()[0] / 1e3
    # the same query from storage rows (otsdb_agg_run_raw_device): every
    # compacted row as the scanner returns it, through query-time compaction
    # (verbatim rows: copied), span assembly and the cells fold
    from opentsdb_amd import storage
    raw = storage.raw_rows_from_cells(cells)
    read_all = stage_reader(eng, all_stages=True)
    read_all()
    dr, _ = timed_reps(
        lambda: storage.run_raw_device(eng, spec, raw, db, res), 1, reps)
    st_raw = read_all()
    eng.lib.otsdb_prof_enable(eng.ctx, 0)
    del raw, cells
    torch.cuda.empty_cache()
    storage_fig = {
        "what": "the same C2 query from storage rows (otsdb_agg_run_raw_device"
                "): query-time compaction, span assembly, the cells fold",
        "value": n / dr, "unit": "data points/s", "ms_per_query": dr * 1e3,
        "stage_ms": {k: v for k, v in zip(STAGES, st_raw) if v},
        "kernels": "k_rows_uniform (+ k_rows_plan / k_rows_write for the rows "
                   "it cannot alias: compaction), k_span_plan "
                   "(assembly), k_cells_prep + k_fold<cells>"}
    fold_ms = st_raw[0]
    if fold_ms:
        storage_fig["fold_frac_of_8TBs"] = cb / (fold_ms / 1e3) / 8e12
    mixed = mixed_cells_figure(eng, config, n_series, db, res, reps)
    del res, db
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
                        "fused into the ordered group fold",
                "kernel": "k_fold<cells> (+ k_cells_prep)",
                "value": n / dq, "unit": "data points/s",
                "ms_per_query": dq * 1e3,
                "kernel_ms": kb * 1e3,
                "achieved_GBs_compacted": cb / kb / 1e9 if kb else None,
                "frac_of_8TBs": cb / kb / 8e12 if kb else None},
            "storage_rows": storage_fig,
            "mixed_resolution_cells": mixed}


def mixed_cells_figure(eng, config, n_series, db_groups, res, reps):
    """The same query over points half on whole seconds, half on
    milliseconds: the encoder writes 2-byte and 4-byte qualifiers, so every
    storage row mixes both (MS_MIXED_COMPACT, RowSeq.java:338-356): k_requal
    rewrites the qualifiers with one width (4-byte ms qualifiers; the value
    pool as it is), then the cells fold streams them."""
    import torch
    from opentsdb_amd import workload
    g = workload.gen_spec(config)
    g.flags = 0
    db = workload.generate_device(eng, g, 0, n_series, config=config)
    n = db.n_points_total
    # every other point on a whole second (10 s cadence: order kept): the
    # encoder gives those 2-byte qualifiers, the rest 4-byte ms ones
    even = db.ts[0::2]
    even -= torch.remainder(even, 1000)
    cells = workload.encode_cells_device(eng, db)
    del db, even
    torch.cuda.empty_cache()
    spec = workload.query_spec(config)
    read = stage_reader(eng, all_stages=True)
    # one untimed call first: its stage times include the rewrite buffer's
    # first allocation
    workload.run_cells_device(eng, spec, cells, db_groups, res)
    eng.lib.otsdb_prof_enable(eng.ctx, 1)
    read()
    dq, _ = timed_reps(
        lambda: workload.run_cells_device(eng, spec, cells, db_groups, res), 0,
        reps)
    st = read()
    eng.lib.otsdb_prof_enable(eng.ctx, 0)
    cb = cells.n_bytes
    del cells
    torch.cuda.empty_cache()
    out = {"what": "the C2 query over ms-stamped points from compacted cells "
                   "whose rows mix 2- and 4-byte qualifiers (qualifiers "
                   "rewritten with one width, then the cells fold)",
           "points": n, "compacted_bytes": cb, "value": n / dq,
           "unit": "data points/s", "ms_per_query": dq * 1e3,
           "stage_ms": {k: v for k, v in zip(STAGES, st) if v},
           "kernels": "k_requal (count + scan + write), k_cells_prep, "
                      "k_fold<cells>"}
    if st[7]:
        # k_requal reads the qualifier pool twice, writes 4 B a point
        out["requal_ms"] = st[7]
    return out


def host_cpus():
    """nproc, the CPUs this process may run on, and the CPU model."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return {"nproc": os.cpu_count() or 1, "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "cpu_model": model}


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
    # every host thread this process may use: its CPU affinity, bounded by
    # the box's per-GPU share (OMP_NUM_THREADS is set to it there; nproc and
    # os.cpu_count() report the whole machine)
    host = host_cpus()
    threads = host["affinity_cpus"]
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
    out["host"] = host
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
        # the whole host, for a node-level comparison: NOT measured (a GPU
        # box's share is its per-GPU slice of the cores); the measured
        # per-thread rate scaled linearly to every CPU, an upper bound for
        # an embarrassingly parallel per-group evaluation
        per_thread = pts / dtm / threads
        out["whole_host_projection"] = {
            "value": per_thread * host["nproc"], "cores": host["nproc"],
            "kind": "projection: measured %d-thread rate x %d / %d CPUs" % (
                threads, host["nproc"], threads)}
    return out


def dry_run(args, world, rank):
    """Launcher rehearsal for CPU tests: the same process-group setup,
    barrier-bracketed timing and max-over-ranks reduction, with a gloo
    all-reduce of a small tensor as the step."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    x = torch.ones(1024, dtype=torch.float64)
    step = (lambda: dist.all_reduce(x)) if world > 1 else (lambda: x.sum())
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    seen = dist.get_world_size() if world > 1 else 1
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit":
                          "data points/s", "n_gpus": world,
                          "ranks_seen": seen, "steps": args.steps,
                          "warmup": args.warmup,
                          "ms_per_step": el / max(args.steps, 1) * 1e3,
                          "dry_run": True}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (
            args.gpus, world))
    if args.dry_run:
        return dry_run(args, world, rank)

    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult, Engine, run_device

    # rehearsal knobs (a multi-rank run on a one-GPU box): every rank on
    # device 0 and gloo instead of RCCL; the driver's runs use neither
    if os.environ.get("OTSDB_BENCH_SAME_DEVICE"):
        local = 0
    backend = os.environ.get("OTSDB_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dist = None
    ranks_seen = 1
    # OTSDB_BENCH_SHARDED=1 at one rank: the cross-rank exchange path over a
    # world of one (RCCL), to time the protocol itself on a one-GPU box
    force_sharded = bool(os.environ.get("OTSDB_BENCH_SHARDED"))
    if force_sharded and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or force_sharded:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl",
                                    device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        ranks_seen = dist.get_world_size()
        assert ranks_seen == world == args.gpus

    cfg = workload.CONFIGS[args.config]
    n_series = args.series or workload.default_series_per_gpu(args.config)
    # groups that span ranks ({dc=*}, no group-by) take the cross-rank
    # exchange: partial all-gather of the shared groups, or the histogram
    # protocol for percentiles (opentsdb_amd/dist.py); host groups stay
    # rank-local
    sharded = (world > 1 or force_sharded) and workload.spans_ranks(args.config)
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
    spec = (named_spec(args.config) if args.named_query
            else workload.query_spec(args.config))
    sz = eng.plan(spec, db)
    res = DeviceResult(torch, db.n_groups, int(sz.max_out_points), "cuda")
    last = [None]
    if sharded:
        from opentsdb_amd import dist as odist

        def step():
            last[0] = odist.run_sharded_any(eng, spec, db, G_glob)
    else:
        def step():
            run_device(eng, spec, db, res)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # the timed steps run with stage timing OFF (no HIP events in the
    # pipeline); the per-stage kernel times come from a separate profiled
    # pass over the same steps afterwards
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    per_step = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        step()  # synchronous: the engine reads the device error word
        per_step.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    read = stage_reader(eng)
    eng.lib.otsdb_prof_enable(eng.ctx, 1)
    read()  # reset
    for _ in range(max(1, min(args.steps, 10))):
        step()
    torch.cuda.synchronize()
    stage_ms = read()
    eng.lib.otsdb_prof_enable(eng.ctx, 0)

    sel_counts = None
    if sharded and cfg["agg"] in ("p99", "p999", "median"):
        c = eng.counters()  # the last otsdb_sel_* session
        sel_counts = {"key_matrix_reads": c["sel_key_reads"],
                      "hist_passes": c["sel_passes"]}
    total_points = n_points * world
    out_points = (last[0].n_points() if sharded
                  else int(res.offsets[-1].item()))
    per_step.sort()
    med = per_step[len(per_step) // 2] if per_step else 0.0
    if dist:
        dev = "cuda" if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed, med], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, med = float(t[0].item()), float(t[1].item())
        tp = torch.tensor([n_points], dtype=torch.int64, device=dev)
        dist.all_reduce(tp)
        total_points = int(tp.item())
    step_s = elapsed / args.steps
    value = total_points / step_s

    # dominant kernel: the downsample stage streams every point once
    # (16 B/point) — k_fold on the fold path.  Rate and selection queries
    # run the row path: its roofline is priced over the whole on-device
    # pipeline (every stage: prep, downsample, transform, group / selection,
    # compact), with the downsample stage alone beside it
    row_path = bool(cfg["rate"]) or cfg["agg"] in ("p99", "p999", "median")
    kb_s = (sum(stage_ms[:5]) if row_path else stage_ms[0]) / 1e3
    kernel_achieved = (BYTES_PER_POINT * n_points / kb_s / 1e9
                       if kb_s > 0 else None)
    # the headline fraction: algorithmic bytes over the driver-timed step
    # (the whole query: every kernel, launch gaps and the read-back); the
    # dominant kernel's own HIP-event time is the secondary figure
    achieved = BYTES_PER_POINT * n_points / step_s / 1e9
    kernel = ("k_fold" if not row_path else
              "pipeline: k_prep + k_bucketize_k (rate-fused) + k_transform + "
              "k_group<MDev> + k_compact"
              if cfg["rate"] else
              "pipeline: k_prep + k_bucketize_k + k_keys_transpose + "
              "k_seg_select + k_compact")
    ds_stage = None
    if row_path and stage_ms[0] > 0:
        ds_stage = {"kernel": "k_bucketize_k", "ms": stage_ms[0],
                    "frac": BYTES_PER_POINT * n_points / (stage_ms[0] / 1e3)
                    / 1e9 / HBM_PEAK_GBS}
    # PMC traffic of this exact workload (scripts/gpu_pmc.sh, default size,
    # one GPU, the shipped kernels), per launch of the dominant kernel
    traffic = tinfo = None
    if not args.series and world == 1 and not args.named_query:
        tinfo = pmc_traffic(args.config)
        # HBM bytes of one whole query (every pipeline kernel, PMC), like
        # `achieved`; the dominant kernel's own beside it
        if tinfo:
            traffic = tinfo["step"] or tinfo["dominant_kernel"]

    extra = {}
    if rank == 0 and world == 1:
        if not args.no_cpu_baseline:
            extra["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        if not args.no_extra and args.config == "C2":
            extra["named_query"] = named_query_figure(eng, db, args.config)
        if not args.no_extra and args.config == "C5":
            extra["p999"] = p999_figure(eng, db, args.config)
        if not args.no_extra:
            extra["pcie_inclusive"] = pcie_figure(eng, args.config)

    n_groups, n_buckets = db.n_groups, int(sz.n_buckets)
    if world == 1 and not args.no_decode and args.config == "C2":
        del db, res
        torch.cuda.empty_cache()
        extra["decode"] = decode_figure(eng, args.config, n_series)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "data points/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": step_s * 1e3,
            "ms_per_step_median": med * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY §8d generator, seed 42, generated in "
                    "HBM; %d series x %d d @10s per GPU)" % (
                        n_series, cfg["days"]),
            "config": {
                "workload": workload_label(args.config, n_series),
                "points_per_gpu": n_points,
                "groups_per_gpu": n_groups,
                "buckets": n_buckets,
                "output_points_per_gpu": out_points,
                "parallelism": "series-sharded dp%d%s" % (
                    world, (" + %s exchange of shared groups" % (
                        "RCCL" if backend == "nccl" else backend))
                    if sharded else ""),
                "stage_ms": {"downsample": stage_ms[0],
                             "transform": stage_ms[1],
                             "group": stage_ms[2], "prep": stage_ms[3],
                             "compact": stage_ms[4]},
                "generate_s": t_gen,
                "sel_protocol": sel_counts,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kernel,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "timed_over": "ms_per_step (the whole query, per GPU)",
                "traffic": traffic,
                "traffic_pmc": tinfo,
                "algorithmic_bytes_per_launch": BYTES_PER_POINT * n_points,
                "kernel_ms": kb_s * 1e3,
                "kernel_achieved": kernel_achieved,
                "kernel_frac": (kernel_achieved / HBM_PEAK_GBS
                                if kernel_achieved else None),
            },
            "cpu_baseline": extra.get("cpu_baseline"),
        }
        if ds_stage:
            line["roofline"]["downsample_stage"] = ds_stage
        for k in ("named_query", "p999", "pcie_inclusive", "decode"):
            if k in extra:
                line[k] = extra[k]
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
