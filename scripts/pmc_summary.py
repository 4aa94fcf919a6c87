"""Summarise rocprofv3 --pmc csv passes (scripts/gpu_pmc.sh) per kernel:
mean counter value per dispatch.  FETCH_SIZE is reported raw (KB, as
rocprofv3 derives it) and corrected (x2 for gfx950 wide streaming reads,
MI355X_MICROARCH.md "HBM")."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    name = name.split("(")[0]
    for key in ("k_fold_prep", "k_fold", "k_bucketize_k", "k_bucketize",
                "k_transform", "k_group",
                "k_combine", "k_compact", "k_prep", "k_gen"):
        if key in name:
            i = name.find("<")
            return key + (name[i:i + 60] if i >= 0 else "")
    return name[:80]


def main(root):
    # per kernel, only the dispatches of its largest grid: the bench's
    # secondary figures launch the same kernels at smaller sizes, which
    # would skew the per-launch mean of the workload's own dispatches
    rows = []
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"),
                          recursive=True):
        with open(path) as f:
            rows.extend(csv.DictReader(f))
    grid = collections.defaultdict(int)
    for row in rows:
        k = row.get("Kernel_Name", "")
        grid[k] = max(grid[k], int(row.get("Grid_Size") or 0))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in rows:
        k = row.get("Kernel_Name", "")
        if int(row.get("Grid_Size") or 0) != grid[k]:
            continue
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    # every kernel of the query pipeline (not the generator's, not the
    # runtime's fills / copies): the HBM bytes of one whole query (per step)
    step = 0.0
    step_k = []
    for k, cs in acc.items():
        if ("k_gen" in k or "rocclr" in k or "at::native" in k or "rocprim" in k
                or "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs):
            continue
        rd = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
        wr = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
        step += rd + wr
        step_k.append(short(k))
    for k, cs in acc.items():
        if ("bucketize" not in k and "k_fold" not in k
                and "k_decode" not in k):
            continue
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        out[k[:160]] = d
    # the figure bench.py reports as roofline.traffic: HBM bytes (read,
    # corrected, + written) per launch of the dominant kernel (the most
    # downsample / fold variant moving the most bytes)
    best_k = max(out, key=lambda k: out[k].get("FETCH_SIZE", 0), default=None)
    best = out.get(best_k, {})
    if "hbm_read_bytes_corrected" in best and "hbm_write_bytes" in best:
        out = {"hbm_bytes_per_launch":
               best["hbm_read_bytes_corrected"] + best["hbm_write_bytes"],
               "kernel": best_k, "kernels": out}
    out["step_hbm_bytes"] = step
    out["step_kernels"] = sorted(step_k)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
