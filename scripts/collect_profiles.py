"""Copies one evidence run's results (scripts/gpu_r5_evidence.sh, merged into
gpurun_out/) into profiles/ under a round tag: bench lines, rocprofv3
kernel-stats summaries, PMC summaries, the storage-row / mixed-width kernel
stats and the GPU test summary.  Usage: python scripts/collect_profiles.py r3"""
import glob
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def last_json_line(path):
    with open(path) as f:
        lines = [x for x in f.read().splitlines() if x.startswith("{")]
    return lines[-1] if lines else None


def first(pattern):
    m = sorted(glob.glob(os.path.join(OUT, pattern), recursive=True))
    return m[0] if m else None


def main(tag):
    done = []
    for cfg in ("C1", "C2", "C3", "C4", "C5"):
        p = os.path.join(OUT, "bench_%s.log" % cfg)
        if os.path.exists(p):
            line = last_json_line(p)
            if line:
                dst = os.path.join(PROF, "%s_bench_%s.json" % (tag, cfg))
                with open(dst, "w") as f:
                    f.write(line + "\n")
                done.append(dst)
        ks = first("ks_%s/**/*kernel_stats.csv" % cfg)
        if ks:
            dst = os.path.join(PROF, "%s_%s_kernel_stats.csv" % (tag, cfg))
            shutil.copy(ks, dst)
            done.append(dst)
    for name, src in (("pmc_C1.json", "pmc_C1/summary.json"),
                      ("pmc_C2.json", "pmc_C2/summary.json"),
                      ("pmc_C3.json", "pmc_C3/summary.json"),
                      ("pmc_C4.json", "pmc_C4/summary.json"),
                      ("pmc_C5.json", "pmc_C5/summary.json"),
                      ("pmc_cells_C2.json", "pmc_cells/summary.json"),
                      ("pmc_C2_named.json", "pmc_C2_named/summary.json")):
        p = os.path.join(OUT, src)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(PROF, "%s_%s" % (tag, name)))
            done.append(name)
    for what in ("rows", "mixed"):
        ks = first("ks_%s/**/*kernel_stats.csv" % what)
        if ks:
            dst = os.path.join(PROF, "%s_%s_kernel_stats.csv" % (tag, what))
            shutil.copy(ks, dst)
            done.append(dst)
    for cfg in ("C5",):  # the cross-rank protocol at a world of one
        p = os.path.join(OUT, "bench_%s_sharded.log" % cfg)
        if os.path.exists(p):
            line = last_json_line(p)
            if line:
                dst = os.path.join(PROF, "%s_bench_%s_sharded.json" % (tag, cfg))
                with open(dst, "w") as f:
                    f.write(line + "\n")
                done.append(dst)
        ks = first("ks_%s_sharded/**/*kernel_stats.csv" % cfg)
        if ks:
            dst = os.path.join(PROF, "%s_%s_sharded_kernel_stats.csv" % (tag, cfg))
            shutil.copy(ks, dst)
            done.append(dst)
    p = os.path.join(OUT, "%s_gpu_suite.log" % tag)
    if os.path.exists(p):
        with open(p) as f:
            tail = f.read().splitlines()[-3:]
        with open(os.path.join(PROF, "%s_gpu_tests_summary.txt" % tag), "w") as f:
            f.write("\n".join(tail) + "\n")
        done.append("gpu tests summary")
    print("\n".join(done))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r3")
