"""Builds libotsdb_agg.so (the HIP engine + C-ABI) for gfx950 in-tree.

hipcc cross-compiles without a GPU, so this runs in the CPU container; the
resulting .so travels to the GPU box with the repository snapshot.

The device code is split over translation units compiled in parallel: the
engine (host code, the non-template kernels and the aggregator-templated
ones) and two units per downsampling monoid (csrc/ds_tu.hip with
-DOTSDB_DS_MONOID=n: the downsample / ordered-fold kernels of that monoid,
and with -DOTSDB_DS_PART=1 the cells fold of that monoid).
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
DEPS = sorted(glob.glob(os.path.join(CSRC, "*.hip")) +
              glob.glob(os.path.join(CSRC, "*.h"))) + [
    os.path.join(ROOT, "include", "otsdb_agg.h")]
OUT_DIR = os.path.join(HERE, "_build")
OUT = os.path.join(OUT_DIR, "libotsdb_agg.so")
ARCH = os.environ.get("OTSDB_OFFLOAD_ARCH", "gfx950")
N_DS_MONOIDS = 12  # dispatch.h with_monoid: distinct reduction state types
HIPCC = "/opt/rocm/bin/hipcc"

FLAGS = [
    "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC",
    # Java rounds every multiply and add separately: no FMA contraction
    "-ffp-contract=off",
    "-Wall", "-Wno-unused-variable", "-Wno-unused-lambda-capture",
    "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result",
]


def up_to_date(out=OUT):
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def _units(out_dir, defines):
    d = ["-D" + x for x in defines]
    units = [(os.path.join(CSRC, "engine.hip"), d,
              os.path.join(out_dir, "engine.o"))]
    # part 1 (the cells fold, cellfold.hip) first: its units are the longest
    for part in (1, 0):
        for m in range(N_DS_MONOIDS):
            units.append((os.path.join(CSRC, "ds_tu.hip"),
                          d + ["-DOTSDB_DS_MONOID=%d" % m,
                               "-DOTSDB_DS_PART=%d" % part],
                          os.path.join(out_dir, "ds_%d_%d.o" % (part, m))))
    return units


def build(force=False, verbose=False, jobs=None, defines=(), out=None):
    """defines / out: a debug or tuning variant (extra -D flags) built into
    its own directory next to the production library."""
    out_dir = OUT_DIR
    if out:
        out_dir = os.path.dirname(out)
    OUT_ = out or OUT
    if not force and up_to_date(OUT_):
        return OUT_
    os.makedirs(out_dir, exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 1)

    def compile_unit(u):
        src, extra, obj = u
        cmd = [HIPCC] + FLAGS + extra + ["-c", "-o", obj + ".tmp", src]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           text=True)
        if r.returncode != 0:
            raise RuntimeError("compile failed: %s\n%s" % (" ".join(cmd),
                                                           r.stdout))
        if r.stdout.strip() and verbose:
            print(r.stdout, flush=True)
        os.replace(obj + ".tmp", obj)
        return obj

    units = _units(out_dir, defines)
    # incremental: a unit is rebuilt when a source it may include is newer
    # than its object (only part-1 units include cellfold.hip)
    # sources only engine.hip includes (ds_tu.hip's include graph:
    # kernels.hip, decode.hip, fold.hip, cellfold.hip and the headers)
    engine_only = ("engine.hip", "select.hip", "raw.hip", "rows.hip",
                   "calendar.hip", "compact.hip")

    def stale(u):
        src, extra, obj = u
        if force or not os.path.exists(obj):
            return True
        t = os.path.getmtime(obj)
        part1 = "-DOTSDB_DS_PART=1" in extra
        ds = src.endswith("ds_tu.hip")
        return any(os.path.getmtime(d) > t for d in DEPS
                   if (part1 or not d.endswith("cellfold.hip")) and
                   not (ds and os.path.basename(d) in engine_only))

    todo = [u for u in units if stale(u)]
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_unit, todo))
    objs = [u[2] for u in units]
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o",
           OUT_ + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(OUT_ + ".tmp", OUT_)
    return OUT_


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
