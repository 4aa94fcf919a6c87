"""Tuning builds for A/B runs: the production objects with only the units
a workload uses recompiled with extra -D flags (default ds_1_1.o: the cells
fold of the avg downsampler, C2 from cells; OTSDB_UNITS=2_0 for C4's rate
fold of the sum downsampler; OTSDB_UNITS=engine for the engine unit alone:
k_requal, the decode / row kernels), linked into opentsdb_amd/_build/var_<name>/.
Usage: [OTSDB_UNITS=part_monoid|engine,...] python scripts/build_cells_variant.py
name=DEF[,DEF...] ..."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opentsdb_amd import build  # noqa: E402

if not os.environ.get("OTSDB_NO_PROD_BUILD"):
    build.build()  # production objects up to date


UNITS = os.environ.get("OTSDB_UNITS", "1_1").split(",")


def one(arg):
    name, _, defs = arg.partition("=")
    d = os.path.join(ROOT, "opentsdb_amd", "_build", "var_" + name)
    os.makedirs(d, exist_ok=True)
    for u in UNITS:
        if u == "engine":
            subprocess.check_call(
                [build.HIPCC] + build.FLAGS +
                ["-D" + x for x in defs.split(",") if x] +
                ["-c", "-o", os.path.join(d, "engine.o"),
                 os.path.join(build.CSRC, "engine.hip")])
            continue
        part, mono = u.split("_")
        subprocess.check_call(
            [build.HIPCC] + build.FLAGS +
            ["-D" + x for x in defs.split(",") if x] +
            ["-DOTSDB_DS_MONOID=" + mono, "-DOTSDB_DS_PART=" + part, "-c",
             "-o", os.path.join(d, "ds_%s.o" % u),
             os.path.join(build.CSRC, "ds_tu.hip")])
    objs = [os.path.join(d, os.path.basename(u[2]))
            if (os.path.basename(u[2])[3:-2] in UNITS or
                (os.path.basename(u[2]) == "engine.o" and "engine" in UNITS))
            else u[2]
            for u in build._units(build.OUT_DIR, [])]
    out = os.path.join(d, "libotsdb_agg.so")
    subprocess.check_call([build.HIPCC, "--offload-arch=" + build.ARCH,
                           "-shared", "-fPIC", "-o", out] + objs)
    return out


with ThreadPoolExecutor(8) as ex:
    for out in ex.map(one, sys.argv[1:]):
        print(out, flush=True)
