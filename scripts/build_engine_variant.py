"""An engine-only tuning variant: engine.hip compiled with extra -D flags and
linked with the production build's downsampling objects (for knobs that only
engine.hip's kernels read, e.g. compact.hip's).  Usage:
python scripts/build_engine_variant.py name=DEF[,DEF...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opentsdb_amd import build  # noqa: E402

build.build()  # production objects up to date
for arg in sys.argv[1:]:
    name, _, defs = arg.partition("=")
    d = os.path.join(build.OUT_DIR, "var_" + name)
    os.makedirs(d, exist_ok=True)
    eng = os.path.join(d, "engine.o")
    subprocess.check_call([build.HIPCC] + build.FLAGS +
                          ["-D" + x for x in defs.split(",") if x] +
                          ["-c", "-o", eng,
                           os.path.join(build.CSRC, "engine.hip")])
    objs = [eng] + [u[2] for u in build._units(build.OUT_DIR, ())[1:]]
    out = os.path.join(d, "libotsdb_agg.so")
    subprocess.check_call([build.HIPCC, "--offload-arch=" + build.ARCH,
                           "-shared", "-fPIC", "-o", out] + objs)
    print(out, flush=True)
