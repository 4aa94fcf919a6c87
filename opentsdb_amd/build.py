"""Builds libotsdb_agg.so (the HIP engine + C-ABI) for gfx950 in-tree.

hipcc cross-compiles without a GPU, so this runs in the CPU container; the
resulting .so travels to the GPU box with the repository snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "engine.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in
        ("engine.hip", "kernels.hip", "kernels.h", "monoids.h", "select.hip",
         "decode.hip", "raw.hip")] + [
    os.path.join(ROOT, "include", "otsdb_agg.h")]
OUT_DIR = os.path.join(HERE, "_build")
OUT = os.path.join(OUT_DIR, "libotsdb_agg.so")
# tuning build: every k_bucketize variant compiled in (scripts/ab_bucketize.py)
OUT_VARIANTS = os.path.join(OUT_DIR, "libotsdb_agg_variants.so")
ARCH = os.environ.get("OTSDB_OFFLOAD_ARCH", "gfx950")

FLAGS = [
    "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
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


def build(force=False, verbose=False, variants=False):
    out = OUT_VARIANTS if variants else OUT
    if not force and up_to_date(out):
        return out
    flags = list(FLAGS)
    if variants:
        flags.append("-DOTSDB_BUCKETIZE_VARIANTS=1")
    os.makedirs(OUT_DIR, exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc"] + flags + ["-o", out + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True,
                variants="--variants" in sys.argv))
