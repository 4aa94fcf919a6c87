"""Builds tuning / debug variants of libotsdb_agg.so next to the production
library (opentsdb_amd/_build/var_<name>/), for A/B runs on the GPU box via
OTSDB_LIB.  Usage: python scripts/build_variants.py name=DEF[,DEF...] ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opentsdb_amd import build  # noqa: E402

for arg in sys.argv[1:]:
    name, _, defs = arg.partition("=")
    out = os.path.join(ROOT, "opentsdb_amd", "_build", "var_" + name,
                       "libotsdb_agg.so")
    build.build(force=True, defines=[d for d in defs.split(",") if d], out=out)
    print(out, flush=True)
