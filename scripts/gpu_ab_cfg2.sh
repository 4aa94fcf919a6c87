#!/bin/bash
# A/B of library variants on one config's bench line:
# VARIANTS="prod k8" CFG=C5 bash scripts/gpu_ab_cfg2.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  timeout -k 10 240 python -u bench.py --config ${CFG:-C5} --steps 10 --no-cpu-baseline --no-decode --no-extra > gpurun_out/abcfg_$v.json 2>gpurun_out/abcfg_$v.err || { tail -5 gpurun_out/abcfg_$v.err; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open("gpurun_out/abcfg_%s.json" % v).read().strip().splitlines()[-1])
print("%-6s %8.3f ms/step  stage %s  frac %.3f" % (v, d["ms_per_step"],
      {k: round(x, 3) for k, x in d["config"]["stage_ms"].items() if x}, d["roofline"]["frac"]), flush=True)
PY
done
