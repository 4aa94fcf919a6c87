#!/bin/bash
# A/B of library variants (opentsdb_amd/_build/var_*/) on one bench config:
# VARIANTS="prod nowait ..." CONFIG=C2 bash scripts/gpu_ab_libs.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  timeout -k 10 240 python -u bench.py --config ${CONFIG:-C2} --steps ${STEPS:-10} --no-cpu-baseline --no-decode $EXTRA > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit $?
  python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
print("%-10s %8.3f ms/step  stage %s  frac %.3f" % (sys.argv[1], d["ms_per_step"],
      {k: round(v, 3) for k, v in d["config"]["stage_ms"].items() if v}, d["roofline"]["frac"]), flush=True)
PY
done
done
