#!/bin/bash
# A/B of library variants on the metric's named query (sum:1m-avg LERP over
# C2's series) and the C2 line: VARIANTS="prod fl64" bash scripts/gpu_ab_named.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  for mode in named plain; do
    extra=""; [ $mode = named ] && extra="--named-query"
    timeout -k 10 240 python -u bench.py --config C2 $extra --steps 10 --no-cpu-baseline --no-decode --no-extra > gpurun_out/abn_${v}_$mode.json 2>gpurun_out/abn_${v}_$mode.err || { tail -5 gpurun_out/abn_${v}_$mode.err; exit 1; }
    python3 - "$v" "$mode" <<'PY'
import json, sys
v, mode = sys.argv[1:]
d = json.loads(open("gpurun_out/abn_%s_%s.json" % (v, mode)).read().strip().splitlines()[-1])
print("%-6s %-6s %8.3f ms/step  stage %s" % (v, mode, d["ms_per_step"],
      {k: round(x, 3) for k, x in d["config"]["stage_ms"].items() if x}), flush=True)
PY
  done
done
