#!/bin/bash
# A/B of library variants (opentsdb_amd/_build/var_*/) on the fused cells
# query of the C2 bench's decode figure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  timeout -k 10 240 python -u bench.py --config C2 --steps 1 --warmup 0 --no-cpu-baseline --no-extra > gpurun_out/abc_$v.json 2>gpurun_out/abc_$v.err || exit $?
  python - "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abc_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
f = d["decode"]["fused_query"]
print("%-10s cells kernel %8.2f ms  query %8.2f ms" % (sys.argv[1], f["kernel_ms"], f["ms_per_query"]), flush=True)
PY
done
