#!/bin/bash
# A/B of library variants (opentsdb_amd/_build/var_*/, "prod" = the
# production library) on one config's bench: stage times per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  timeout -k 10 240 python -u bench.py --config ${CFG:-C4} --steps 5 --warmup 2 --no-cpu-baseline \
    --no-extra --no-decode > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  grep '^{' gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '%.3f ms' % d['ms_per_step'], {k: round(v, 3) for k, v in d['config']['stage_ms'].items()})"
done
