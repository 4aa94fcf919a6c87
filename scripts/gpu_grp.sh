#!/bin/bash
# Group-fused zimsum (k_bucketize_group): every GPU parity test, then the C2
# bench with the fused kernel off / on / off / on (same box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_grp.log 2>&1 \
  || { tail -40 gpurun_out/pytest_grp.log; exit 1; }
tail -1 gpurun_out/pytest_grp.log
for f in 0 1 0 1; do
  OTSDB_GRP_FUSED=$f timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline \
    > gpurun_out/bench_grp_$f.log 2>&1 || { tail -20 gpurun_out/bench_grp_$f.log; exit 1; }
  grep '^{' gpurun_out/bench_grp_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused=$f', round(d['value']/1e9,1), round(d['ms_per_step'],3), d['config']['stage_ms'])"
done
