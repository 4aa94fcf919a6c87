#!/bin/bash
# Rate-fused k_bucketize_k at 3 (140 VGPRs) vs 4 waves / SIMD (128 VGPRs,
# launch bound): the GPU parity tests with the 4-wave variant, then the C4
# bench interleaved (same box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
OTSDB_RATE_WAVES=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rw.log 2>&1 \
  || { tail -40 gpurun_out/pytest_rw.log; exit 1; }
tail -1 gpurun_out/pytest_rw.log
for w in ${RWS:-1 4 1 4}; do
  OTSDB_RATE_WAVES=$w timeout -k 10 300 python -u bench.py --config C4 --steps 10 \
    --no-cpu-baseline > gpurun_out/bench_rw_$w.log 2>&1 || { tail -20 gpurun_out/bench_rw_$w.log; exit 1; }
  grep '^{' gpurun_out/bench_rw_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('waves=$w', round(d['value']/1e9,1), round(d['ms_per_step'],3), d['config']['stage_ms'])"
done
