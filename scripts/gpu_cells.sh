#!/bin/bash
# Cells path: decode / fused-query parity tests, the rest of the GPU suite,
# then the C2 bench (decode + fused query figures).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_rows.py -m gpu -q \
  --maxfail=20 --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_dec.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_dec.log | grep -v "^  " | tail -25
[ $rc -eq 0 ] || exit $rc
if [ -z "$NO_FULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
    || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python -u bench.py --config ${CFG:-C2} --steps 5 --no-cpu-baseline --no-extra \
  > gpurun_out/bench_dec.log 2>&1 || { tail -20 gpurun_out/bench_dec.log; exit 1; }
grep '^{' gpurun_out/bench_dec.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('decode'), indent=1))"
