#!/bin/bash
# Cells path: decode parity tests, then the C2 bench (decode + fused query).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dec.log 2>&1 \
  || { tail -40 gpurun_out/pytest_dec.log; exit 1; }
tail -1 gpurun_out/pytest_dec.log
timeout -k 10 300 python -u bench.py --config ${CFG:-C2} --steps 5 --no-cpu-baseline \
  > gpurun_out/bench_dec.log 2>&1 || { tail -20 gpurun_out/bench_dec.log; exit 1; }
grep '^{' gpurun_out/bench_dec.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('decode'), indent=1))"
