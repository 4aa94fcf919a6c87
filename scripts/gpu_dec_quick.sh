#!/bin/bash
# decode tests + the mixed-width decode timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_rows.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
timeout -k 10 200 python3 -u scripts/rows_probe.py --series ${SERIES:-100000} --mixed > gpurun_out/mixed_probe.log 2>&1 || { tail -5 gpurun_out/mixed_probe.log; exit 1; }
tail -1 gpurun_out/mixed_probe.log
