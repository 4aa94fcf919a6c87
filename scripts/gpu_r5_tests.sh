#!/bin/bash
# The whole GPU suite (round 5), then the new large-dev tests' timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  --durations=15 -m gpu tests/ > gpurun_out/r5_gpu_suite.log 2>&1
r=$?; tail -25 gpurun_out/r5_gpu_suite.log; exit $r
