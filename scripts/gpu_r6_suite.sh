#!/bin/bash
# Round 6: the whole GPU suite, then the C2 cells probe (production build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  --durations=15 -s -m gpu tests/ ${PYTEST_ARGS} > gpurun_out/r6_gpu_suite.log 2>&1
r=$?; grep -E "max rel err|exact order" gpurun_out/r6_gpu_suite.log; tail -22 gpurun_out/r6_gpu_suite.log; [ $r -ne 0 ] && exit $r
[ -n "$NO_PROBE" ] && exit 0
NO_PMC=${NO_PMC} VARIANTS="prod ${VARIANTS}" bash scripts/gpu_r6_abl.sh
