#!/bin/bash
# GPU-box: the parity suite (or the tests named in $TESTS), then a short C2
# bench.  Each GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 \
  --timeout-method thread --maxfail=${MAXFAIL:-20} -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py $BENCH > gpurun_out/bench.log 2>&1 || exit $?
  tail -1 gpurun_out/bench.log
fi
exit $rc
