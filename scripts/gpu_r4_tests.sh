#!/bin/bash
# GPU-box test run (round 4): the GPU suite (or the files given), smoke, a
# short bench.  Each GPU step has its own time limit; the chain stops at
# the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${*:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -v --timeout 120 \
  --timeout-method thread --maxfail=40 -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
exit $rc
