#!/bin/bash
# GPU-box test run: parity tests, smoke, a short bench.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 \
  --timeout-method thread --maxfail=30 -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --series ${BENCH_SERIES:-20000} --steps 10 \
  --cpu-seconds 3 > gpurun_out/bench_small.log 2>&1 || exit $?
tail -1 gpurun_out/bench_small.log
exit $rc
