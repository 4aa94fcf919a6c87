#!/bin/bash
# C2's bench line, its kernel stats, the storage-row / mixed-width kernel
# stats and the GPU suite (the rows of the final evidence a decode change
# touches)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
NO_PROF=1 CONFIGS=C2 STEPS=10 CPU_S=${CPU_S:-10} bash scripts/gpu_bench_all.sh > gpurun_out/bench_all.out 2>&1 || { tail -5 gpurun_out/bench_all.out; exit 1; }
CONFIGS="C2" bash scripts/gpu_kernel_stats.sh > gpurun_out/ks_all.log 2>&1 || { tail -5 gpurun_out/ks_all.log; exit 1; }
SERIES=100000 bash scripts/gpu_rows_prof.sh > gpurun_out/rows_prof.out 2>&1 || { tail -5 gpurun_out/rows_prof.out; exit 1; }
echo "kernel stats ok"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -1 gpurun_out/pytest_gpu.log
exit $rc
