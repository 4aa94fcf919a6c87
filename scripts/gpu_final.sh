#!/bin/bash
# End-of-round measurement set: every config's bench line (CPU baseline
# included), rocprofv3 --kernel-trace --stats per config, PMC traffic of
# the C2 headline and of the cells fold.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
NO_PROF=1 STEPS=10 CPU_S=${CPU_S:-10} bash scripts/gpu_bench_all.sh || exit $?
CONFIGS="C2 C3 C4 C5" bash scripts/gpu_kernel_stats.sh > gpurun_out/ks_all.log 2>&1 || { tail -5 gpurun_out/ks_all.log; exit 1; }
echo "kernel stats ok"
[ -n "$NO_PMC" ] && exit 0
PMC_CFG=C2 PMC_PASSES="sq fetch write" bash scripts/gpu_pmc.sh > gpurun_out/pmc_c2.log 2>&1 || { tail -5 gpurun_out/pmc_c2.log; exit 1; }
echo "pmc C2 ok"
bash scripts/gpu_pmc_cells.sh > gpurun_out/pmc_cells.log 2>&1 || { tail -5 gpurun_out/pmc_cells.log; exit 1; }
echo "pmc cells ok"
