#!/bin/bash
# Round-4 evidence, two box calls (each within gpurun's limit):
#   PART=pmc   PMC traffic / instruction counts of the dominant kernels (C2
#              fold, C4 rate bucketize, the cells fold, the named query);
#   PART=bench every config's bench line, rocprofv3 kernel stats C2-C5 and
#              of the storage-row / mixed-width paths.
# Copy into profiles/ with `python scripts/collect_profiles.py r4`.
# Each step stops the chain at its first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${PART:-bench}" = pmc ]; then
  PMC_CFG=C2 PMC_PASSES="sq fetch write" bash scripts/gpu_pmc.sh > gpurun_out/pmc_c2.log 2>&1 || { tail -5 gpurun_out/pmc_c2.log; exit 1; }
  PMC_CFG=C4 PMC_PASSES="sq fetch write" bash scripts/gpu_pmc.sh > gpurun_out/pmc_c4.log 2>&1 || { tail -5 gpurun_out/pmc_c4.log; exit 1; }
  bash scripts/gpu_pmc_cells.sh > gpurun_out/pmc_cells.log 2>&1 || { tail -5 gpurun_out/pmc_cells.log; exit 1; }
  PMC_CFG=C2 PMC_TAG=_named PMC_BENCH_ARGS=--named-query PMC_PASSES="sq fetch write lds" bash scripts/gpu_pmc.sh > gpurun_out/pmc_named.log 2>&1 || { tail -5 gpurun_out/pmc_named.log; exit 1; }
  echo "pmc ok"
  exit 0
fi
NO_PROF=1 STEPS=10 CPU_S=${CPU_S:-10} bash scripts/gpu_bench_all.sh || exit $?
CONFIGS="C2 C3 C4 C5" bash scripts/gpu_kernel_stats.sh > gpurun_out/ks_all.log 2>&1 || { tail -5 gpurun_out/ks_all.log; exit 1; }
SERIES=100000 bash scripts/gpu_rows_prof.sh > gpurun_out/rows_prof.out 2>&1 || { tail -5 gpurun_out/rows_prof.out; exit 1; }
echo "kernel stats ok"
