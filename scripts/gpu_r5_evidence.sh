#!/bin/bash
# Round-5 evidence, two box calls (each within gpurun's limit):
#   PART=pmc   PMC passes (fetch / write, + SQ where named) over every config
#              and the cells fold: HBM bytes per query and per dominant kernel;
#   PART=bench every config's bench line (CPU baseline included) and the
#              rocprofv3 --kernel-trace --stats summaries C1-C5.
# Copy into profiles/ with `python scripts/collect_profiles.py r5`.
# Each step stops the chain at its first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${PART:-bench}" = pmc ]; then
  for c in C1 C2 C3 C4 C5; do
    passes="fetch write"
    case $c in C2|C4|C5) passes="sq fetch write" ;; esac
    PMC_CFG=$c PMC_PASSES="$passes" bash scripts/gpu_pmc.sh > gpurun_out/pmc_$c.log 2>&1 || { tail -5 gpurun_out/pmc_$c.log; exit 1; }
    echo "pmc $c ok"
  done
  bash scripts/gpu_pmc_cells.sh > gpurun_out/pmc_cells.log 2>&1 || { tail -5 gpurun_out/pmc_cells.log; exit 1; }
  PMC_CFG=C2 PMC_TAG=_named PMC_BENCH_ARGS=--named-query PMC_PASSES="sq fetch write" bash scripts/gpu_pmc.sh > gpurun_out/pmc_named.log 2>&1 || { tail -5 gpurun_out/pmc_named.log; exit 1; }
  echo "pmc ok"
  exit 0
fi
NO_PROF=1 STEPS=20 CPU_S=${CPU_S:-10} bash scripts/gpu_bench_all.sh || exit $?
CONFIGS="C1 C2 C3 C4 C5" bash scripts/gpu_kernel_stats.sh > gpurun_out/ks_all.log 2>&1 || { tail -5 gpurun_out/ks_all.log; exit 1; }
echo "kernel stats ok"
