#!/bin/bash
# Round-3 evidence set at HEAD: every config's bench line, kernel stats
# C2-C5, PMC traffic of C2 / C4 / the cells fold.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NO_PMC=1 bash scripts/gpu_final.sh || exit $?
PMC_CFG=C4 PMC_PASSES="sq fetch write" bash scripts/gpu_pmc.sh > gpurun_out/pmc_c4.log 2>&1 || { tail -5 gpurun_out/pmc_c4.log; exit 1; }
echo "pmc C4 ok"
PMC_CFG=C2 PMC_PASSES="sq fetch write" bash scripts/gpu_pmc.sh > gpurun_out/pmc_c2.log 2>&1 || { tail -5 gpurun_out/pmc_c2.log; exit 1; }
echo "pmc C2 ok"
bash scripts/gpu_pmc_cells.sh > gpurun_out/pmc_cells.log 2>&1 || { tail -5 gpurun_out/pmc_cells.log; exit 1; }
echo "pmc cells ok"
