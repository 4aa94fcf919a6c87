#!/bin/bash
# Round-6 evidence, two box calls (each within gpurun's limit):
#   PART=pmc   PMC passes (fetch / write, + SQ where named) over every config,
#              the cells fold and the named query: HBM bytes per query and per
#              dominant kernel (collect them into profiles/ before PART=bench:
#              bench.py reads the latest round's traffic from there);
#   PART=bench in ONE session: every config's bench line (CPU baseline
#              included), then the rocprofv3 --kernel-trace --stats summaries
#              of the same configs, and C5 through the cross-rank protocol at
#              a world of one (bench line + kernel stats).
# Copy into profiles/ with `python scripts/collect_profiles.py r6`.
# Each step stops the chain at its first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ "${PART:-bench}" = pmc ]; then
  for c in ${CONFIGS:-C1 C2 C3 C4 C5}; do
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
OTSDB_BENCH_SHARDED=1 timeout -k 10 300 python3 -u bench.py --config C5 --steps 20 \
  --no-cpu-baseline --no-extra > gpurun_out/bench_C5_sharded.log 2>&1 || exit $?
tail -1 gpurun_out/bench_C5_sharded.log
OTSDB_BENCH_SHARDED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/ks_C5_sharded -o ks -- python3 -u bench.py --config C5 --steps 5 \
  --warmup 2 --no-cpu-baseline --no-extra --no-decode > gpurun_out/ks_C5_sharded.log 2>&1 || exit $?
echo "sharded C5 ok"
