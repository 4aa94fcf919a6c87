#!/bin/bash
# Round 6: the random parity sweeps over many seeds on the final build
# (general, rate, cells — the last through the uniform cells fold).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
N=${1:-10000}
NC=${2:-2000}
timeout -k 10 600 python -u scripts/sweep_many.py $N 0 0 > gpurun_out/r6_sweep_general.log 2>&1
r1=$?; tail -2 gpurun_out/r6_sweep_general.log; grep FAIL gpurun_out/r6_sweep_general.log | head
[ $r1 -gt 1 ] && exit $r1
timeout -k 10 500 python -u scripts/sweep_many.py 0 $N 0 > gpurun_out/r6_sweep_rate.log 2>&1
r2=$?; tail -2 gpurun_out/r6_sweep_rate.log; grep FAIL gpurun_out/r6_sweep_rate.log | head
[ $r2 -gt 1 ] && exit $r2
timeout -k 10 600 python -u scripts/sweep_cells.py $NC 0 > gpurun_out/r6_sweep_cells.log 2>&1
r3=$?; tail -2 gpurun_out/r6_sweep_cells.log; grep FAIL gpurun_out/r6_sweep_cells.log | head
exit $(( r1 | r2 | r3 ))
