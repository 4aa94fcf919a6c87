#!/bin/bash
# The random sweeps over many seeds (general 0..N-1, rate 0..N-1, cells).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
N=${1:-6500}
NC=${2:-1500}
timeout -k 10 500 python -u scripts/sweep_many.py $N 0 0 > gpurun_out/r4_sweep_general.log 2>&1
r1=$?; tail -2 gpurun_out/r4_sweep_general.log; grep FAIL gpurun_out/r4_sweep_general.log | head
[ $r1 -gt 1 ] && exit $r1
timeout -k 10 400 python -u scripts/sweep_many.py 0 $N 0 > gpurun_out/r4_sweep_rate.log 2>&1
r2=$?; tail -2 gpurun_out/r4_sweep_rate.log; grep FAIL gpurun_out/r4_sweep_rate.log | head
[ $r2 -gt 1 ] && exit $r2
timeout -k 10 250 python -u scripts/sweep_cells.py $NC 0 > gpurun_out/r4_sweep_cells.log 2>&1
r3=$?; tail -2 gpurun_out/r4_sweep_cells.log; grep FAIL gpurun_out/r4_sweep_cells.log | head
exit $(( r1 | r2 | r3 ))
