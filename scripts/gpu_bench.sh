#!/bin/bash
# Full-size bench (C2 on one MI355X) + rocprofv3 kernel trace of the same run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --steps 20 ${BENCH_ARGS} > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/prof_c2" -o run -- python -u "$R/bench.py" --steps 10 \
  --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_c2_prof.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2_prof.log
find gpurun_out/prof_c2 -name "*stats*" | head
