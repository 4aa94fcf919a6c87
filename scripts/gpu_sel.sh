#!/bin/bash
# Percentile path: the selection parity tests (large groups, full-size C5,
# sharded), then the C5 bench under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider \
  -k "percentile or selection or C5 or median or pct" > gpurun_out/pytest_sel.log 2>&1 \
  || { tail -40 gpurun_out/pytest_sel.log; exit 1; }
tail -1 gpurun_out/pytest_sel.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/prof_sel" -o run -- python3 -u "$R/bench.py" \
  --config C5 --steps 5 --no-cpu-baseline > gpurun_out/bench_C5_sel.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_C5_sel.log | tail -1 | cut -c1-400
python3 scripts/prof_summary.py gpurun_out/prof_sel/run_kernel_stats.csv > gpurun_out/prof_sel/summary.txt && head -12 gpurun_out/prof_sel/summary.txt
