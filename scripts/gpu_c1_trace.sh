#!/bin/bash
# rocprofv3 kernel + memory-copy trace of the C1 bench (latency-bound: where
# a 0.23 ms query spends its time)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r5_c1_trace -o t \
  -- python3 -u bench.py --config C1 --steps 10 --no-cpu-baseline --no-extra --no-decode > gpurun_out/r5_c1_trace.log 2>&1 || { tail -5 gpurun_out/r5_c1_trace.log; exit 1; }
tail -1 gpurun_out/r5_c1_trace.log | cut -c1-200
