#!/bin/bash
# rocprofv3 kernel stats of the mixed-width cells query (scripts/rows_probe.py --mixed)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_mixed -o ks \
  -- python3 -u scripts/rows_probe.py --series ${SERIES:-100000} --mixed > gpurun_out/ks_mixed.log 2>&1 || { tail -20 gpurun_out/ks_mixed.log; exit 1; }
tail -1 gpurun_out/ks_mixed.log
head -14 $(find gpurun_out/ks_mixed -name '*kernel_stats.csv' | head -1) | cut -d, -f1-8 | cut -c1-200
