#!/bin/bash
# rocprofv3 kernel stats of the storage-row path and the mixed-width decode
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
SER=${SERIES:-20000}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_rows -o ks \
  -- python3 -u scripts/rows_probe.py --series $SER > gpurun_out/ks_rows.log 2>&1 || { tail -20 gpurun_out/ks_rows.log; exit 1; }
tail -1 gpurun_out/ks_rows.log
head -12 $(find gpurun_out/ks_rows -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4 | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_mixed -o ks \
  -- python3 -u scripts/rows_probe.py --series $SER --mixed > gpurun_out/ks_mixed.log 2>&1 || { tail -20 gpurun_out/ks_mixed.log; exit 1; }
tail -1 gpurun_out/ks_mixed.log
head -12 $(find gpurun_out/ks_mixed -name '*kernel_stats.csv' | head -1) | cut -d, -f1-4 | cut -c1-160
