#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_bucketize.py ${AB_ARGS} > gpurun_out/ab.log 2>&1 || exit $?
tail -1 gpurun_out/ab.log
