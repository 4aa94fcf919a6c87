#!/bin/bash
# one box: the GPU test suite, then the prefetch A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_tests.sh > gpurun_out/tests.out 2>&1
rc=$?
tail -4 gpurun_out/tests.out
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VARIANTS="prod pf1 pf2" bash scripts/gpu_ab_pf.sh || exit $?
exit $rc
