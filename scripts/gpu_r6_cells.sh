#!/bin/bash
# Round 6: the cells-path GPU tests (decode, fused cells queries incl. the
# uniform kernel, storage rows, the cells sweep), then the C2 cells probe
# and an SQ PMC pass over it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_decode.py tests/test_gpu_rows.py "tests/test_gpu_sweep.py::test_random_cells_sweep" \
  > gpurun_out/r6_cells_tests.log 2>&1
r=$?; tail -15 gpurun_out/r6_cells_tests.log; [ $r -ne 0 ] && exit $r
[ -n "$NO_PROBE" ] && exit 0
NO_PMC=${NO_PMC} SERIES=100000 bash scripts/gpu_pmc_cells.sh || exit $?
