#!/bin/bash
# Round 5: parity tests, then short benches of C1, C2, C3 (no extras).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_fullsize.py \
  tests/test_gpu_fillins.py > gpurun_out/r5_tests3.log 2>&1
r=$?; tail -2 gpurun_out/r5_tests3.log; [ $r -ne 0 ] && exit $r
for c in ${CONFIGS:-C1 C2 C3}; do
  timeout -k 10 200 python -u bench.py --config $c --steps 20 --warmup 3 \
    --no-cpu-baseline --no-extra --no-decode > gpurun_out/r5_q_$c.log 2>&1 || exit 1
  tail -1 gpurun_out/r5_q_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:3], 'ms/step %.4f med %.4f' % (d['ms_per_step'], d['ms_per_step_median']), 'frac %.3f kernel_frac %.3f' % (d['roofline']['frac'], d['roofline']['kernel_frac'] or 0), {k: round(v, 4) for k, v in d['config']['stage_ms'].items()})"
done
