#!/bin/bash
# Round 5: the GPU suite, then short benches of C1 and C2 (no extras).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  --durations=15 -m gpu tests/ > gpurun_out/r5_gpu_suite.log 2>&1
r=$?; tail -22 gpurun_out/r5_gpu_suite.log; [ $r -ne 0 ] && exit $r
for c in C1 C2; do
  timeout -k 10 200 python -u bench.py --config $c --steps 20 --warmup 3 \
    --no-cpu-baseline --no-extra --no-decode > gpurun_out/r5_q_$c.log 2>&1 || exit 1
  tail -1 gpurun_out/r5_q_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:3], 'ms/step %.4f med %.4f' % (d['ms_per_step'], d['ms_per_step_median']), 'frac %.3f kernel_frac %.3f' % (d['roofline']['frac'], d['roofline']['kernel_frac'] or 0), d['config']['stage_ms'])"
done
