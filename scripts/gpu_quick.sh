#!/bin/bash
# GPU parity tests, then each CONFIGS bench (no CPU baseline), one line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 \
    || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
for cfg in ${CONFIGS:-C1 C2 C3 C4 C5}; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-10} \
    --no-cpu-baseline > gpurun_out/q_$cfg.log 2>&1 || { tail -20 gpurun_out/q_$cfg.log; exit 1; }
  grep '^{' gpurun_out/q_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', '%.4g pts/s' % d['value'], '%.3f ms' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'], {k: round(v, 3) for k, v in d['config']['stage_ms'].items()})"
done
