#!/bin/bash
# the GPU test suite, then the C5 bench line (and C3 as a fold control)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for cfg in ${CONFIGS:-C5}; do
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --no-cpu-baseline --no-extra \
  > gpurun_out/bench_q_$cfg.log 2>&1 || { tail -20 gpurun_out/bench_q_$cfg.log; exit 1; }
python3 - $cfg <<'PY'
import json, sys
d = json.loads(open("gpurun_out/bench_q_%s.log" % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], round(d["ms_per_step"], 3), "ms", {k: round(v, 3) for k, v in d["config"]["stage_ms"].items() if v}, "frac", round(d["roofline"]["frac"], 3))
PY
done
