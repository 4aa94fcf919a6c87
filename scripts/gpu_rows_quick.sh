#!/bin/bash
# rows tests + the C2 bench line with its decode / storage-row figures
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/rows_tests.log 2>&1 || { tail -30 gpurun_out/rows_tests.log; exit 1; }
tail -2 gpurun_out/rows_tests.log
timeout -k 10 400 python -u bench.py --config C2 --steps 5 --no-cpu-baseline --no-extra ${BENCH_ARGS} \
  > gpurun_out/bench_c2_dec.log 2>&1 || { tail -20 gpurun_out/bench_c2_dec.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_c2_dec.log").read().strip().splitlines()[-1])
dec = d.get("decode", {})
print("C2", round(d["ms_per_step"], 3), "ms; decode", round(dec.get("ms", 0), 2))
for k in ("fused_query", "storage_rows", "mixed_resolution_cells"):
    x = dec.get(k, {})
    print(k, round(x.get("ms_per_query", 0), 2), x.get("stage_ms"))
PY
