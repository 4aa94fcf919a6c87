#!/bin/bash
# decode / rows tests, then the C2 line's decode, fused-cells, storage-row and
# mixed-width figures
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_rows.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
timeout -k 10 400 python -u bench.py --config C2 --steps 3 --no-cpu-baseline --no-extra \
  > gpurun_out/bench_c2_dec.log 2>&1 || { tail -20 gpurun_out/bench_c2_dec.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_c2_dec.log").read().strip().splitlines()[-1])
dec = d["decode"]
print("decode ms %.2f fused %.2f storage %.2f mixed %.2f" % (
    dec["ms"], dec["fused_query"]["ms_per_query"],
    dec["storage_rows"]["ms_per_query"],
    dec["mixed_resolution_cells"]["ms_per_query"]))
PY
