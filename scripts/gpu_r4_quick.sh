#!/bin/bash
# Quick GPU check: the given test files, then the C2 bench (with the decode /
# storage-row / mixed-width figures) and the named query.  Each step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TESTS:-tests/test_gpu_decode.py}
timeout -k 10 600 python -u -m pytest $T -m gpu -q -x --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1 \
  || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || { tail -20 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('C2', d['ms_per_step'], d['roofline']['frac'])
dc=d.get('decode',{})
for k in ('fused_query','storage_rows','mixed_resolution_cells'):
    x=dc.get(k,{}); print(k, x.get('ms_per_query'), x.get('stage_ms'))
print('named', json.dumps(d.get('named_query',{}))[:400])
"
timeout -k 10 300 python -u bench.py --steps 10 --named-query --no-cpu-baseline --no-extra --no-decode > gpurun_out/bench_named.log 2>&1 || { tail -20 gpurun_out/bench_named.log; exit 1; }
tail -1 gpurun_out/bench_named.log | cut -c1-600
