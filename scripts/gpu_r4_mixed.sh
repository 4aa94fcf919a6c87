#!/bin/bash
# Mixed-width cells: the decode tests, then rocprofv3 kernel stats of the
# mixed-width query (scripts/rows_probe.py --mixed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -m gpu -q -x --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1 \
  || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -1 gpurun_out/pytest_quick.log
bash scripts/gpu_mixed_prof.sh > gpurun_out/mixed_prof.out 2>&1 || { tail -20 gpurun_out/mixed_prof.out; exit 1; }
grep "mixed cells" gpurun_out/ks_mixed.log
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/ks_mixed/**/*kernel_trace.csv', recursive=True)[0]
seen = {}
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    if any(k in n for k in ('requal', 'k_fold<', 'cells_prep')):
        seen.setdefault(n[:60], []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for k, v in seen.items():
    print(k, ['%.2f' % x for x in v[-4:]])
PY
