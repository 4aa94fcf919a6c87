#!/bin/bash
# k_requal A/B over engine variants (opentsdb_amd/_build/var_<name>): the
# decode tests on prod, then rocprofv3 kernel traces of the mixed-width query
# per variant.  VARIANTS="prod a b"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/rq_ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -m gpu -q -x --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1 \
  || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -1 gpurun_out/pytest_quick.log
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then L=opentsdb_amd/_build/libotsdb_agg.so; else L=opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  OTSDB_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rq_ab/$v -o t \
    -- python3 -u scripts/rows_probe.py --series ${SERIES:-100000} --mixed > gpurun_out/rq_ab/$v.log 2>&1 || { tail -20 gpurun_out/rq_ab/$v.log; exit 1; }
  python3 - gpurun_out/rq_ab/$v "$v" "$(grep 'mixed cells' gpurun_out/rq_ab/$v.log | sed 's/.*GB: //;s/;.*//')" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
seen = {}
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    for k in ('k_requal<0>', 'k_requal<1>'):
        if k in n:
            seen.setdefault(k, []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
print(sys.argv[2], sys.argv[3], {k: round(sorted(v)[len(v) // 2], 3) for k, v in seen.items()})
PY
done
