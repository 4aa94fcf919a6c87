#!/bin/bash
# PMC passes over the mixed-width query (k_requal, the cells fold)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/rq_pmc
mkdir -p $OUT
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$n -o p \
    -- python3 -u scripts/rows_probe.py --series ${SERIES:-100000} --mixed --reps 1 > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; exit 1; }
}
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || exit 1
run lds SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM || exit 1
python3 - $OUT <<'PY'
import collections, csv, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        n = r['Kernel_Name']
        if 'requal' in n or 'k_fold<' in n:
            acc[n[:40]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in acc.items():
    print(k, {c: '%.4g' % (sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
