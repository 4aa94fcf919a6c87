#!/bin/bash
# SQ counters of the storage-row path (scripts/rows_probe.py), one pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/pmc_rows
mkdir -p "$OUT"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv \
  -d "$OUT/sq" -o sq -- python3 -u scripts/rows_probe.py --series ${SERIES:-20000} --reps 1 ${ARGS} > "$OUT/sq.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU \
  SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --output-format csv \
  -d "$OUT/sq2" -o sq2 -- python3 -u scripts/rows_probe.py --series ${SERIES:-20000} --reps 1 ${ARGS} > "$OUT/sq2.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import collections, csv, glob, os, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        acc[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "otsdb" not in k:
        continue
    print(k, {c: "%.3g" % (sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
