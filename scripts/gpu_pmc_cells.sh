#!/bin/bash
# Cells path: probe timing, then SQ / fetch PMC passes over k_bucketize_cells
# (one counter group per run, as MI355X_MICROARCH.md prescribes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/pmc_cells
mkdir -p "$OUT"
SER=${SERIES:-100000}
timeout -k 10 200 python3 -u scripts/cells_probe.py --series $SER > "$OUT/probe.log" 2>&1 \
  || { tail -20 "$OUT/probe.log"; exit 1; }
tail -1 "$OUT/probe.log"
[ -n "$NO_PMC" ] && exit 0
run_pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv \
    -d "$OUT/$name" -o "$name" -- \
    python3 -u scripts/cells_probe.py --series $SER --reps 1 > "$OUT/$name.log" 2>&1
}
run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU || exit $?
run_pass sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM || exit $?
run_pass fetch FETCH_SIZE || exit $?
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.json" || exit $?
cat "$OUT/summary.json"
