#!/bin/bash
# PMC passes over the k_bucketize A/B script (one counter group per run, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes).  PMC_KS picks the
# variants (OTSDB_BUCKETIZE_K values), PMC_CFG the workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
KS=${PMC_KS:-0}
CFG=${PMC_CFG:-C2}
OUT=gpurun_out/pmc_${CFG}
mkdir -p "$OUT"
run_pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv \
    -d "$OUT/$name" -o "$name" -- \
    python3 -u scripts/ab_bucketize.py --config "$CFG" --ks "$KS" --rounds 1 \
    --reps 2 > "$OUT/$name.log" 2>&1
}
run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU || exit $?
run_pass fetch FETCH_SIZE || exit $?
run_pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || exit $?
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.json" || exit $?
cat "$OUT/summary.json"
