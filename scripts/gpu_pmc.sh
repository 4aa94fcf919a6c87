#!/bin/bash
# PMC passes over the bench (one counter group per rocprofv3 run, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes).  PMC_CFG picks the
# workload, PMC_PASSES the groups (sq fetch write).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${PMC_CFG:-C2}
OUT=gpurun_out/pmc_${CFG}${PMC_TAG}
mkdir -p "$OUT"
run_pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv \
    -d "$OUT/$name" -o "$name" -- \
    python3 -u bench.py --config "$CFG" --steps 2 --warmup 1 \
    --no-cpu-baseline --no-extra ${PMC_NO_DECODE---no-decode} ${PMC_BENCH_ARGS} \
    > "$OUT/$name.log" 2>&1
}
for p in ${PMC_PASSES:-sq fetch write}; do
  case $p in
    sq) run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
          SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU || exit $? ;;
    lds) run_pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU \
          SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAVES || exit $? ;;
    fetch) run_pass fetch FETCH_SIZE || exit $? ;;
    write) run_pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || exit $? ;;
  esac
done
python3 scripts/pmc_summary.py "$OUT" > "$OUT/summary.json" || exit $?
cat "$OUT/summary.json"
