#!/bin/bash
# Round 6: cells-fold ablation variants (opentsdb_amd/_build/var_<name>/,
# scripts/build_cells_variant.py): probe timing and one SQ PMC pass each.
# VARIANTS="abl1 abl2 ..." ("prod" = the production library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r6_abl
mkdir -p "$OUT"
SER=${SERIES:-100000}
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  timeout -k 10 200 python3 -u scripts/cells_probe.py --series $SER ${PROBE_ARGS} > "$OUT/$v.probe.log" 2>&1 \
    || { tail -20 "$OUT/$v.probe.log"; exit 1; }
  echo "$v: $(grep 'min' "$OUT/$v.probe.log" | tail -1)"
  [ -n "$NO_PMC" ] && continue
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES \
    SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv \
    -d "$OUT/$v" -o sq -- python3 -u scripts/cells_probe.py --series $SER --reps 1 ${PROBE_ARGS} \
    > "$OUT/$v.sq.log" 2>&1 || { tail -5 "$OUT/$v.sq.log"; exit 1; }
  python3 scripts/pmc_summary.py "$OUT/$v" > "$OUT/$v.json" || exit 1
  python3 - "$OUT/$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, c in d.items():
    if not isinstance(c, dict) or "SQ_INSTS_VALU" not in c:
        continue
    steps = 5732854731 / 512.0 if "k_fold" in k else None
    if steps:
        print(sys.argv[2], k[:60], "VALU/step %.0f SALU/step %.0f VMEM/step %.2f LDS/step %.1f" % (
            c["SQ_INSTS_VALU"] / steps, c["SQ_INSTS_SALU"] / steps,
            c["SQ_INSTS_VMEM_RD"] / steps, c["SQ_INSTS_LDS"] / steps))
PY
done
