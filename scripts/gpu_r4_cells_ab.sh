#!/bin/bash
# Cells fold A/B over tuning builds (opentsdb_amd/_build/var_<name>): time
# (scripts/cells_probe.py) and one SQ counter pass each.  VARIANTS="prod a b"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/cells_ab
mkdir -p "$OUT"
SER=${SERIES:-100000}
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then L=opentsdb_amd/_build/libotsdb_agg.so; else L=opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  OTSDB_LIB=$L timeout -k 10 200 python3 -u scripts/cells_probe.py --series $SER $ARGS > "$OUT/$v.log" 2>&1 || { tail -5 "$OUT/$v.log"; exit 1; }
  echo "$v: $(grep 'round 0' $OUT/$v.log | sed 's/.*query/query/')"
  if [ -z "$NO_PMC" ]; then
    OTSDB_LIB=$L timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv \
      -d "$OUT/pmc_$v" -o p -- python3 -u scripts/cells_probe.py --series $SER --reps 1 $ARGS > "$OUT/pmc_$v.log" 2>&1 || exit $?
  fi
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, os, sys
for d in sorted(glob.glob(os.path.join(sys.argv[1], "pmc_*"))):
    if not os.path.isdir(d): continue
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if "k_fold" in r["Kernel_Name"]:
                acc[r["Kernel_Name"][:30]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        steps = 5732854731 / 512 * int(os.environ.get("SERIES", "100000")) / 100000
        print(os.path.basename(d), "VALU/step %.0f SALU/step %.0f LDS/step %.1f VMEM/step %.1f waves %.0f busy %.3g" % (
            m.get("SQ_INSTS_VALU", 0) / steps, m.get("SQ_INSTS_SALU", 0) / steps,
            m.get("SQ_INSTS_LDS", 0) / steps, m.get("SQ_INSTS_VMEM_RD", 0) / steps,
            m.get("SQ_WAVES", 0), m.get("SQ_BUSY_CYCLES", 0)))
PY
