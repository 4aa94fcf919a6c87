#!/bin/bash
# A/B of kernels between the production library and variant builds
# (VARIANTS="old"): rocprofv3 kernel stats per library of each of QUERIES
# (C1..C5, named = C2's named query), the prep / fold / selection lines
# printed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in prod ${VARIANTS:-old} prod; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  for q in ${QUERIES:-C1 named}; do
    args="--config $q"; [ $q = named ] && args="--config C2 --named-query"
    d=gpurun_out/abp_${v}_$q; rm -rf $d
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o ks \
      -- python3 -u bench.py $args --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-decode \
      > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    python3 - "$v" "$q" "$f" <<'PY'
import csv, sys
v, q, f = sys.argv[1:]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(x in n for x in ("k_fold_prep", "void otsdb::k_fold<", "k_prep", "k_keys_transpose", "k_seg_select")):
        print("%-5s %-6s %-40s %10.1f us" % (v, q, n.split("(")[0][-40:], float(r["AverageNs"]) / 1e3), flush=True)
PY
  done
done
