#!/bin/bash
# Columnar fold A/B over tuning builds: bench.py (C2 headline + the named
# query figure) per library.  VARIANTS="prod a b"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/fold_ab
mkdir -p "$OUT"
for rnd in 1 2; do
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then L=opentsdb_amd/_build/libotsdb_agg.so; else L=opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  OTSDB_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --no-decode ${ARGS} > "$OUT/$v.$rnd.log" 2>&1 || { tail -5 "$OUT/$v.$rnd.log"; exit 1; }
  python3 - "$OUT/$v.$rnd.log" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
nq = d.get("named_query", {})
print(sys.argv[2], "C2 %.3f ms/step frac %.3f | named %s ms frac %s" % (
    d["ms_per_step"], d["roofline"]["frac"], nq.get("ms_per_query"), nq.get("frac_of_8TBs", nq.get("frac"))))
PY
done
done
