#!/bin/bash
# Config A/B over tuning builds: bench.py --config $CFG per library, two
# rounds (stage times of the pipeline).  VARIANTS="prod a b" CFG=C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/cfg_ab
mkdir -p "$OUT"
for rnd in 1 2; do
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then L=opentsdb_amd/_build/libotsdb_agg.so; else L=opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  OTSDB_LIB=$L timeout -k 10 300 python3 -u bench.py --config ${CFG:-C4} --steps 10 --no-cpu-baseline --no-extra --no-decode ${ARGS} > "$OUT/$v.$rnd.log" 2>&1 || { tail -5 "$OUT/$v.$rnd.log"; exit 1; }
  python3 - "$OUT/$v.$rnd.log" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = d["config"].get("stage_ms", {})
print(sys.argv[2], "%.3f ms/step frac %.3f stages %s" % (
    d["ms_per_step"], d["roofline"]["frac"], {k: round(v, 3) for k, v in st.items() if v}))
PY
done
done
