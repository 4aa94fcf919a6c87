#!/bin/bash
# A/B of library variants (opentsdb_amd/_build/var_*/) on the streams the
# prefetch knobs touch: the C2 columnar fold, the C2 cells fold
# (scripts/cells_probe.py), the C4 rate bucketize and the C5 bucketize.
# VARIANTS="prod pf1 pf2" bash scripts/gpu_ab_pf.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  timeout -k 10 240 python -u scripts/cells_probe.py --reps 5 > gpurun_out/abpf_cells_$v.log 2>&1 || exit $?
  echo "$v cells: $(tail -1 gpurun_out/abpf_cells_$v.log)"
  for cfg in ${CONFIGS:-C2 C4 C5}; do
    timeout -k 10 240 python -u bench.py --config $cfg --steps ${STEPS:-10} --no-cpu-baseline --no-decode --no-extra > gpurun_out/abpf_${cfg}_$v.json 2>gpurun_out/abpf_${cfg}_$v.err || exit $?
    python - "$v" "$cfg" <<'PY'
import json, sys
v, cfg = sys.argv[1:]
d = json.loads(open("gpurun_out/abpf_%s_%s.json" % (cfg, v)).read().strip().splitlines()[-1])
print("%-5s %s %8.3f ms/step  stage %s  frac %.3f" % (v, cfg, d["ms_per_step"],
      {k: round(x, 3) for k, x in d["config"]["stage_ms"].items() if x}, d["roofline"]["frac"]), flush=True)
PY
  done
done
