#!/bin/bash
# A/B of tuning builds (scripts/build_variants.py) on one box, one config:
# each library runs the same bench, alternating production / variant twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CFG=${CFG:-C5}
for rep in $(seq 1 ${REPS:-2}); do
  for v in prod ${VARIANTS}; do
    lib=opentsdb_amd/_build/libotsdb_agg.so
    [ "$v" != prod ] && lib=opentsdb_amd/_build/var_$v/libotsdb_agg.so
    OTSDB_LIB=$lib timeout -k 10 200 python -u bench.py --config $CFG --steps ${STEPS:-20} \
      --warmup 3 --no-cpu-baseline --no-extra --no-decode > gpurun_out/ab_${CFG}_$v.log 2>&1 || exit 1
    tail -1 gpurun_out/ab_${CFG}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rep $v', 'ms %.4f' % d['ms_per_step'], {k: round(x, 4) for k, x in d['config']['stage_ms'].items()})"
  done
done
