#!/bin/bash
# Round 6 A/B: short bench runs of CONFIGS (C1..C5, "named" = the metric's
# own query shape on C2 data) for each library in LIBS ("prod" or a variant
# name under opentsdb_amd/_build/var_<name>/), interleaved ROUNDS times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6_cfg
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-1}); do
for c in ${CONFIGS:-C2}; do
  for v in ${LIBS:-prod}; do
    if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
    if [ "$c" = named ]; then cfg="--config C2 --named-query"; else cfg="--config $c"; fi
    log=gpurun_out/r6_cfg/${c}_${v}_$r.log
    timeout -k 10 300 python3 -u bench.py $cfg --steps ${STEPS:-10} --warmup 3 \
      --no-cpu-baseline --no-extra --no-decode > $log 2>&1 || { tail -20 $log; exit 1; }
    tail -1 $log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$c $v round $r: ms/step %.3f med %.3f frac %.3f kernel_frac %s stages %s' % (d['ms_per_step'], d.get('ms_per_step_median', 0), d['roofline']['frac'], d['roofline'].get('kernel_frac'), d['config'].get('stage_ms')))"
  done
done
done
