#!/bin/bash
# A/B of cells-fold tuning builds (scripts/build_cells_variant.py) on the
# C2-shaped fused cells query (scripts/cells_probe.py), one process each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  timeout -k 10 200 python3 -u scripts/cells_probe.py --series ${SERIES:-100000} --reps 3 \
    > gpurun_out/cab_$v.log 2>&1 || { tail -5 gpurun_out/cab_$v.log; exit 1; }
  echo "$v: $(grep 'round 0' gpurun_out/cab_$v.log)"
done
