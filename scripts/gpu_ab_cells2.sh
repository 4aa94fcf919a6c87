#!/bin/bash
# A/B of library variants on the C2 cells fold (scripts/cells_probe.py):
# VARIANTS="prod w4" bash scripts/gpu_ab_cells2.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rnd in 1 2; do
for v in ${VARIANTS:-prod}; do
  if [ "$v" = prod ]; then unset OTSDB_LIB; else export OTSDB_LIB=$PWD/opentsdb_amd/_build/var_$v/libotsdb_agg.so; fi
  timeout -k 10 200 python -u scripts/cells_probe.py --series ${SERIES:-100000} --reps 5 > gpurun_out/abc2_$v.log 2>&1 || { tail -5 gpurun_out/abc2_$v.log; exit 1; }
  echo "$v: $(tail -2 gpurun_out/abc2_$v.log | head -1)"
done
done
