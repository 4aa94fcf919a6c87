#!/bin/bash
# rocprofv3 --kernel-trace --stats of the bench for each config in
# $CONFIGS (one run each), CSV summaries under gpurun_out/ks_<cfg>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for cfg in ${CONFIGS:-C2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/ks_$cfg -o ks -- python3 -u bench.py --config $cfg \
    --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-extra --no-decode \
    ${BENCH_ARGS} > gpurun_out/ks_$cfg.log 2>&1 || exit $?
  tail -1 gpurun_out/ks_$cfg.log > gpurun_out/ks_$cfg.json
  f=$(find gpurun_out/ks_$cfg -name "*kernel_stats.csv" | head -1)
  echo "== $cfg: $f"
  head -8 "$f" | cut -c1-220
done
