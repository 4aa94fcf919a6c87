#!/bin/bash
# rocprofv3 kernel-trace stats of one bench config per run (CONFIGS list).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for cfg in ${CONFIGS:-C4 C5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof_$cfg" -o run -- python3 -u "$R/bench.py" \
    --config $cfg --steps ${STEPS:-5} --no-cpu-baseline \
    > gpurun_out/bench_${cfg}_prof.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_${cfg}_prof.log | tail -1 | cut -c1-300
done
