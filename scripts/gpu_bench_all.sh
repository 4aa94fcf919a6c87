#!/bin/bash
# Every BASELINE config on one MI355X (C3/C5 at their per-GPU share of the
# 8-GPU node config), then the C2 headline under rocprofv3 --kernel-trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in ${CONFIGS:-C1 C3 C4 C5 C2}; do
  # (C1's 0.12 ms steps: 300 of them, so the mean is not one host hiccup)
  steps=${STEPS:-10}; [ $cfg = C1 ] && steps=300
  timeout -k 10 300 python -u bench.py --config $cfg --steps $steps \
    --cpu-seconds ${CPU_S:-10} > gpurun_out/bench_$cfg.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$cfg.log
done
if [ -n "$NO_PROF" ]; then exit 0; fi
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$R/gpurun_out/prof_c2" -o run -- python -u "$R/bench.py" --steps 10 \
  --no-cpu-baseline > gpurun_out/bench_c2_prof.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2_prof.log
