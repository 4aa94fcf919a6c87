#!/bin/bash
# Perf probe: the read ceiling of k_bucketize's access pattern
# (tools/stream_probe), an interleaved A/B of the k_bucketize variants
# (variants build), then the PMC passes of the default kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 ./tools/stream_probe 100000 > gpurun_out/stream_probe.log 2>&1 || exit $?
cat gpurun_out/stream_probe.log
OTSDB_LIB=$(pwd)/opentsdb_amd/_build/libotsdb_agg_variants.so \
  timeout -k 10 300 python -u scripts/ab_bucketize.py --ks ${AB_KS:-8,89,82,99,97,85,86,88,16,81,4} \
  --rounds ${AB_ROUNDS:-3} --reps ${AB_REPS:-3} > gpurun_out/ab.log 2>&1 || exit $?
tail -1 gpurun_out/ab.log
if [ -n "$NO_PMC" ]; then exit 0; fi
bash scripts/gpu_pmc.sh || exit $?
