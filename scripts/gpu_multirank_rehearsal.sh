#!/bin/bash
# Rehearses bench.py's multi-rank path on a one-GPU box through the same
# entry the driver uses (bench.py --gpus N spawns the N ranks itself): the
# ranks share device 0 and talk over gloo (the driver's 8-GPU runs use
# RCCL).  Small per-rank shards; every config, so both the rank-local (C2)
# and the cross-rank exchange paths (C3/C4 shared-group partials, C5
# histogram protocol) run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 OTSDB_BENCH_SAME_DEVICE=1 OTSDB_BENCH_BACKEND=gloo
for n in ${RANKS:-2 4}; do
  for cfg in ${CONFIGS:-C2 C3 C4 C5}; do
    timeout -k 10 300 python bench.py --gpus $n --config $cfg \
      --series ${SERIES:-4000} --steps 3 --warmup 1 --no-extra \
      > gpurun_out/rehearse_${cfg}_n$n.log 2>&1 || { tail -30 gpurun_out/rehearse_${cfg}_n$n.log; exit 1; }
    grep '^{' gpurun_out/rehearse_${cfg}_n$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n=$n', '$cfg', d['n_gpus'], d['ranks_seen'], '%.4g' % d['value'], d['config']['parallelism'], d['config']['output_points_per_gpu'])"
  done
done
