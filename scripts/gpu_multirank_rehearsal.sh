#!/bin/bash
# Rehearses bench.py's multi-rank path on a one-GPU box: N ranks share
# device 0 and talk over gloo (the driver's 8-GPU runs use RCCL).  Small
# per-rank shards; every config, so both the rank-local (C1/C2) and the
# cross-rank exchange paths (C3/C4 partials, C5 histogram protocol) run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 OTSDB_BENCH_SAME_DEVICE=1 OTSDB_BENCH_BACKEND=gloo
P=29511
for n in ${RANKS:-2 4}; do
  for cfg in ${CONFIGS:-C2 C3 C4 C5}; do
    P=$((P + 1))
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $n --master-addr 127.0.0.1 --master-port $P bench.py \
      --gpus $n --config $cfg --series ${SERIES:-4000} --steps 3 --warmup 1 \
      > gpurun_out/rehearse_${cfg}_n$n.log 2>&1 || { tail -30 gpurun_out/rehearse_${cfg}_n$n.log; exit 1; }
    grep '^{' gpurun_out/rehearse_${cfg}_n$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n=$n', '$cfg', '%.4g' % d['value'], d['config']['parallelism'], d['config']['output_points_per_gpu'])"
  done
done
