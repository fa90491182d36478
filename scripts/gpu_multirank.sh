#!/usr/bin/env bash
# Rehearse the multi-rank bench path on a 1-GPU box: N ranks share GPU 0 over gloo (RCCL
# needs one GPU per rank; the driver's 8-GPU node uses RCCL). Ranks stay well under 16.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2 4; do
  YODA_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 1 \
    > gpurun_out/multirank_$n.log 2>&1
  rc=$?; echo "n=$n rc=$rc"; grep '^{' gpurun_out/multirank_$n.log | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
done
