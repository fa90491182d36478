#!/usr/bin/env bash
# config 6 (device scorer) at several scheduler batch sizes, alternating, on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/c6_batch.jsonl
: > $out
for r in 1 2; do
  for b in 256 128 64; do
    timeout -k 10 200 python bench.py --config 6 --steps 5 --warmup 1 --alt none --device on --batch $b > gpurun_out/c6b_one.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/c6b_one.log; exit $rc; }
    grep '^{' gpurun_out/c6b_one.log | sed "s/^{/{\"batch_arg\": $b, /" >> $out
    tail -1 $out | cut -c1-120
  done
done
