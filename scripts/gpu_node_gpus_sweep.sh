#!/usr/bin/env bash
# BASELINE protocol item 5: configs 2-5 at 1, 2, 4 and 8 GPUs per node, one JSON line each
# into gpurun_out/node_gpus_sweep.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/node_gpus_sweep.jsonl
: > $out
for cfg in 2 3 4 5; do
  for g in 1 2 4 8; do
    args="--config $cfg --node-gpus $g --steps 3 --warmup 1 --alt none"
    echo "=== bench $args ($(date +%T))"
    timeout -k 10 240 python bench.py $args > gpurun_out/bench_one.log 2>&1
    rc=$?
    grep '^{' gpurun_out/bench_one.log | sed "s/^{/{\"args\": \"$args\", /" >> $out
    echo "rc=$rc"; tail -1 $out | cut -c1-200
    case $rc in 0) ;; *) echo "stop after rc=$rc"; exit $rc ;; esac
  done
done
