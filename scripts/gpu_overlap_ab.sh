#!/usr/bin/env bash
# A/B: config 6 (4096 nodes, device scorer) with native batches inline vs overlapped with
# binding on the engine worker thread (the default, auto); plus the headline config 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/overlap_ab.jsonl
: > $out
for args in "--config 6 --overlap off --steps 3 --warmup 1" "--config 6 --steps 3 --warmup 1" \
            "--config 6 --overlap off --steps 3 --warmup 1" "--config 6 --steps 3 --warmup 1" \
            "--config 3"; do
  echo "=== bench $args ($(date +%T))"
  timeout -k 10 240 python bench.py $args > gpurun_out/bench_one.log 2>&1
  rc=$?
  grep '^{' gpurun_out/bench_one.log | sed "s/^{/{\"args\": \"$args\", /" >> $out
  echo "rc=$rc"; tail -1 $out | cut -c1-220
  case $rc in 0) ;; *) echo "stop after rc=$rc"; tail -20 gpurun_out/bench_one.log; exit $rc ;; esac
done
