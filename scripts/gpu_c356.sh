#!/usr/bin/env bash
# Configs 3, 5 and 6 (device scorer) on one box, REPS times each, one JSON line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/${OUT:-c356}.jsonl
: > $out
for r in $(seq 1 ${REPS:-2}); do
  for args in "--config 3 --alt none" "--config 5 --steps 5 --warmup 1 --alt none" \
              "--config 6 --steps 5 --warmup 1 --alt none --device on"; do
    echo "=== bench $args ($(date +%T))"
    timeout -k 10 300 python bench.py $args > gpurun_out/bench_one.log 2>&1
    rc=$?
    grep '^{' gpurun_out/bench_one.log | sed "s/^{/{\"args\": \"$args\", /" >> $out
    echo "rc=$rc"; tail -1 $out | cut -c1-200
    case $rc in 0) ;; *) echo "stop after rc=$rc"; exit $rc ;; esac
  done
done
