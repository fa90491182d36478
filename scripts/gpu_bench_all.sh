#!/usr/bin/env bash
# All BASELINE configs on the GPU box, one JSON line each into gpurun_out/bench_all.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/bench_all.jsonl
: > $out
# headline transport: HTTP (apiserver in its own process); config 3 also reports in-process under "alt"
for args in "--config 1 --steps 20 --alt none" "--config 2 --alt none" "--config 3" "--config 4 --alt none" \
            "--config 5 --steps 5 --warmup 1 --alt none" "--config 6 --steps 5 --warmup 1 --alt none" \
            "--config 6 --steps 2 --warmup 1 --alt none --device off" \
            "--config 6 --steps 2 --warmup 1 --alt none --device off --engine-threads 8" "--config 3 --batch 1 --alt none" \
            "--config 3 --compat --alt none" "--config 3 --reference-qps --steps 1 --warmup 0 --alt none"; do
  echo "=== bench $args ($(date +%T))"
  timeout -k 10 300 python bench.py $args > gpurun_out/bench_one.log 2>&1
  rc=$?
  grep '^{' gpurun_out/bench_one.log | sed "s/^{/{\"args\": \"$args\", /" >> $out
  echo "rc=$rc"; tail -1 $out | cut -c1-300
  case $rc in 0) ;; *) echo "stop after rc=$rc"; exit $rc ;; esac
done
