#!/usr/bin/env bash
# In-tree fake apiserver vs yoda-fake-apiserver-base (the previous build), alternating, on
# configs 3, 5 and 6: one JSON line per run into gpurun_out/fakeapi_ab.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/fakeapi_ab.jsonl
: > $out
for r in 1 2; do
  for args in "--config 3 --alt none" "--config 5 --steps 5 --warmup 1 --alt none" \
              "--config 6 --steps 5 --warmup 1 --alt none --device on"; do
    for v in base new; do
      bin=""; [ $v = base ] && bin="$PWD/yoda_scheduler_amd/_native/yoda-fake-apiserver-base"
      YODA_FAKEAPI_BIN=$bin timeout -k 10 300 python bench.py $args > gpurun_out/fab_one.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/fab_one.log; exit $rc; }
      grep '^{' gpurun_out/fab_one.log | sed "s/^{/{\"variant\": \"$v\", \"args\": \"$args\", /" >> $out
      tail -1 $out | cut -c1-140
    done
  done
done
