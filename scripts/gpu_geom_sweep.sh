#!/usr/bin/env bash
# k_batch geometry sweep (nodes per block x waves per block) at 4096 and 16384 nodes, two rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/geom_sweep.jsonl
: > $out
for r in 1 2; do
  for g in "0 0" "64 4" "64 8" "128 4"; do
    set -- $g
    YODA_DEV_NPB=$1 YODA_DEV_BWAVES=$2 timeout -k 10 120 python scripts/device_batch_bench.py --nodes 4096,16384 --modes batch --trace --busy 0.3 --pods 520 --batch 256 > gpurun_out/geom_one.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/geom_one.log; exit $rc; }
    grep '^{' gpurun_out/geom_one.log | sed "s/^{/{\"npb_env\": $1, \"waves_env\": $2, /" >> $out
    tail -2 $out | cut -c1-120
  done
done
