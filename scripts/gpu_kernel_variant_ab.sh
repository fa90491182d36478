#!/usr/bin/env bash
# k_batch variant (the in-tree build) vs the committed kernel
# (libyoda_hip_base.so, built from git HEAD:native/hip/scorer.hip): parity suite, then alternating
# phase-traced device benches and config-6 bench runs on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_scorer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kvar_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/kvar_parity.log
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/kvar_ab.jsonl
: > $out
for r in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib="$PWD/yoda_scheduler_amd/_native/libyoda_hip_base.so"
    for busy in 0 0.3; do
      YODA_HIP_LIB=$lib timeout -k 10 120 python scripts/device_batch_bench.py --nodes 4096,16384 --modes batch --trace --busy $busy --pods 520 --batch 256 > gpurun_out/kvab_one.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "devbench rc=$rc"; tail -5 gpurun_out/kvab_one.log; exit $rc; }
      grep '^{' gpurun_out/kvab_one.log | sed "s/^{/{\"variant\": \"$v\", \"busy\": $busy, /" >> $out
    done
    YODA_HIP_LIB=$lib timeout -k 10 200 python bench.py --config 6 --steps 5 --warmup 1 --alt none --device on > gpurun_out/kvab_bench.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/kvab_bench.log; exit $rc; }
    grep '^{' gpurun_out/kvab_bench.log | sed "s/^{/{\"variant\": \"$v\", \"bench\": 6, /" >> $out
    echo "$v r$r done"; tail -1 $out | cut -c1-200
  done
done
