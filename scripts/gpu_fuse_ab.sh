#!/usr/bin/env bash
# A/B: fused select (score kernel's last block normalises + argmaxes) vs the separate
# k_select launch, by cluster size. Parity first with everything fused.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
YODA_DEV_FUSE_MAX=1000000 timeout -k 10 300 python -m pytest tests/test_gpu_device_scorer.py -x -q > gpurun_out/fuse_parity.log 2>&1
rc=$?; echo "parity(all fused) rc=$rc"; tail -2 gpurun_out/fuse_parity.log
[ $rc -eq 0 ] || exit $rc
for fm in 2048 1000000 2048 1000000; do
  YODA_DEV_FUSE_MAX=$fm timeout -k 10 300 python scripts/device_batch_bench.py --nodes 4096,8192,16384,65536 --pods 520 > gpurun_out/fuse_$fm.jsonl 2>/dev/null
  rc=$?; echo "fuse_max=$fm rc=$rc"; cat gpurun_out/fuse_$fm.jsonl
  [ $rc -eq 0 ] || exit $rc
done
