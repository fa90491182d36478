#!/usr/bin/env bash
# A/B: accumulator atomics with / without the check-before-atomic load.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_device_scorer.py -x -q > gpurun_out/dev.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/dev.log
[ $rc -eq 0 ] || exit $rc
YODA_DEV_DIRECT_ATOMICS=1 timeout -k 10 300 python -m pytest tests/test_gpu_device_scorer.py -x -q > gpurun_out/dev_direct.log 2>&1
rc=$?; echo "parity(direct) rc=$rc"; tail -2 gpurun_out/dev_direct.log
[ $rc -eq 0 ] || exit $rc
for mode in 0 1 0 1; do
YODA_DEV_DIRECT_ATOMICS=$mode timeout -k 10 300 python scripts/device_bench.py --nodes 1024,4096,16384,65536 --kinds single,gang4 --pods 100 --paths gpu > gpurun_out/ab_$mode.jsonl 2>/dev/null
rc=$?; echo "direct=$mode rc=$rc"
python -c "
import json
for l in open('gpurun_out/ab_$mode.jsonl'):
    d=json.loads(l); print(d['nodes'], d['pod'], d['cycle_us_p50'], d['device_kernels_us_p50'])
"
[ $rc -eq 0 ] || exit $rc
done
