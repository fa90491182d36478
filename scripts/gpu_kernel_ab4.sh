# two-level gather: parity suite, then timing at 4096 (flat), 16 384 and 65 536 nodes (leaders)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_scorer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kab_tests.log 2>&1 || { tail -30 gpurun_out/kab_tests.log; exit 1; }
tail -1 gpurun_out/kab_tests.log
: > gpurun_out/kab4.jsonl
timeout -k 10 300 python scripts/device_batch_bench.py --nodes 4096,16384,65536 --modes batch --trace --busy 0.3 --pods 264 --batch 256 > gpurun_out/kab_one.log 2>&1 || exit 1
grep '^{' gpurun_out/kab_one.log >> gpurun_out/kab4.jsonl
