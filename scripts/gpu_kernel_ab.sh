# k_batch geometry A/B (waves per block) after the lane-parallel tail + gang replicas;
# GPU parity tests first
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_scorer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kab_tests.log 2>&1 || { tail -30 gpurun_out/kab_tests.log; exit 1; }
tail -2 gpurun_out/kab_tests.log
: > gpurun_out/kab.jsonl
for w in 4 8; do
  YODA_DEV_BWAVES=$w timeout -k 10 200 python scripts/device_batch_bench.py --nodes 4096,16384 --modes batch --trace --busy 0 --pods 520 --batch 256 > gpurun_out/kab_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/kab_one.log | sed "s/^{/{\"waves\": $w, /" >> gpurun_out/kab.jsonl
  YODA_DEV_BWAVES=$w timeout -k 10 200 python scripts/device_batch_bench.py --nodes 4096 --modes batch --trace --busy 0.3 --pods 520 --batch 256 > gpurun_out/kab_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/kab_one.log | sed "s/^{/{\"waves\": $w, \"busy\": 0.3, /" >> gpurun_out/kab.jsonl
done
