# k_batch gather polling: one granule per record until all landed (this build) — parity + timing
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_scorer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kab_tests.log 2>&1 || { tail -30 gpurun_out/kab_tests.log; exit 1; }
tail -1 gpurun_out/kab_tests.log
: > gpurun_out/kab3.jsonl
for cfg in "4 32" "4 16" "8 32"; do
  set -- $cfg
  YODA_DEV_BWAVES=$1 YODA_DEV_NPB=$2 timeout -k 10 200 python scripts/device_batch_bench.py --nodes 4096,16384 --modes batch --trace --busy 0.3 --pods 520 --batch 256 > gpurun_out/kab_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/kab_one.log | sed "s/^{/{\"waves\": $1, \"npb_min\": $2, /" >> gpurun_out/kab3.jsonl
done
