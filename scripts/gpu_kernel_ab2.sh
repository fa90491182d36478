# k_batch: 8 waves over 32 nodes per block (gang replicas: two lane groups per node) vs 4 waves
set -u
mkdir -p gpurun_out
: > gpurun_out/kab2.jsonl
for cfg in "4 32" "8 32" "8 16" "4 16"; do
  set -- $cfg
  YODA_DEV_BWAVES=$1 YODA_DEV_NPB=$2 timeout -k 10 200 python scripts/device_batch_bench.py --nodes 4096 --modes batch --trace --busy 0.3 --pods 520 --batch 256 > gpurun_out/kab_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/kab_one.log | sed "s/^{/{\"waves\": $1, \"npb_min\": $2, /" >> gpurun_out/kab2.jsonl
done
