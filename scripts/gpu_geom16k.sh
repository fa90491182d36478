# k_batch geometry at 16 384 / 65 536 nodes: fewer, fuller blocks vs more blocks
set -u
mkdir -p gpurun_out
: > gpurun_out/geom16k.jsonl
for cfg in "8 64 16384" "8 128 16384" "4 128 16384" "8 256 65536"; do
  set -- $cfg
  YODA_DEV_BWAVES=$1 YODA_DEV_NPB=$2 timeout -k 10 200 python scripts/device_batch_bench.py --nodes $3 --modes batch --trace --busy 0.3 --pods 264 --batch 256 > gpurun_out/g_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/g_one.log | sed "s/^{/{\"waves\": $1, \"npb_min\": $2, /" >> gpurun_out/geom16k.jsonl
done
