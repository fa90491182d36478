# config-6 timelines: drain budget x overlap depth (main-thread CPU and wall per burst)
set -u
mkdir -p gpurun_out
: > gpurun_out/knobs.jsonl
for b in 512 256; do
  for d in 2 3 4; do
    YODA_DRAIN_BUDGET=$b timeout -k 10 200 python scripts/timeline_burst.py --config 6 --repeat 2 --bursts 3 --overlap-depth $d > gpurun_out/k_one.jsonl 2> gpurun_out/k_one.err || exit 1
    sed "s/^{/{\"budget\": $b, \"depth\": $d, /" gpurun_out/k_one.jsonl >> gpurun_out/knobs.jsonl
  done
done
