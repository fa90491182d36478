set -u
mkdir -p gpurun_out
: > gpurun_out/ab_drain.jsonl
for b in 512 256 128; do
  for c in 6 3; do
    if [ $c = 6 ]; then args="--config 6 --steps 5 --warmup 1 --alt none"; else args="--config 3 --alt none"; fi
    YODA_DRAIN_BUDGET=$b timeout -k 10 200 python bench.py $args > gpurun_out/ab_one.log 2>&1 || exit 1
    grep '^{' gpurun_out/ab_one.log | sed "s/^{/{\"budget\": $b, /" >> gpurun_out/ab_drain.jsonl
    echo "budget $b config $c done"
  done
done
YODA_DRAIN_BUDGET=256 timeout -k 10 200 python scripts/timeline_burst.py --config 6 --repeat 2 --bursts 2 --device-trace > gpurun_out/tl6c.jsonl 2> gpurun_out/tl6c.err
