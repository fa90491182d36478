# config-6 / config-3 timelines (main-thread CPU per burst) + repeated benches (same box)
set -u
mkdir -p gpurun_out
timeout -k 10 200 python scripts/timeline_burst.py --config 6 --repeat 2 --bursts 3 > gpurun_out/tl6j.jsonl 2> gpurun_out/tl6g.err || exit 1
timeout -k 10 200 python scripts/timeline_burst.py --config 3 --repeat 2 --bursts 3 > gpurun_out/tl3j.jsonl 2> gpurun_out/tl3g.err || exit 1
: > gpurun_out/ab_c6.jsonl
for i in 1 2; do
  for args in "--config 6 --steps 5 --warmup 1 --alt none" "--config 3 --alt none"; do
    timeout -k 10 200 python bench.py $args > gpurun_out/ab_one.log 2>&1 || exit 1
    grep '^{' gpurun_out/ab_one.log >> gpurun_out/ab_c6.jsonl
    echo "$args done"
  done
done
