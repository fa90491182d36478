# config 5 (5000-pod bursts) vs config 3 on the same box, twice
set -u
mkdir -p gpurun_out
: > gpurun_out/ab_c5.jsonl
for i in 1 2; do
  for args in "--config 5 --steps 5 --warmup 1 --alt none" "--config 3 --alt none"; do
    timeout -k 10 300 python bench.py $args > gpurun_out/ab_one.log 2>&1 || exit 1
    grep '^{' gpurun_out/ab_one.log >> gpurun_out/ab_c5.jsonl
    echo "$args done"
  done
done
