# config 6 on the CPU engine with 1 / 8 / 12 worker threads vs the device scorer; config 3 check
set -u
mkdir -p gpurun_out
: > gpurun_out/ab_cpu.jsonl
for args in "--config 6 --steps 2 --warmup 1 --alt none --device off --engine-threads 8" \
            "--config 6 --steps 2 --warmup 1 --alt none --device off --engine-threads 12" \
            "--config 6 --steps 5 --warmup 1 --alt none" "--config 3 --alt none"; do
  timeout -k 10 300 python bench.py $args > gpurun_out/ab_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab_one.log | sed "s/^{/{\"args\": \"$args\", /" >> gpurun_out/ab_cpu.jsonl
  echo "$args done"
done
