set -u
mkdir -p gpurun_out
for a in "--config 5 --steps 5 --warmup 1" "--config 3" "--config 5 --steps 5 --warmup 1" "--config 3 --batch 1"; do
  timeout -k 10 300 python bench.py $a > gpurun_out/c5.log 2>&1 || exit $?
  grep '^{' gpurun_out/c5.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$a',d['value'],d['p99_latency_ms'],d['cpu_us_per_pod'])" | tee -a gpurun_out/c5_sum.txt
done
