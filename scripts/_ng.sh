set -u
mkdir -p gpurun_out/ng
for g in 1 2 4 8; do
  timeout -k 10 200 python bench.py --node-gpus $g --steps 20 --warmup 5 --alt none > gpurun_out/ng/g$g.log 2>&1 || exit $?
  tail -1 gpurun_out/ng/g$g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d["pods_bound"], d["pods_unschedulable"], d["cpu_us_per_pod"])' g$g
done
