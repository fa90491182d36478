set -u
mkdir -p gpurun_out/r3all
for spec in "3|--config 3 --steps 20 --warmup 5" "1|--config 1 --steps 20 --warmup 2" "2|--config 2 --steps 10 --warmup 2" "4|--config 4 --steps 10 --warmup 2" "5|--config 5 --steps 5 --warmup 2" "6|--config 6 --steps 5 --warmup 1" "6off|--config 6 --steps 2 --warmup 1 --device off" "3ref|--config 3 --steps 1 --warmup 0 --reference-qps" "3b|--config 3 --steps 20 --warmup 5"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python bench.py --alt none $args > gpurun_out/r3all/c$name.log 2>&1
  rc=$?
  echo "c$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r3all/c*.log")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d.get("e2e_scheduling_p99_ms"), d["cpu_us_per_pod"], d.get("apiserver_cpu_us_per_pod"), d["device_cycles"], d["host"]["calib_loop_ms"])
PY
