set -u
mkdir -p gpurun_out/kab
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_scorer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kab/parity.log 2>&1 || { echo parity rc=$?; tail -30 gpurun_out/kab/parity.log; exit 1; }
tail -1 gpurun_out/kab/parity.log
timeout -k 10 500 python scripts/gpu_ab.py --variant base:YODA_HIP_LIB=$PWD/_ab/hip_base.so --variant fast1:YODA_HIP_LIB=$PWD/_ab/hip_fast1.so --reps 3 --out gpurun_out/kab/fast1.jsonl -- python scripts/device_batch_bench.py --nodes 4096 --pods 1032 --batch 256 --modes batch --trace --mix bench > gpurun_out/kab/fast1.log 2>&1 || exit $?
python - <<'PY'
import json
for l in open("gpurun_out/kab/fast1.jsonl"):
    d = json.loads(l)
    print(d.get("variant"), d.get("nodes"), d.get("us_per_pod"), d.get("phase_us_mean"), {k: v[1] for k, v in d.get("score_a_us_by_gpus", {}).items()})
PY
