set -u
mkdir -p gpurun_out/kab
timeout -k 10 500 python scripts/gpu_ab.py --variant npb32: --variant npb16:YODA_DEV_NPB=16 --variant npb8:YODA_DEV_NPB=8 --reps 2 --out gpurun_out/kab/npb1024.jsonl -- python scripts/device_batch_bench.py --nodes 1024,2048 --pods 1032 --batch 256 --modes batch --trace > gpurun_out/kab/npb.log 2>&1 || exit $?
timeout -k 10 500 python scripts/gpu_ab.py --variant npb32: --variant npb16:YODA_DEV_NPB=16 --reps 2 --out gpurun_out/kab/npb4096.jsonl -- python scripts/device_batch_bench.py --nodes 4096 --pods 1032 --batch 256 --modes batch --trace >> gpurun_out/kab/npb.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/kab/npb1024.jsonl", "gpurun_out/kab/npb4096.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(d.get("variant"), d.get("nodes"), d.get("grid"), d.get("nodes_per_block"), d.get("us_per_pod"), d.get("phase_us_mean"), {k: v[1] for k, v in d.get("score_a_us_by_gpus", {}).items()})
PY
