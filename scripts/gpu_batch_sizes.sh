# per-dispatch fixed cost of k_batch: engine-level us/pod at several batch sizes (4096 nodes)
set -u
mkdir -p gpurun_out
: > gpurun_out/bsz.jsonl
for b in 8 32 64 128 256; do
  timeout -k 10 200 python scripts/device_batch_bench.py --nodes 4096 --modes batch --busy 0.3 --pods 1032 --batch $b > gpurun_out/bsz_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/bsz_one.log >> gpurun_out/bsz.jsonl
done
