# k_batch phase-time ablations (timing only: the ablated builds compute wrong scores).
# The variants were built from a copy of native/hip/scorer.hip with (a) the score tail of
# score_node_a replaced by a trivial assignment (ABL_TAIL) and (b) the k >= 2 gang-search
# branch disabled (ABL_GANG), each as yoda_scheduler_amd/_native/libyoda_hip_abl_{tail,gang}.so
# (hipcc --offload-arch=gfx950 -O3 -shared -fPIC scorer.hip probes.hip); results in
# profiles/device/ablation_r2.jsonl.
set -u
mkdir -p gpurun_out
: > gpurun_out/ablate.jsonl
for v in base tail gang; do
  lib=""
  [ $v != base ] && lib="$PWD/yoda_scheduler_amd/_native/libyoda_hip_abl_$v.so"
  YODA_HIP_LIB=$lib timeout -k 10 120 python scripts/device_batch_bench.py --nodes 4096 --modes batch --trace --busy 0 --pods 520 --batch 256 > gpurun_out/abl_one.log 2>&1 || exit 1
  grep '^{' gpurun_out/abl_one.log | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/ablate.jsonl
done
