#!/usr/bin/env bash
# PMC counters of the persistent k_batch kernel at 4096 nodes (two passes, each within the
# per-block counter limits; --pmc only with --kernel-trace/--stats)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM --kernel-trace --stats \
  --output-format csv -d gpurun_out/pmcb1 -o kb -- python3 scripts/device_batch_bench.py --nodes 4096 --modes batch --busy 0.3 --pods 264 --batch 256 > gpurun_out/pmcb1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-trace --stats \
  --output-format csv -d gpurun_out/pmcb2 -o kb -- python3 scripts/device_batch_bench.py --nodes 4096 --modes batch --busy 0.3 --pods 264 --batch 256 > gpurun_out/pmcb2.log 2>&1
rc=$?; echo "pmc rc=$rc"
exit $rc
