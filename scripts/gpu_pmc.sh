#!/usr/bin/env bash
# PMC counters of the device scorer kernels (own run: --pmc with --kernel-trace/--stats only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --stats \
  --output-format csv -d gpurun_out/pmc -o dev -- python3 scripts/device_bench.py --nodes 4096 --pods 40 \
  --kinds single,gang4 --paths gpu > gpurun_out/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 gpurun_out/pmc.log
exit $rc
