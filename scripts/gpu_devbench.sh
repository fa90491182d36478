#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python scripts/device_bench.py --nodes 1024,4096,16384,65536 --pods 50 --paths gpu,cpu,cpu-adaptive > gpurun_out/devbench.jsonl 2> gpurun_out/devbench.err
rc=$?; echo "devbench rc=$rc"; cat gpurun_out/devbench.jsonl
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dev -o dev -- python3 scripts/device_bench.py --nodes 16384 --pods 100 --paths gpu > gpurun_out/prof_dev.log 2>&1
echo "prof rc=$?"
find gpurun_out/prof_dev -name "*stats*" | head
