#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_device_scorer.py -x -q > gpurun_out/dev.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -15 gpurun_out/dev.log
case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 400 python scripts/device_bench.py --nodes ${NODES:-1024,16384,65536} --pods 50 --paths ${PATHS_:-gpu} > gpurun_out/devbench.jsonl 2> gpurun_out/devbench.err
rc=$?; echo "devbench rc=$rc"; cat gpurun_out/devbench.jsonl; tail -3 gpurun_out/devbench.err
case $rc in 0|1) ;; *) exit $rc ;; esac
if [ -n "${PROF:-}" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dev -o dev -- python3 scripts/device_bench.py --nodes 16384 --pods 100 --paths gpu > gpurun_out/prof_dev.log 2>&1
echo "prof rc=$?"
fi
