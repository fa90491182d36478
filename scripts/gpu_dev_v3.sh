#!/usr/bin/env bash
# Device scorer check: parity tests, per-cycle latency sweep, config-6 bench (x2), kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_device_scorer.py -x -q > gpurun_out/dev.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/dev.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/device_bench.py --nodes ${NODES:-1024,4096,16384,65536} --pods 100 --paths gpu > gpurun_out/devbench_v3.jsonl 2> gpurun_out/devbench_v3.err
rc=$?; echo "devbench rc=$rc"; cut -c1-220 gpurun_out/devbench_v3.jsonl
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
timeout -k 10 300 python bench.py --config 6 --steps 3 --warmup 1 --device on > gpurun_out/bench6_on_v3_$k.log 2>&1
rc=$?; echo "bench6 rc=$rc"; grep '^{' gpurun_out/bench6_on_v3_$k.log | cut -c1-330
[ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6_v3 -o run -- python3 bench.py --config 6 --steps 2 --warmup 1 --device on > gpurun_out/prof6_v3.log 2>&1
echo "prof rc=$?"
