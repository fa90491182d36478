#!/usr/bin/env bash
# End-of-session record: GPU suite, smoke, every BASELINE config (gpu_bench_all.sh), and a
# rocprofv3 kernel trace of config 6 on the device scorer.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_all.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6 -o run -- python3 bench.py --config 6 --steps 2 --warmup 1 --alt none --device on > gpurun_out/prof6.log 2>&1
echo "prof rc=$?"
