#!/usr/bin/env bash
# rocprofv3 kernel stats of the config-6 burst (4096 nodes, device scorer on).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6 -o run -- \
  python3 bench.py --config 6 --steps 2 --warmup 1 --device on > gpurun_out/prof6.log 2>&1
rc=$?
echo "prof6 rc=$rc"; tail -3 gpurun_out/prof6.log
exit $rc
