#!/usr/bin/env bash
# config-6 bursts with k_batch phase stamps: the in-tree kernel vs libyoda_hip_base.so, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/c6_trace_ab.jsonl
: > $out
for r in 1 2; do
  for v in base new; do
    lib=""; [ $v = base ] && lib="$PWD/yoda_scheduler_amd/_native/libyoda_hip_base.so"
    YODA_HIP_LIB=$lib timeout -k 10 200 python scripts/timeline_burst.py --config 6 --bursts 3 --device-trace > gpurun_out/c6t_one.jsonl 2> gpurun_out/c6t_one.err
    rc=$?; [ $rc -eq 0 ] || { echo "timeline rc=$rc"; tail -5 gpurun_out/c6t_one.err; exit $rc; }
    grep '^{' gpurun_out/c6t_one.jsonl | sed "s/^{/{\"variant\": \"$v\", /" >> $out
    echo "$v r$r"; tail -1 $out | cut -c1-160
  done
done
