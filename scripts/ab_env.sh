#!/usr/bin/env bash
# Same-box A/B of an environment knob: ARGS (bench args) run REPS times per setting,
# settings alternate. AB="VAR=a VAR=b" (one assignment per setting).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/${OUT:-ab_env}.jsonl
: > $out
for r in $(seq 1 ${REPS:-3}); do
  for kv in $AB; do
    echo "=== $kv bench $ARGS ($(date +%T))"
    env "$kv" timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_one.log 2>&1
    rc=$?
    grep '^{' gpurun_out/bench_one.log | sed "s/^{/{\"setting\": \"$kv\", \"args\": \"$ARGS\", /" >> $out
    echo "rc=$rc"; tail -1 $out | cut -c1-160
    case $rc in 0) ;; *) echo "stop after rc=$rc"; exit $rc ;; esac
  done
done
