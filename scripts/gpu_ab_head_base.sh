#!/usr/bin/env bash
# Same-box A/B of the headline bench: HEAD vs the tree in _ab_base (a git worktree of an
# older commit, built in place), alternating, 3 runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
out=gpurun_out/ab_head_base.jsonl
: > $out
for i in 1 2 3; do
  for t in head base; do
    if [ $t = head ]; then d=$R; else d=$R/_ab_base; fi
    (cd $d && timeout -k 10 200 python bench.py ${AB_ARGS:-} > $R/gpurun_out/ab_one.log 2>&1)
    rc=$?
    grep '^{' gpurun_out/ab_one.log | sed "s/^{/{\"tree\": \"$t\", /" >> $out
    echo "$t rc=$rc $(tail -1 $out | grep -o '"value": [0-9.]*')"
    case $rc in 0) ;; *) tail -5 gpurun_out/ab_one.log; exit $rc ;; esac
  done
done
