#!/usr/bin/env python3
"""Same-box A/B runner: one command, several environment variants, alternated.

Replaces the round-1/2 one-off shell wrappers (``gpu_kernel_ab*.sh``, ``ab_env.sh``,
``gpu_dev_ab.sh``, ...): every A/B those ran is one invocation of this script, e.g.

    # k_batch waves per block, device batch bench, 3 alternating repeats
    python scripts/gpu_ab.py --variant w4:YODA_DEV_BWAVES=4 --variant w8:YODA_DEV_BWAVES=8 \\
        --reps 3 --pre "python -m pytest tests/test_gpu_device_scorer.py -x -q" \\
        -- python scripts/device_batch_bench.py --nodes 4096 --modes batch --pods 520

    # a bench knob on config 5
    python scripts/gpu_ab.py --variant base: --variant knob:YODA_DRAIN_BUDGET=128 \\
        -- python bench.py --config 5 --steps 5 --warmup 1

Each run is a child process under its own time limit. Every JSON line the command prints
goes to ``--out`` (JSONL) prefixed with ``variant``, ``rep`` and the variant's env. The
runner stops at the first crash-like exit (timeout, abort, segfault) and never retries a
failing GPU step.
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys
import time

CRASH = {124, 134, 137, 139, -6, -9, -11}


def parse_variant(text: str) -> tuple[str, dict, str | None]:
    """``name[@dir]:VAR=a,VAR2=b`` → (name, env, cwd); ``name:`` is the unmodified environment.

    ``@dir`` runs that variant's command in another tree (e.g. a git worktree of an older
    commit, built in place), so commits can be bisected on one box."""
    name, _, rest = text.partition(":")
    name, _, cwd = name.partition("@")
    env = {}
    for kv in filter(None, rest.split(",")):
        k, _, v = kv.partition("=")
        env[k.strip()] = v
    return name or "base", env, cwd or None


def run(cmd: list[str], env: dict, timeout: float, log, cwd: str | None = None) -> tuple[int, list[dict]]:
    try:
        r = subprocess.run(cmd, env={**os.environ, **env}, capture_output=True, text=True, timeout=timeout,
                           cwd=cwd)
    except subprocess.TimeoutExpired as e:
        log.write((e.stdout or b"").decode() if isinstance(e.stdout, bytes) else (e.stdout or ""))
        return 124, []
    log.write(r.stdout)
    log.write(r.stderr)
    rows = []
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            try:
                rows.append(json.loads(line))
            except ValueError:
                pass
    return r.returncode, rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--variant", action="append", required=True,
                    help="name[@dir]:VAR=value[,VAR=value] (repeatable)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--timeout", type=float, default=300.0, help="seconds per run")
    ap.add_argument("--pre", default="", help="command run once per variant before the A/B (e.g. parity tests)")
    ap.add_argument("--out", default="gpurun_out/ab.jsonl")
    ap.add_argument("cmd", nargs=argparse.REMAINDER, help="-- command to measure")
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("no command given after --")
    variants = [parse_variant(v) for v in a.variant]
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    logp = os.path.splitext(a.out)[0] + ".log"
    with open(a.out, "w") as out, open(logp, "w") as log:
        if a.pre:
            for name, env, cwd in variants:
                rc, _ = run(shlex.split(a.pre), env, a.timeout, log, cwd)
                print(f"pre[{name}] rc={rc}", flush=True)
                if rc != 0:
                    return rc if rc > 0 else 1
        for rep in range(a.reps):
            for name, env, cwd in variants:
                t0 = time.time()
                rc, rows = run(cmd, env, a.timeout, log, cwd)
                for row in rows:
                    out.write(json.dumps({"variant": name, "rep": rep, "env": env, **row}) + "\n")
                out.flush()
                print(f"{name} rep={rep} rc={rc} rows={len(rows)} {time.time() - t0:.1f}s", flush=True)
                if rc in CRASH:
                    print(f"stopping after crash-like exit {rc}", flush=True)
                    return rc if rc > 0 else 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
