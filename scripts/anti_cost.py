#!/usr/bin/env python3
"""Where a Python-path pod's main-thread CPU goes during ``bench.py``'s timed bursts.

    python scripts/anti_cost.py [bench.py args...]     (e.g. --config 3 --mix-anti 10)

Wraps a few coarse entry points of the event loop's work with ``time.thread_time`` (one
clock read each side, so the wrapping costs ≈ 1 µs per call) and prints, for the timed
bursts only, the interpreter thread's total CPU and each entry point's share per burst.
Nested entry points are counted once, at the outermost one."""
from __future__ import annotations

import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import bench
    from yoda_scheduler_amd.bench import harness as H
    from yoda_scheduler_amd.framework import events as E
    from yoda_scheduler_amd.framework import lane as L
    from yoda_scheduler_amd.framework import scheduler as S
    from yoda_scheduler_amd.kube import native as N
    acc: collections.Counter = collections.Counter()
    cnt: collections.Counter = collections.Counter()
    state = {"on": False, "depth": 0}

    def wrap(cls, name, label=None):
        f = getattr(cls, name)
        key = label or f"{cls.__name__}.{name}"

        def g(*a, **k):
            if not state["on"] or state["depth"]:
                return f(*a, **k)
            state["depth"] += 1
            t = time.thread_time()
            try:
                return f(*a, **k)
            finally:
                acc[key] += time.thread_time() - t
                cnt[key] += 1
                state["depth"] -= 1
        setattr(cls, name, g)

    wrap(S.Scheduler, "schedule_batch")
    wrap(L.NativeLane, "_drain")
    wrap(S.Scheduler, "_native_bind_done")
    wrap(N.NativeTransport, "_drain") if hasattr(N, "NativeTransport") and hasattr(N.NativeTransport, "_drain") else None
    for n in dir(E):
        c = getattr(E, n)
        if isinstance(c, type) and n.endswith("Recorder") and hasattr(c, "run"):
            wrap(c, "run")
    tb = [0.0, 0]
    orig = H.HttpShard.burst

    async def burst(self, tag="b", timeout=600.0):
        timed = tag.startswith("s")
        state["on"] = timed
        t = time.thread_time()
        try:
            return await orig(self, tag, timeout)
        finally:
            if timed:
                tb[0] += time.thread_time() - t
                tb[1] += 1
            state["on"] = False
    H.HttpShard.burst = burst
    bench.main(sys.argv[1:])
    n = max(tb[1], 1)
    print(f"anti_cost: interpreter thread CPU in {tb[1]} timed bursts: {tb[0] / n * 1e3:.3f} ms/burst")
    for k, v in acc.most_common():
        print(f"anti_cost:   {k:34s} {cnt[k] / n:8.1f} calls/burst {v / n * 1e3:8.3f} ms/burst")
    print(f"anti_cost:   {'(rest: loop, harness, other callbacks)':34s} {'':19s} "
          f"{(tb[0] - sum(acc.values())) / n * 1e3:8.3f} ms/burst")
    return 0


if __name__ == "__main__":
    sys.exit(main())
