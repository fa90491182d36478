#!/usr/bin/env python3
"""Timeline of one timed burst over the HTTP transport: when pods reach the queue, each
native engine call (batch size, start, duration), and bind completions — relative to the
burst start. Diagnoses where a burst's wall time goes (arrival vs engine vs binding).

    python scripts/timeline_burst.py --config 6 [--batch 256] [--device on]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


async def run(a) -> dict:
    from yoda_scheduler_amd.bench.harness import HttpShard
    from yoda_scheduler_amd.bench.workloads import make_workload
    w = make_workload(a.config)
    sh = HttpShard(w, batch=a.batch, device=a.device, overlap=a.overlap)
    sh.cfg.trace = True
    await sh.start()
    sched = sh.sched
    for i in range(a.warmup):
        await sh.burst(f"w{i}")
    arrivals: list[float] = []
    q = sched.queue
    orig_add = q.add

    def add(pi, *args, **kw):
        arrivals.append(time.perf_counter())
        return orig_add(pi, *args, **kw)
    q.add = add
    pops: list = []
    orig_pb = q.pop_batch

    def pop_batch(n, *args, **kw):
        t = time.perf_counter()
        out = orig_pb(n, *args, **kw)
        pops.append((t, len(out), len(q._active_entries)))
        return out
    q.pop_batch = pop_batch
    eng_calls: list = []
    orig_sb = sched.engine.schedule_batch

    class _EngProxy:      # times every engine batch call (any thread)
        def __getattr__(self, k):
            return getattr(eng, k)

        def schedule_batch(self, ids, reqs):
            t = time.perf_counter()
            r = orig_sb(ids, reqs)
            eng_calls.append((t, time.perf_counter(), len(ids)))
            return r
    eng = sched.engine
    sched.engine = _EngProxy()
    tr = sched.tracer
    dev_trace = a.device_trace and sched.engine.device_enabled
    if dev_trace:
        from yoda_scheduler_amd.ops import device_scorer as ds
        ds.batch_trace(sched.engine, True)
    t0 = time.perf_counter()
    t0_us = tr.now_us()
    res = await sh.burst("s0")
    t1 = time.perf_counter()
    spans = list(tr.chrome_trace()["traceEvents"])
    batches = [(round((e["ts"] - t0_us) / 1000, 3), round(e.get("dur", 0) / 1000, 3), e["args"].get("pods"))
               for e in spans if e["name"] == "native_batch"]
    binds = sorted((e["ts"] + e.get("dur", 0) - t0_us) / 1000 for e in spans if e["name"] == "bind"
                   and e["ts"] + e.get("dur", 0) >= t0_us)
    batches = [b for b in batches if b[0] + b[1] >= 0]
    # everything relative to the first pod reaching the queue (the burst's reset phase and
    # the create request precede it)
    ta = min(arrivals) if arrivals else t0
    t0_us += (ta - t0) * 1e6
    arr = sorted((x - ta) * 1000 for x in arrivals)
    calls_rel = [(round((t - ta) * 1000, 3), round((e - t) * 1000, 3), n) for t, e, n in eng_calls if e >= ta]
    pops_rel = [(round((t - ta) * 1000, 3), n, left) for t, n, left in pops if t >= ta]
    pct = lambda xs, p: round(xs[min(len(xs) - 1, int(p * (len(xs) - 1)))], 3) if xs else None
    out = {"config": a.config, "batch": a.batch, "pods": res.pods, "bound": res.bound,
           "wall_ms": round((t1 - t0) * 1000, 3), "apiserver_elapsed_ms": round(res.elapsed_s * 1000, 3),
           "arrival_ms": {"first": pct(arr, 0), "p50": pct(arr, .5), "last": pct(arr, 1)},
           "bind_done_ms": {"first": pct(binds, 0), "p50": pct(binds, .5), "last": pct(binds, 1)},
           "pop_batch(ms,popped,left)": pops_rel[:20],
           "engine_schedule_batch(ms,dur_ms,pods)": calls_rel[:20],
           "device_cycles": sched.engine.device_cycles}
    if dev_trace:
        trc = ds.read_batch_trace(sched.engine)
        if trc:
            out["k_batch_last_chunk"] = {"pods": len(trc), "grid_npb": ds.batch_geometry(sched.engine),
                                         "phase_us_mean": {k: round(sum(x[k] for x in trc) / len(trc), 2)
                                                           for k in trc[0]}}
    sched.engine = eng
    await sh.stop()
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=6)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--overlap", default="auto")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--device-trace", action="store_true", help="k_batch phase stamps of the last chunk")
    a = ap.parse_args()
    try:
        import torch  # noqa: F401 - share torch's HIP runtime, as bench.py does
    except ImportError:
        pass
    print(json.dumps(asyncio.run(run(a))), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
