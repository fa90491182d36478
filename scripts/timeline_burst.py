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


async def run(a) -> list:
    from yoda_scheduler_amd.bench.harness import HttpShard
    from yoda_scheduler_amd.bench.workloads import make_workload
    w = make_workload(a.config)
    sh = HttpShard(w, batch=a.batch, device=a.device, overlap=a.overlap)
    sh.cfg.trace = True
    if a.overlap_depth:
        sh.cfg.overlap_depth = a.overlap_depth
    await sh.start()
    sched = sh.sched
    for i in range(a.warmup):
        await sh.burst(f"w{i}")
    for i in range(a.repeat - 1):      # extra untimed bursts: steady state like bench.py's later steps
        await sh.burst(f"x{i}")
    outs = []
    for rep in range(a.bursts):
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
        sched.engine_spans = eng_calls        # (start, end, pods) of every native engine batch
        # bind round trips: submit (native transport) → completion callback on the loop
        submits: dict = {}
        rtts: list = []
        nat = sched.native
        orig_bind = nat.bind if nat is not None else None
        orig_many = nat.bind_many if nat is not None else None

        def traced(uid, cb, now):
            submits[uid] = now

            def done(status, body, uid=uid, cb=cb):
                t = time.perf_counter()
                rtts.append((submits.get(uid, t), t))
                return cb(status, body)
            return done

        def bind(ns, name, uid, node, ann, cb, timeout=0.0):
            return orig_bind(ns, name, uid, node, ann, traced(uid, cb, time.perf_counter()), timeout)

        def bind_many(binds, cbs, timeout=0.0):
            now = time.perf_counter()
            return orig_many(binds, [traced(b[2], cb, now) for b, cb in zip(binds, cbs)], timeout)
        if nat is not None:
            nat.bind = bind
            nat.bind_many = bind_many
        tr = sched.tracer
        dev_trace = a.device_trace and sched.engine.device_enabled
        if dev_trace:
            from yoda_scheduler_amd.ops import device_scorer as ds
            ds.batch_trace(sched.engine, True)
        import gc
        gc_pauses: list = []
        gc_t = [0.0]

        def gc_cb(phase, info):
            if phase == "start":
                gc_t[0] = time.perf_counter()
            else:
                gc_pauses.append((info.get("generation"), time.perf_counter() - gc_t[0], info.get("collected", 0)))
        gc.callbacks.append(gc_cb)
        from yoda_scheduler_amd.ops.native import core
        lk0 = core().engine_lock_stats()
        # event-loop idle time: the time the loop's selector spends blocked in select()
        sel = asyncio.get_event_loop()._selector
        orig_select = sel.select
        idle = [0.0, 0]

        def timed_select(timeout=None):
            t = time.perf_counter()
            try:
                return orig_select(timeout)
            finally:
                idle[0] += time.perf_counter() - t
                idle[1] += 1
        sel.select = timed_select
        t0 = time.perf_counter()
        c0 = time.thread_time()
        t0_us = tr.now_us()
        res = await sh.burst(f"s{rep}")
        t1 = time.perf_counter()
        c1 = time.thread_time()
        lk1 = core().engine_lock_stats()
        sel.select = orig_select
        gc.callbacks.remove(gc_cb)
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
               "gc": {"collections": len(gc_pauses), "pause_ms_total": round(sum(p[1] for p in gc_pauses) * 1000, 3),
                      "pause_ms_max": round(max((p[1] for p in gc_pauses), default=0) * 1000, 3),
                      "by_generation": {str(g): sum(1 for p in gc_pauses if p[0] == g) for g in (0, 1, 2)}},
               "latency_ms": {"p50": round(sorted(res.latencies_s)[len(res.latencies_s) // 2] * 1000, 3),
                              "p99": round(sorted(res.latencies_s)[int(len(res.latencies_s) * 0.99)] * 1000, 3)}
               if res.latencies_s else None,
               "device_cycles": sched.engine.device_cycles,
               "engine_lock_contended(n,wait_us)": [lk1[0] - lk0[0], lk1[1] - lk0[1]],
               "loop_idle_ms": round(idle[0] * 1000, 3), "loop_selects": idle[1],
               # main-thread CPU time: (wall - idle) - cpu ≈ time the loop thread was runnable but
               # blocked (GIL hand-offs to the engine worker, lock waits, page faults)
               "main_cpu_ms": round((c1 - c0) * 1000, 3),
               "reset_ms": round(getattr(sh, "last_reset_s", 0.0) * 1000, 3)}
        if dev_trace:
            trc = ds.read_batch_trace(sched.engine)
            if trc:
                out["k_batch_last_chunk"] = {"pods": len(trc), "grid_npb": ds.batch_geometry(sched.engine),
                                             "phase_us_mean": {k: round(sum(x[k] for x in trc) / len(trc), 2)
                                                               for k in trc[0]}}
        out["burst"] = rep
        if nat is not None:
            nat.bind = orig_bind
            nat.bind_many = orig_many
            rr = sorted((e - s0) * 1000 for s0, e in rtts)
            subs = sorted((s0 - ta) * 1000 for s0, _ in rtts)
            out["bind_submit_ms"] = {"first": pct(subs, 0), "p50": pct(subs, .5), "last": pct(subs, 1)}
            out["bind_rtt_ms"] = {"p50": pct(rr, .5), "p90": pct(rr, .9), "max": pct(rr, 1)}
        outs.append(out)
        sched.engine_spans = None
        q.add, q.pop_batch = orig_add, orig_pb
    await sh.stop()
    return outs


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=6)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--overlap", default="auto")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--repeat", type=int, default=1, help="untimed bursts before the traced ones")
    ap.add_argument("--bursts", type=int, default=1, help="consecutive traced bursts (one JSON line each)")
    ap.add_argument("--device-trace", action="store_true", help="k_batch phase stamps of the last chunk")
    ap.add_argument("--overlap-depth", type=int, default=0, help="yodaRuntime.overlapDepth (0: config default)")
    a = ap.parse_args()
    try:
        import torch  # noqa: F401 - share torch's HIP runtime, as bench.py does
    except ImportError:
        pass
    for o in asyncio.run(run(a)):
        print(json.dumps(o), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
