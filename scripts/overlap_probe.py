#!/usr/bin/env python3
"""Where the per-batch time goes with native batches inline vs overlapped (config 6 on
the device scorer by default): engine call (worker thread or inline), batch preparation,
result application, and everything else the event loop does between batches."""
import argparse
import asyncio
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from yoda_scheduler_amd.bench.harness import Shard  # noqa: E402
from yoda_scheduler_amd.bench.workloads import make_workload  # noqa: E402
from yoda_scheduler_amd.framework import scheduler as S  # noqa: E402


class TimedEngine:
    def __init__(self, e, acc, server=None):
        self._e, self._acc, self._srv = e, acc, server

    def __getattr__(self, n):
        return getattr(self._e, n)

    def schedule_batch(self, ids, reqs):
        t = time.perf_counter()
        b0 = len(self._srv.bind_log) if self._srv is not None else 0
        try:
            return self._e.schedule_batch(ids, reqs)
        finally:
            self._acc["engine_s"] += time.perf_counter() - t
            if self._srv is not None:     # binds the event loop completed meanwhile
                self._acc["binds_during_engine"] += len(self._srv.bind_log) - b0
            self._acc["batches"] += 1
            self._acc["pods"] += len(ids)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=6)
    ap.add_argument("--device", default="on")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--modes", default="off,on,off,on")
    ap.add_argument("--switch-interval", type=float, default=0.0,
                    help="sys.setswitchinterval (s) for the run; 0 keeps Python's 5 ms default")
    a = ap.parse_args()
    if a.switch_interval > 0:
        sys.setswitchinterval(a.switch_interval)
    out = []
    for mode in a.modes.split(","):
        acc = collections.Counter()
        orig_prep, orig_fin = S.Scheduler._prepare_run, S.Scheduler._finish_run

        def prep(self, *x, _o=orig_prep):
            t = time.perf_counter()
            try:
                return _o(self, *x)
            finally:
                acc["prepare_s"] += time.perf_counter() - t

        def fin(self, *x, _o=orig_fin):
            t = time.perf_counter()
            try:
                return _o(self, *x)
            finally:
                acc["finish_s"] += time.perf_counter() - t
        S.Scheduler._prepare_run, S.Scheduler._finish_run = prep, fin
        w = make_workload(a.config, seed=0)
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
        shards = [Shard(w, seed=i, device=a.device, overlap=mode, batch=a.batch) for i in range(a.steps + 1)]
        for s in shards:
            loop.run_until_complete(s.start())
            s.sched.engine = TimedEngine(s.sched.engine, acc, s.server)
        loop.run_until_complete(shards[0].burst("w"))
        acc.clear()
        t = time.perf_counter()
        res = [loop.run_until_complete(s.burst("s")) for s in shards[1:]]
        el = time.perf_counter() - t
        bound = sum(r.bound for r in res)
        row = {"overlap": mode, "batch": a.batch, "switch_interval": sys.getswitchinterval(), "pods_per_s": round(bound / el), "elapsed_s": round(el, 4),
               "engine_us_per_pod": round(acc["engine_s"] / max(acc["pods"], 1) * 1e6, 2),
               "prepare_us_per_pod": round(acc["prepare_s"] / max(acc["pods"], 1) * 1e6, 2),
               "finish_us_per_pod": round(acc["finish_s"] / max(acc["pods"], 1) * 1e6, 2),
               "wall_us_per_pod": round(el / max(bound, 1) * 1e6, 2),
               "mean_batch": round(acc["pods"] / max(acc["batches"], 1), 1),
               "binds_during_engine_pct": round(100.0 * acc["binds_during_engine"] / max(bound, 1), 1),
               "device_cycles": sum(s.sched.engine.device_cycles for s in shards)}
        print(json.dumps(row), flush=True)
        out.append(row)
        for s in shards:
            loop.run_until_complete(s.stop())
        loop.close()
        S.Scheduler._prepare_run, S.Scheduler._finish_run = orig_prep, orig_fin
    return 0


if __name__ == "__main__":
    sys.exit(main())
