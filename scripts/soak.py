#!/usr/bin/env python3
"""Soak test: many burst → complete → delete rounds through one long-lived scheduler,
with bind faults and watch drops injected, checking that nothing accumulates.

Per round: create a mixed burst (scv/memory, multi-GPU gangs), wait until every pod is
bound, delete them all (the workload finished), wait until the scheduler's cache, the
native HBM ledger and the queue are empty again, and run the cache debugger's comparer
(cache vs informers vs ledger). Reports pods/s per round, RSS and the Python object
count; fails (exit 1) on drift, leftovers, unbound pods or RSS growth past the budget.

    python scripts/soak.py --rounds 40 --pods 1000 --nodes 4
"""
from __future__ import annotations

import argparse
import asyncio
import gc
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rss_mb() -> float:
    try:
        import psutil
        return psutil.Process().memory_info().rss / 2**20
    except ImportError:          # pragma: no cover
        return 0.0


async def soak(rounds: int, pods: int, nodes: int, bind_fail: float, drop_watch: int, seed: int,
               rss_budget_mb: float, log=print) -> dict:
    from yoda_scheduler_amd.bench.workloads import _mixed_labels, pod_object
    from yoda_scheduler_amd.fakeapi.server import FakeApiServer, Faults
    from yoda_scheduler_amd.testing import FakeCluster, yoda_config

    rng = random.Random(seed)
    faults = Faults(bind_fail_ratio=bind_fail, drop_watch_every=drop_watch, seed=seed)
    # the fake apiserver keeps a bounded watch history (etcd's compaction window): small here so
    # its own retention saturates within a round and RSS growth measures the scheduler
    server = FakeApiServer(history=4 * pods, faults=faults)
    c = FakeCluster(yoda_config(batch=256, backoff=0.01, max_backoff=0.05), server=server, seed=seed)
    for i in range(nodes):
        c.add_node(f"node-{i}", interval_ms=3_600_000)
    sched = await c.start()
    srv = c.server
    out = {"rounds": [], "ok": True, "problems": []}
    rss0 = None
    for r in range(rounds):
        srv.reset_logs()
        names = []
        t0 = time.perf_counter()
        for i in range(pods):
            o = pod_object(i, _mixed_labels(rng), "yoda-scheduler", prefix=f"r{r}")
            srv.create("pods", o)
            names.append(o["metadata"]["name"])
            if i % 64 == 63:
                await asyncio.sleep(0)
        bound = await c.wait(lambda: len(srv.bind_log) >= pods, timeout=120, step=0.002)
        dt = time.perf_counter() - t0
        for n in names:
            srv.delete("pods", n, "default")
            if len(names) > 256 and names.index(n) % 256 == 255:
                await asyncio.sleep(0)
        drained = await c.wait(lambda: not sched.cache.pods and sched.engine.ledger_size == 0 and not len(sched.queue)
                               and sched.pending_binds == 0, timeout=30, step=0.005)
        await asyncio.sleep(0.05)
        drift = sched.debugger.drift()
        reserved = sum(g["reserved"] for n in sched.cache.nodes for g in sched.cache.node_gpu_state(n))
        gc.collect()
        rss = _rss_mb()
        if r == 1:
            rss0 = rss
        row = {"round": r, "bound": len(srv.bind_log), "pods_per_s": round(len(srv.bind_log) / dt, 1),
               "drained": drained, "drift": drift, "reserved_mb_left": reserved, "rss_mb": round(rss, 1),
               "objects": len(gc.get_objects()), "bind_errors": sched.bind_errors,
               "device_cycles": sched.engine.device_cycles, "device_fallbacks": sched.engine.device_fallbacks,
               "relists": sum(inf.relists for inf in sched.informers.values())}
        out["rounds"].append(row)
        log(json.dumps(row))
        for bad, what in ((not bound, "unbound pods"), (not drained, "cache/ledger/queue not drained"),
                          (bool(drift), f"drift {drift}"), (reserved != 0, f"{reserved} MB still reserved")):
            if bad:
                out["ok"] = False
                out["problems"].append(f"round {r}: {what}")
    if rss0 is not None and rounds > 2 and out["rounds"][-1]["rss_mb"] - rss0 > rss_budget_mb:
        out["ok"] = False
        out["problems"].append(f"RSS grew {out['rounds'][-1]['rss_mb'] - rss0:.1f} MB after round 1")
    out["ledger_size"] = sched.engine.ledger_size
    await c.stop()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--pods", type=int, default=1000)
    ap.add_argument("--nodes", type=int, default=4)
    ap.add_argument("--bind-fail", type=float, default=0.02)
    ap.add_argument("--drop-watch", type=int, default=5000, help="close watches every N events (0 = never)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--rss-budget-mb", type=float, default=64.0)
    a = ap.parse_args(argv)
    res = asyncio.run(soak(a.rounds, a.pods, a.nodes, a.bind_fail, a.drop_watch, a.seed, a.rss_budget_mb))
    print(json.dumps({"ok": res["ok"], "problems": res["problems"], "ledger_size": res["ledger_size"],
                      "rounds": len(res["rounds"])}))
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
