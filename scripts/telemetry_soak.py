#!/usr/bin/env python3
"""Telemetry soak: a fleet of simulated amd-smi sniffers publishing Scv objects for N
nodes while pods that fit nowhere sit parked in the scheduler's unschedulable queue.

Two modes (verdict r1, 'change-driven telemetry plus event-aware requeue'):
  * legacy — every agent PUTs its Scv every second (heartbeat = interval = 1 s) and every
    Scv event moves the whole unschedulable queue (scvQueueingHint off): round 1's design;
  * change — agents publish only on a meaningful change (free HBM ±1 GiB, health, CU
    occupancy, link load) or a 10 s heartbeat, and the scheduler's queueing hint requeues
    parked pods only when a node's filter-visible capacity grew.

Tenant load is a random walk: every simulated second each GPU's used HBM moves by up to
±64 MiB (noise), and with probability ``--job-rate`` per node a job starts or ends on 1–4
GPUs (±30 GiB). Each simulated second takes one wall second (``--fast``: as fast as
the process goes), so the scheduler's backoff timers (deploy defaults 1 s → 10 s) run in
real time; the sniffer agents use the simulated clock. Reported per mode: apiserver Scv writes per simulated
second, the scheduler's own CPU per simulated second (Scv handlers + scheduling cycles,
timed around the calls), parked-pod scheduling attempts per simulated second, and how
many real capacity increases were caught (jobs ending → pods that fit get bound).

    python scripts/telemetry_soak.py --nodes 1000 --seconds 20 --parked 50
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


async def soak(mode: str, nodes: int, seconds: int, parked: int, job_rate: float, seed: int,
               realtime: bool = True) -> dict:
    from yoda_scheduler_amd.sniffer.collector import FakeBackend
    from yoda_scheduler_amd.sniffer.publisher import SnifferAgent
    from yoda_scheduler_amd.testing import FakeCluster, yoda_config

    legacy = mode == "legacy"
    cfg = yoda_config(batch=256, backoff=1.0, max_backoff=10.0)     # the shipped deploy's backoff
    cfg["yodaRuntime"]["scvQueueingHint"] = not legacy
    cfg["yodaRuntime"]["unschedulableFlushSeconds"] = 60.0              # upstream default (tests use 5 s)
    c = FakeCluster(cfg, seed=seed)
    rng = random.Random(seed)
    sim = [0.0]
    backends, agents = [], []
    for i in range(nodes):
        name = f"n{i:04d}"
        c.add_node(name, scv=False)
        be = FakeBackend(seed=seed * 100003 + i, node=name)
        for st in be.state:
            st.used_mb = rng.randint(0, 120_000)
        backends.append(be)
        agents.append(SnifferAgent(c.client, name, be, interval=1.0, heartbeat=1.0 if legacy else 10.0,
                                   clock=lambda: sim[0]))
    for a in agents:                     # first publish (creates the Scv objects)
        await a.publish_once(force=True)
    sched = await c.start()
    # the scheduler's own time: Scv handlers and scheduling cycles
    spent = [0.0]

    def timed(fn):
        def w(*args, **kw):
            t = time.perf_counter()
            try:
                return fn(*args, **kw)
            finally:
                spent[0] += time.perf_counter() - t
        return w
    sched.on_scv_update = timed(sched.on_scv_update)
    sched.informers["scvs"].on_update = sched.on_scv_update
    sched.schedule_one = timed(sched.schedule_one)
    sched.schedule_batch = timed(sched.schedule_batch)
    for k in range(parked):              # fit nowhere: 400 GB on one card
        c.add_pod(f"parked-{k}", {"scv/memory": "400000"})
    await c.wait(lambda: len(sched.queue._unsched) >= parked, 10.0)
    # pods that fit only once a job ends somewhere: 250 GB on one GPU
    fit_after = 0
    w0 = sum(a.published for a in agents)
    f0, s0 = sched.failed, spent[0]
    m0, k0 = sched.scv_requeues, sched.scv_requeue_skips
    t_wall = time.perf_counter()
    jobs_ended = 0
    for sec in range(seconds):
        sim[0] = float(sec + 1)
        t_tick = time.perf_counter()
        for be in backends:
            for st in be.state:
                st.used_mb = min(be.spec.hbm_mb, max(0, st.used_mb + rng.randint(-64, 64)))
            if rng.random() < job_rate:
                gpus = rng.sample(range(be.gpus), rng.choice([1, 2, 4]))
                delta = 30_000 if rng.random() < 0.5 else -30_000
                jobs_ended += delta < 0
                for g in gpus:
                    st = be.state[g]
                    st.used_mb = min(be.spec.hbm_mb, max(0, st.used_mb + delta))
        for a in agents:
            await a.publish_once(force=legacy)
        if sec == seconds // 2:
            # a pod that needs ~250 GB free on one card: fits once a tenant frees a card
            for be in backends[: max(1, nodes // 100)]:
                be.state[0].used_mb = 1_000
            c.add_pod("fits-after-free", {"scv/memory": "250000"})
            fit_after = 1
        # let informers and the scheduling loop catch up; in real time, pace to 1 s per tick
        # so the scheduler's backoff timers see real seconds
        await asyncio.sleep(max(0.01, (1.0 - (time.perf_counter() - t_tick)) if realtime else 0.01))
    await asyncio.sleep(0.3)
    wall = time.perf_counter() - t_wall
    out = {
        "mode": mode, "nodes": nodes, "simulated_s": seconds, "parked": parked,
        "scv_writes_per_s": round((sum(a.published for a in agents) - w0) / seconds, 1),
        "agent_samples_skipped": sum(a.skipped for a in agents),
        "scheduler_cpu_ms_per_s": round((spent[0] - s0) * 1000 / seconds, 2),
        "parked_attempts_per_s": round((sched.failed - f0) / seconds, 1),
        "scv_requeues": sched.scv_requeues - m0, "scv_requeue_skips": sched.scv_requeue_skips - k0,
        "fits_after_free_bound": bool(fit_after and c.node_of("fits-after-free")),
        "still_parked": len(sched.queue._unsched), "wall_s": round(wall, 2),
    }
    await c.stop()
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--seconds", type=int, default=20)
    ap.add_argument("--parked", type=int, default=50)
    ap.add_argument("--job-rate", type=float, default=0.01)
    ap.add_argument("--mode", choices=["legacy", "change", "both"], default="both")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--fast", action="store_true", help="do not pace simulated seconds to wall seconds")
    a = ap.parse_args()
    for m in (["legacy", "change"] if a.mode == "both" else [a.mode]):
        print(json.dumps(asyncio.run(soak(m, a.nodes, a.seconds, a.parked, a.job_rate, a.seed, not a.fast))), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
