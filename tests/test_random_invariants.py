"""Randomised end-to-end invariants: mixed SPX/CPX nodes, GPU pods of every size, priorities
(preemption), required anti-affinity, topology spread, deletions mid-run. Whatever the
scheduler decides, at quiescence:

* every GPU's ledger equals the scv/memory of the live pods annotated onto it, ≤ its HBM;
* a bound pod holds exactly scv/number distinct, eligible GPUs of its node;
* required anti-affinity and DoNotSchedule spread constraints hold among bound pods;
* a pending pod is not schedulable as the cluster stands (checked for plain GPU pods:
  no node has scv/number GPUs with scv/memory free).
"""
import asyncio
import random
import time

import pytest

from yoda_scheduler_amd.models.device import make_node, make_scv
from yoda_scheduler_amd.testing import FakeCluster, yoda_config

ZONE = "topology.kubernetes.io/zone"


def run(c):
    return asyncio.run(c)


def _scenario(seed: int):
    rng = random.Random(seed)

    async def go():
        c = FakeCluster(yoda_config(backoff=0.01, max_backoff=0.05, yoda_args={"sampleSettleSeconds": 0.0}))
        nodes = {}
        for i in range(rng.randint(3, 5)):
            name = f"n{i}"
            part = rng.choice(["SPX", "SPX", "CPX"])
            c.server.create("nodes", make_node(name, labels={ZONE: f"z{i % 2}", "kubernetes.io/hostname": name}))
            s = make_scv(name, partition=part, update_time=time.time(),
                         used_mb=[rng.choice([0, 0, 100000]) for _ in range(8 * (8 if part == "CPX" else 1))])
            s.update_interval_ms = 600_000
            c.server.create("scvs", s.to_json())
            nodes[name] = s
        deleted = []                    # every pod deleted by the test or by preemption
        real_delete = c.server.delete

        def delete(res, name, namespace=None):
            if res == "pods":
                deleted.append(name)
            return real_delete(res, name, namespace)
        c.server.delete = delete
        await c.start()
        pods = {}
        for i in range(rng.randint(60, 120)):
            lab = {"scv/memory": str(rng.choice([1000, 8000, 30000, 120000]))}
            k = rng.choice([1, 1, 1, 2, 4, 8])
            if k > 1:
                lab["scv/number"] = str(k)
            extra = {}
            r = rng.random()
            if r < 0.15:
                lab["app"] = "db"
                extra["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                    {"topologyKey": "kubernetes.io/hostname", "labelSelector": {"matchLabels": {"app": "db"}}}]}}
            elif r < 0.3:
                lab["app"] = "web"
                extra["topologySpreadConstraints"] = [{"maxSkew": 2, "topologyKey": ZONE,
                                                       "whenUnsatisfiable": "DoNotSchedule",
                                                       "labelSelector": {"matchLabels": {"app": "web"}}}]
            prio = rng.choice([0, 0, 0, 10, 100])
            name = f"p{i}"
            c.add_pod(name, lab, priority=prio, **extra)
            pods[name] = (lab, extra)
            if rng.random() < 0.1 and pods:
                victim = rng.choice(sorted(pods))
                try:
                    c.server.delete("pods", victim, "default")
                    pods.pop(victim)
                except Exception:
                    pass
            if i % 16 == 0:
                await asyncio.sleep(0.005)
        # quiescence: nothing bound for a while, no binds in flight
        last, stable = -1, 0
        for _ in range(400):
            await asyncio.sleep(0.02)
            n = len(c.server.bind_log)
            stable = stable + 1 if n == last and c.sched.pending_binds == 0 else 0
            last = n
            if stable >= 10:
                break
        live = {}
        labels = {name: lab for name, (lab, _) in pods.items()}
        for name in list(pods):
            try:
                live[name] = c.pod(name)
            except Exception:
                pods.pop(name)
        state = {n: c.sched.cache.node_gpu_state(n) for n in nodes}
        q = c.sched.queue
        diag = {"queue": {pi.name: ("active" if uid in q._active_entries else "backoff" if uid in q._backoff_pods
                                    else "unschedulable", pi.attempts) for uid, pi in q._pods.items()},
                "nominations": {uid: v[0] for uid, v in c.sched.nominations.items()},
                "move_request_cycle": q._move_request_cycle, "cycle": q.scheduling_cycle,
                "deleted_web": sum(1 for n in deleted if labels.get(n, {}).get("app") == "web")}
        await c.stop()
        return nodes, pods, live, state, diag

    return run(go())


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_cluster_invariants(seed):
    nodes, pods, live, state, diag = _scenario(seed)
    want: dict = {}
    bound = {}
    for name, obj in live.items():
        node = (obj.get("spec") or {}).get("nodeName")
        if not node:
            continue
        bound[name] = node
        lab = pods[name][0]
        mem = int(lab["scv/memory"])
        gpus = [int(x) for x in ((obj["metadata"].get("annotations") or {}).get("scv.amd.com/gpus") or "").split(",")
                if x]
        assert len(gpus) == int(lab.get("scv/number", "1")) and len(set(gpus)) == len(gpus), (name, gpus)
        for g in gpus:
            want[(node, g)] = want.get((node, g), 0) + mem
    for node, gs in state.items():
        for g, st in enumerate(gs):
            assert st["reserved"] == want.get((node, g), 0), (node, g, st)
            assert st["reserved"] <= st["total"], (node, g, st)
    # required anti-affinity: at most one bound "db" pod per node
    db_nodes = [bound[n] for n in bound if pods[n][0].get("app") == "db"]
    assert len(db_nodes) == len(set(db_nodes)), db_nodes
    # spread: web pods' zone counts differ by at most maxSkew (2) — checked against the zones
    # that could host them, i.e. both zones exist on every seed. Each bind kept the skew of the
    # scheduler's view ≤ 2; a member deleted afterwards (by the test or as a preemption victim)
    # may widen it by one, so the bound is 2 + the number of deleted web pods.
    web = [bound[n] for n in bound if pods[n][0].get("app") == "web"]
    zones = {z: 0 for z in ("z0", "z1")}
    for n in web:
        zones["z" + str(int(n[1:]) % 2)] += 1
    assert max(zones.values()) - min(zones.values()) <= 2 + diag["deleted_web"], (zones, diag["deleted_web"])
    # pending plain pods really do not fit anywhere (per-GPU effective free HBM)
    for name, obj in live.items():
        lab, extra = pods[name]
        if name in bound or extra or obj.get("spec", {}).get("priority"):
            continue
        k, mem = int(lab.get("scv/number", "1")), int(lab["scv/memory"])
        for node, gs in state.items():
            free = [g for g in gs if g["healthy"] and min(g["free"] - g["pending"], g["total"] - g["reserved"]) >= mem]
            assert len(free) < k, (name, node, k, mem, free, diag)
