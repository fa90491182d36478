#!/usr/bin/env python3
"""Per-pod engine cost of the default plugins that read other pods, on a cluster with many
reserved pods (CPU engine, one ``Engine.schedule`` call per probe pod, median of 30-50).

    python scripts/engine_scale_bench.py [--nodes 64] [--pods-per-node 150]

Scenarios:
  pref     a pod with a preferred hostname anti-affinity term (single-label selector) among
           pods without terms — InterPodAffinity scoring counts matching pods per node
  spread   a ReplicaSet-owned pod whose DefaultSelector has two labels (app + pod-template-hash),
           PodTopologySpread System defaults (ScheduleAnyway) — per-node counts of a multi-label
           selector
  holders  a plain pod (and one whose labels match) beside pods that all carry a preferred
           anti-affinity term — the existing pods' terms are checked against the new pod
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from yoda_scheduler_amd.models.device import make_node, make_scv  # noqa: E402
from yoda_scheduler_amd.models.pod import NodeInfo, PodInfo  # noqa: E402
from yoda_scheduler_amd.models.selectors import LabelSelector  # noqa: E402
from yoda_scheduler_amd.ops.native import core, pod_req, push_node, push_scv  # noqa: E402

C = core()
_uid = [0]


def _pod(labels, spec=None, owner=False):
    _uid[0] += 1
    meta = {"name": f"p{_uid[0]}", "namespace": "default", "uid": f"u{_uid[0]}", "labels": labels}
    if owner:
        meta["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs3", "uid": "rs3",
                                    "controller": True}]
    return PodInfo.from_obj({"metadata": meta, "spec": dict(
        {"schedulerName": "yoda-scheduler", "containers": [{"name": "c", "resources": {"requests": {"cpu": "10m"}}}]},
        **(spec or {}))})


def _anti(app):
    return {"affinity": {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 100, "podAffinityTerm": {"topologyKey": "kubernetes.io/hostname",
                                            "labelSelector": {"matchLabels": {"app": app}}}}]}}}


def _engine(nodes: int):
    e = C.Engine(False, 1)
    for i in range(nodes):
        idx = push_node(e, NodeInfo.from_obj(make_node(f"n{i}", pods=100000,
                                                       labels={"topology.kubernetes.io/zone": f"z{i % 3}"})))
        push_scv(e, idx, make_scv(f"n{i}", gpus=8, update_time=time.time()), False)
    return e


def _median_us(e, make, reps=40):
    ts = []
    for _ in range(reps):
        pi = make()
        r = pod_req(e, pi)
        t = time.perf_counter()
        e.schedule(pi.num_id, r, False)
        ts.append(time.perf_counter() - t)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 1)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=64)
    ap.add_argument("--pods-per-node", type=int, default=150)
    a = ap.parse_args()
    out = {"nodes": a.nodes, "reserved_pods": a.nodes * a.pods_per_node}

    e = _engine(a.nodes)
    e.set_score_weight(C.S_INTERPOD, 1)
    for i in range(a.nodes):
        for j in range(a.pods_per_node):
            pi = _pod({"app": f"a{j % 10}"})
            e.reserve(pi.num_id, pod_req(e, pi), i, [j % 8])
    out["pref_us"] = _median_us(e, lambda: _pod({"app": "a3"}, _anti("a3")))

    e = _engine(a.nodes)
    e.set_score_weight(C.S_SPREAD, 1)
    e.set_spread_defaults([("kubernetes.io/hostname", 3, "ScheduleAnyway"),
                           ("topology.kubernetes.io/zone", 5, "ScheduleAnyway")])
    e.set_controller("replicasets", "default", "rs3",
                     LabelSelector({"matchLabels": {"app": "a3", "pod-template-hash": "h3"}}).native())
    for i in range(a.nodes):
        for j in range(a.pods_per_node):
            pi = _pod({"app": f"a{j % 10}", "pod-template-hash": f"h{j % 10}"})
            e.reserve(pi.num_id, pod_req(e, pi), i, [j % 8])
    out["spread_us"] = _median_us(e, lambda: _pod({"app": "a3", "pod-template-hash": "h3"}, owner=True))

    e = _engine(a.nodes)
    e.set_score_weight(C.S_INTERPOD, 1)
    e.filters = C.F_INTERPOD
    for i in range(a.nodes):
        for j in range(a.pods_per_node):
            pi = _pod({"app": f"a{j % 10}"}, _anti(f"a{j % 10}"))
            e.reserve(pi.num_id, pod_req(e, pi), i, [j % 8])
    out["holders_plain_us"] = _median_us(e, lambda: _pod({"app": "zz"}))
    out["holders_matching_us"] = _median_us(e, lambda: _pod({"app": "a3"}))
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
