#!/usr/bin/env python3
"""How often k_batch's record 1 would repeat from one pod to the next (VERDICT r5 next #5:
measure before building). Record 1 is the first of the three dependent exchanges per pod: the
six per-metric maxima over the pod's eligible cards on feasible nodes, the feasible count and
the reason histogram. CPU engine only (the same policy the device runs, bit-exact).

For a burst of the bench's label mix (BASELINE configs 3/5/6: ``workloads._mixed_labels``) on
a synthetic 4096-node cluster, each pod is placed in order and, before its placement, compared
with the previous pod:

* ``same_template``: identical GPU labels (the only per-pod input of the maxima);
* ``maxima_equal``: the six maxima equal the previous pod's;
* ``maxima_equal_first``: they equal the first pod's (a cluster-wide constant);
* ``feasible_equal`` / ``reasons_equal`` / ``record_equal`` (all of record 1).

    python scripts/record1_reuse.py --nodes 4096 --pods 1000 --busy 0.3 0.5
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(nodes: int, pods: int, busy: float, seed: int) -> dict:
    from yoda_scheduler_amd.bench.workloads import _mixed_labels
    from yoda_scheduler_amd.models.pod import PodInfo
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core, pod_req
    eng = core().Engine(False, 1)
    eng.set_percentage_of_nodes_to_score(100)
    ds.synthetic_cluster(eng, nodes, seed=seed, busy=busy)
    rng = random.Random(seed + 1)
    n = {"pods": 0, "same_template": 0, "maxima_equal": 0, "maxima_equal_first": 0, "feasible_equal": 0,
         "reasons_equal": 0, "record_equal": 0, "maxima_equal_given_other_template": 0, "other_template": 0}
    prev = first = None
    for k in range(pods):
        labels = _mixed_labels(rng)
        pi = PodInfo.from_obj({"metadata": {"name": f"p{k}", "uid": f"p{seed}-{k}", "labels": labels},
                               "spec": {"containers": [{"name": "c", "resources": {"requests": {
                                   "cpu": "100m", "memory": "128Mi"}}}]}})
        req = pod_req(eng, pi)
        feas, reasons = eng.feasible_nodes(req, [], True)
        mx = tuple(eng.maxima(req, feas)) if feas else None
        rec = (tuple(sorted(labels.items())), mx, len(feas), tuple(reasons))
        if first is None:
            first = rec
        if prev is not None:
            n["pods"] += 1
            same = rec[0] == prev[0]
            n["same_template"] += same
            n["maxima_equal"] += rec[1] == prev[1]
            n["maxima_equal_first"] += rec[1] == first[1]
            n["feasible_equal"] += rec[2] == prev[2]
            n["reasons_equal"] += rec[3] == prev[3]
            n["record_equal"] += rec[1:] == prev[1:]
            if not same:
                n["other_template"] += 1
                n["maxima_equal_given_other_template"] += rec[1] == prev[1]
        prev = rec
        eng.schedule(pi.num_id, req, True)
    out = {"nodes": nodes, "busy": busy, "pods": n["pods"]}
    for key, v in n.items():
        if key not in ("pods", "other_template", "maxima_equal_given_other_template"):
            out[key] = round(v / max(1, n["pods"]), 4)
    out["maxima_equal_given_other_template"] = round(n["maxima_equal_given_other_template"] / max(1, n["other_template"]), 4)
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--pods", type=int, default=1000)
    ap.add_argument("--busy", type=float, nargs="+", default=[0.3, 0.5])
    ap.add_argument("--seed", type=int, default=4096)
    a = ap.parse_args()
    for busy in a.busy:
        print(json.dumps(run(a.nodes, a.pods, busy, a.seed)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
