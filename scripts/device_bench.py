#!/usr/bin/env python3
"""Per-cycle latency of the native engine: CPU path vs the gfx950 device scorer on large
synthetic MI355X clusters (8 GPUs/node). Prints one JSON line per (nodes, pod kind, path).

CPU rows are measured twice: scoring every feasible node (pct=100, same work as the device)
and with upstream's adaptive percentageOfNodesToScore sampling (pct=0).
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(nodes: int, kind: str, path: str, pods: int, threads: int) -> dict:
    from yoda_scheduler_amd.models.pod import PodInfo
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core, pod_req
    eng = core().Engine(False, threads)
    eng.set_percentage_of_nodes_to_score(0 if path == "cpu-adaptive" else 100)
    ds.synthetic_cluster(eng, nodes, seed=nodes, busy=0.3)
    if path == "gpu":
        ds.enable(eng, 0, capacity=nodes + 16, min_nodes=1)
    labels = {"single": {"scv/memory": "4096"}, "gang4": {"scv/number": "4", "scv/memory": "4096"},
              "gang8": {"scv/number": "8", "scv/memory": "1024"}}[kind]
    ts, dev_us = [], []
    for k in range(pods + 5):
        pi = PodInfo.from_obj({"metadata": {"name": f"b{k}", "uid": f"{path}-{nodes}-{kind}-{k}", "labels": labels},
                               "spec": {}})
        req = pod_req(eng, pi)
        t0 = time.perf_counter()
        res = eng.schedule(pi.num_id, req, True)
        dt = time.perf_counter() - t0
        if k >= 5:
            ts.append(dt * 1e6)
        assert res[0] >= 0, res
    if path == "gpu":
        # kernel time (events around the launches) in a separate pass: timing adds a sync
        eng.device_set_timing(True)
        for k in range(max(10, pods // 4)):
            pi = PodInfo.from_obj({"metadata": {"name": f"t{k}", "uid": f"t-{nodes}-{kind}-{k}", "labels": labels},
                                   "spec": {}})
            eng.schedule(pi.num_id, pod_req(eng, pi), True)
            dev_us.append(eng.device_last_us())
        eng.device_set_timing(False)
    out = {"nodes": nodes, "gpus": nodes * 8, "pod": kind, "path": path, "threads": threads,
           "cycle_us_p50": round(statistics.median(ts), 1), "cycle_us_p90": round(sorted(ts)[int(len(ts) * .9)], 1),
           "pods_per_s": round(1e6 / statistics.mean(ts), 1)}
    if dev_us:
        out["device_kernels_us_p50"] = round(statistics.median(dev_us), 1)
        out["device_cycles"] = eng.device_cycles
        out["fallbacks"] = eng.device_fallbacks
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", default="1024,4096,16384,65536")
    ap.add_argument("--pods", type=int, default=100)
    ap.add_argument("--kinds", default="single,gang4,gang8")
    ap.add_argument("--paths", default="gpu,cpu,cpu-adaptive")
    ap.add_argument("--threads", type=int, default=1)
    a = ap.parse_args()
    for n in map(int, a.nodes.split(",")):
        for kind in a.kinds.split(","):
            for path in a.paths.split(","):
                print(json.dumps(bench(n, kind, path, a.pods, a.threads)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
