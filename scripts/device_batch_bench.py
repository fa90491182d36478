#!/usr/bin/env python3
"""Engine-level throughput of a burst on a large synthetic cluster: per-pod device cycles
(one host round trip each) vs batched device cycles (yoda_dev_schedule_batch: cycles
enqueued back to back, winners assumed on the device). One JSON line per (nodes, mode)."""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(nodes: int, mode: str, pods: int, batch: int) -> dict:
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core, pod_req
    eng = core().Engine(False, 1)
    eng.set_percentage_of_nodes_to_score(100)
    ds.synthetic_cluster(eng, nodes, seed=nodes, busy=0.3)
    ds.enable(eng, 0, capacity=nodes + 16, min_nodes=1)
    rng = random.Random(1)
    reqs = []
    for k in range(pods):
        pi, req = ds.random_request(eng, rng, f"{mode}-{nodes}-{k}")
        reqs.append((pi.num_id, req))
    # warm up (kernels, first full-table upload)
    eng.schedule_batch([p for p, _ in reqs[:8]], [r for _, r in reqs[:8]])
    t0 = time.perf_counter()
    if mode == "batch":
        for i in range(8, pods, batch):
            chunk = reqs[i:i + batch]
            eng.schedule_batch([p for p, _ in chunk], [r for _, r in chunk])
    else:
        for p, r in reqs[8:]:
            eng.schedule(p, r, True)
    dt = time.perf_counter() - t0
    n = pods - 8
    return {"nodes": nodes, "mode": mode, "pods": n, "batch": batch if mode == "batch" else 1,
            "us_per_pod": round(dt / n * 1e6, 1), "pods_per_s": round(n / dt, 1),
            "device_cycles": eng.device_cycles, "fallbacks": eng.device_fallbacks}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", default="1024,4096,16384")
    ap.add_argument("--pods", type=int, default=520)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    import torch  # noqa: F401 - load torch's HIP runtime first (same SONAME as ours)
    for n in (int(x) for x in a.nodes.split(",")):
        for mode in ("per-pod", "batch"):
            print(json.dumps(run(n, mode, a.pods, a.batch)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
