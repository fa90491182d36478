#!/usr/bin/env python3
"""What k_batch's score columns cost, by phase: 200-pod batches on a zoned cloud pool
(``device_scorer.cloud_cluster``) of pods that need no column (``plain``), an ImageLocality
column only (``image``), PodTopologySpread columns only (``spread``), or both (``both``).
One JSON line per kind: wall µs per pod (engine.schedule_batch) and block 0's per-phase µs
(``read_batch_trace``) of the last batch.

    python scripts/cols_trace.py --nodes 4096 --batches 3
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

KINDS = {"plain": ("rocm/pytorch", 0.0), "image": ("docker.io/rocm/vllm:v0.6.4", 0.0),
         "spread": ("rocm/pytorch", 1.0), "both": ("docker.io/rocm/vllm:v0.6.4", 1.0)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--batch", type=int, default=200)
    ap.add_argument("--kinds", default=",".join(KINDS))
    a = ap.parse_args()
    import torch  # noqa: F401 - load torch's HIP runtime first (same SONAME as ours)
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core, pod_req
    for kind in a.kinds.split(","):
        image, trainer = KINDS[kind]
        eng = core().Engine(False, 1)
        ds.cloud_cluster(eng, a.nodes, 31)
        ds.enable(eng, 0, capacity=a.nodes + 16, min_nodes=1)
        rng = random.Random(7)
        walls = []
        for b in range(a.batches + 1):
            pods = [ds.cloud_pod(eng, rng, f"{kind}-{b}-{k}", image=image, trainer=trainer) for k in range(a.batch)]
            reqs = [pod_req(eng, p) for p in pods]
            if b == a.batches:
                ds.batch_trace(eng, True)
            t = time.perf_counter()
            eng.schedule_batch([p.num_id for p in pods], reqs)
            if b:
                walls.append((time.perf_counter() - t) / len(pods) * 1e6)
        tr = ds.read_batch_trace(eng)
        ds.batch_trace(eng, False)
        keys = list(dict.fromkeys(k for x in tr for k in x))
        phases = {k: round(sum(x[k] for x in tr if k in x) / max(1, sum(k in x for x in tr)), 2) for k in keys}
        print(json.dumps({"kind": kind, "nodes": a.nodes, "batch": a.batch, "us_per_pod": [round(w, 2) for w in walls],
                          "device_batches": eng.device_batches, "fallbacks": eng.device_fallbacks,
                          "kbatch_pods": ds.counters(eng)["kbatch_pods"], "phase_us_mean": phases}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
