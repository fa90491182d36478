#!/usr/bin/env python3
"""Engine-level throughput of a burst on a large synthetic cluster: per-pod device cycles
(one host round trip each) vs batched device cycles (yoda_dev_schedule_batch) as per-pod launch
chains enqueued back to back (``batch-chain``) or as ONE persistent k_batch dispatch per batch
(``batch``, node rows resident in LDS), against the CPU engine alone (``cpu``: the same batches
on one engine thread, no device attached — where the two cross is ``deviceScorer.minNodes``).
One JSON line per (nodes, mode)."""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench_request(engine, rng: random.Random, uid: str):
    """A pod of the bench's BASELINE label mix (configs 3/5/6: 70 % one GPU, 18 % two, 9 %
    four, 3 % eight) with the bench's container requests."""
    from yoda_scheduler_amd.bench.workloads import _mixed_labels
    from yoda_scheduler_amd.models.pod import PodInfo
    from yoda_scheduler_amd.ops.native import pod_req
    pi = PodInfo.from_obj({"metadata": {"name": uid, "uid": uid, "labels": _mixed_labels(rng)},
                           "spec": {"containers": [{"name": "c", "resources": {"requests": {
                               "cpu": "100m", "memory": "128Mi"}}}]}})
    return pi, pod_req(engine, pi)


def run(nodes: int, mode: str, pods: int, batch: int, trace: bool = False, busy: float = 0.3,
        mix: str = "random") -> dict:
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core, pod_req
    eng = core().Engine(False, 1)
    eng.set_percentage_of_nodes_to_score(100)
    ds.synthetic_cluster(eng, nodes, seed=nodes, busy=busy)
    # batch-chain: per-pod launch chains enqueued back to back; batch: the persistent k_batch
    if mode != "cpu":
        os.environ["YODA_DEV_PERSIST"] = "0" if mode == "batch-chain" else "1"
        ds.enable(eng, 0, capacity=nodes + 16, min_nodes=1)
        os.environ.pop("YODA_DEV_PERSIST", None)
    rng = random.Random(1)
    reqs, ks = [], []
    for k in range(pods):
        make = bench_request if mix == "bench" else ds.random_request
        pi, req = make(eng, rng, f"{mode}-{nodes}-{k}")
        reqs.append((pi.num_id, req))
        ks.append(pi.gpu.number if pi.gpu.has_number else 1)
    # warm up (kernels, first full-table upload)
    eng.schedule_batch([p for p, _ in reqs[:8]], [r for _, r in reqs[:8]])
    t0 = time.perf_counter()
    if mode.startswith("batch") or mode == "cpu":
        for i in range(8, pods, batch):
            chunk = reqs[i:i + batch]
            eng.schedule_batch([p for p, _ in chunk], [r for _, r in chunk])
    else:
        for p, r in reqs[8:]:
            eng.schedule(p, r, True)
    dt = time.perf_counter() - t0
    n = pods - 8
    extra = {}
    if mode == "batch":
        grid, npb = ds.batch_geometry(eng)
        extra["grid"], extra["nodes_per_block"] = grid, npb
        if trace:
            ds.batch_trace(eng, True)
            chunk = reqs[8:8 + batch]
            eng.schedule_batch([p for p, _ in chunk], [r for _, r in chunk])
            tr = ds.read_batch_trace(eng)
            if tr:
                keys = list(dict.fromkeys(k for x in tr for k in x))   # owner phases: pods with a fix-up
                extra["phase_us_mean"] = {k: round(sum(x[k] for x in tr if k in x) / sum(k in x for x in tr), 2)
                                          for k in keys}
                by_k: dict = {}
                for x, kk in zip(tr, ks[8:8 + len(tr)]):
                    by_k.setdefault(kk, []).append(x["score_a"])
                extra["score_a_us_by_gpus"] = {str(kk): [len(v), round(sum(v) / len(v), 2)]
                                               for kk, v in sorted(by_k.items())}
                by_k = {}
                for x, kk in zip(tr, ks[8:8 + len(tr)]):
                    if "own_sa_score" in x:   # PAIRS: the fix-up owner's score A of the pod
                        by_k.setdefault(kk, []).append(x["own_sa_score"])
                if by_k:
                    extra["own_sa_score_us_by_gpus"] = {str(kk): [len(v), round(sum(v) / len(v), 2)]
                                                        for kk, v in sorted(by_k.items())}
            ds.batch_trace(eng, False)
    return {**extra, "nodes": nodes, "mode": mode, "mix": mix, "pods": n, "batch": batch if mode.startswith("batch") or mode == "cpu" else 1,
            "us_per_pod": round(dt / n * 1e6, 1), "pods_per_s": round(n / dt, 1),
            "device_cycles": eng.device_cycles, "fallbacks": eng.device_fallbacks}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", default="1024,4096,16384")
    ap.add_argument("--pods", type=int, default=520)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--modes", default="per-pod,batch-chain,batch")
    ap.add_argument("--trace", action="store_true", help="k_batch phase breakdown (block 0 stamps)")
    ap.add_argument("--busy", type=float, default=0.3, help="synthetic cluster load (0: every node fits)")
    ap.add_argument("--mix", choices=["random", "bench"], default="random",
                    help="random: the parity suite's request mix; bench: the BASELINE label mix")
    a = ap.parse_args()
    import torch  # noqa: F401 - load torch's HIP runtime first (same SONAME as ours)
    for n in (int(x) for x in a.nodes.split(",")):
        for mode in a.modes.split(","):
            print(json.dumps(run(n, mode, a.pods, a.batch, a.trace, a.busy, a.mix)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
