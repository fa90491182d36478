#!/usr/bin/env python3
"""DefaultPreemption cost per attempt: the native search (``Engine::preempt``) vs its Python spec
(``plugins.defaults.preempt_spec``, the path pods with Python filters still take) on a full
cluster — every GPU of every node held by a low-priority pod, the preemptor needs a whole
8-GPU node (≤ 5 ms at 4096 nodes × 8 pods).

    python scripts/preempt_bench.py --nodes 512 4096 --attempts 20 [--spec]

One JSON line per cluster size: per-attempt min / median / p99 ms, potential nodes, nodes dry-run,
candidates, victims. With --spec the Python spec is timed too (one attempt per size: it is ~100x
slower)."""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from yoda_scheduler_amd.framework.cache import SchedulerCache  # noqa: E402
from yoda_scheduler_amd.models.device import make_node, make_scv  # noqa: E402
from yoda_scheduler_amd.models.pod import PodInfo  # noqa: E402
from yoda_scheduler_amd.ops.native import core, pod_req  # noqa: E402
from yoda_scheduler_amd.plugins.defaults import preempt_spec  # noqa: E402

CARD_MB = 294912


def full_cluster(n_nodes: int, seed: int):
    rng = random.Random(seed)
    eng = core().Engine(False, 1)
    cache = SchedulerCache(eng)
    for i in range(n_nodes):
        cache.add_node(make_node(f"n{i}"))
        cache.set_scv(make_scv(f"n{i}", update_time=time.time()))
    k = 0
    for i in range(n_nodes):
        for g in range(8):
            prio = rng.randint(0, 5)
            cache.add_pod({"metadata": {"name": f"f{k}", "namespace": "default", "uid": f"pf-{k}",
                                        "labels": {"app": f"job-{k % 17}", "scv/memory": str(CARD_MB)},
                                        "annotations": {"scv.amd.com/gpus": str(g), "scv.amd.com/reserved-mb": str(CARD_MB)}},
                           "spec": {"nodeName": f"n{i}", "priority": prio,
                                    "containers": [{"name": "c", "resources": {"requests": {"cpu": "1"}}}]}})
            k += 1
    return eng, cache


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nodes", type=int, nargs="+", default=[512, 4096])
    ap.add_argument("--attempts", type=int, default=20)
    ap.add_argument("--spec", action="store_true", help="also time the Python spec (one attempt)")
    a = ap.parse_args(argv)
    for n in a.nodes:
        t0 = time.perf_counter()
        eng, cache = full_cluster(n, n)
        setup = time.perf_counter() - t0
        pod = PodInfo.from_obj({"metadata": {"name": "hi", "namespace": "default", "uid": "hi",
                                             "labels": {"scv/memory": str(CARD_MB), "scv/number": "8"}},
                                "spec": {"priority": 100, "containers": [{"name": "c"}]}})
        req = pod_req(eng, pod)
        ts, last = [], None
        for _ in range(a.attempts):
            t = time.perf_counter()
            last = eng.preempt(req, 100, [], 10, 100, -1)
            ts.append((time.perf_counter() - t) * 1e3)
        ts.sort()
        row = {"nodes": n, "pods": n * 8, "attempts": a.attempts, "native_ms_min": round(ts[0], 3),
               "native_ms_median": round(statistics.median(ts), 3),
               "native_ms_p99": round(ts[min(len(ts) - 1, int(len(ts) * 0.99))], 3),
               "potential": last[4], "evaluated": last[5], "candidates": last[6], "victims": len(last[1]),
               "setup_s": round(setup, 1)}
        if a.spec:
            t = time.perf_counter()
            got = preempt_spec(eng, cache, pod, req, [], 10, 100, 0)
            row["spec_ms"] = round((time.perf_counter() - t) * 1e3, 1)
            row["spec_victims"] = len(got[1]) if got else 0
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
