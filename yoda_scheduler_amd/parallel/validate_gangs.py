"""Gang-placement validation: does the GPU set the scheduler picks for
a k-GPU pod actually get better collective bandwidth than the set its objective ranks worst?

The reference has no notion of *which* GPUs a multi-GPU pod gets (``scv/number`` only counts
cards, ``/root/reference/pkg/yoda/filter/filter.go:11-16``); this framework chooses the set
by xGMI link load, NUMA locality, HBM headroom and occupancy (``Engine::select_gpus``,
``parallel/gang.py``). This harness closes the loop on one node, one process per GPU:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m yoda_scheduler_amd.parallel.validate_gangs --k 4 --load-pairs 0-1,2-3

rank 0
  1. loads the ``--load-pairs`` xGMI links with gfx950 peer-write streams (``ops/hip.py``
     ``peer_write_bandwidth``) on a background thread that keeps running through step 4;
  2. samples amd-smi twice (C++ collector; link load from the counter deltas) and builds the
     node's ``Scv`` exactly as the sniffer publishes it;
  3. places a ``scv/number=k`` pod on that node through the native engine — the scheduler's
     own code path — (best set) and enumerates every k-subset with the Python reference
     objective (``parallel/gang.objective``) for the set it ranks worst;
every rank
  4. joins an all-reduce over the ranks of each set (rank r = HIP ordinal r; the card's
     ``hipId`` from the sample maps amd-smi order to ranks) and times it
     (``parallel/rccl_probe.allreduce_bandwidth``, RCCL over xGMI with backend ``nccl``).

Rank 0 prints one JSON line: both sets, their objectives and link terms, bus bandwidth of
each and the ratio. ``--fake`` replaces amd-smi by ``FakeBackend`` with ``--fake-load``
link loads (a CPU rehearsal under gloo: there is no xGMI, so the two sets' bandwidths are
the host's and their ratio carries no placement signal — the JSON says so).
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import threading
import time
from typing import Optional, Sequence


def _pairs(spec: str) -> list[tuple[int, int]]:
    out = []
    for p in (spec or "").split(","):
        p = p.strip()
        if p:
            a, b = p.split("-")
            out.append((int(a), int(b)))
    return out


class LinkLoad:
    """Background xGMI traffic: peer-write streams over the given (src, dst) HIP ordinals
    until ``stop()``. Reports what the device said (unsupported on a 1-GPU box)."""

    def __init__(self, pairs: Sequence[tuple[int, int]], nbytes: int = 256 << 20) -> None:
        self.pairs = list(pairs)
        self.nbytes = nbytes
        self.gbps: dict[str, float] = {}
        self.supported = True
        self.error = ""
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None

    def _run(self) -> None:
        from ..ops import hip
        while not self._stop.is_set():
            for s, d in self.pairs:
                try:
                    r = hip.peer_write_bandwidth(s, d, self.nbytes, 4)
                except Exception as e:  # noqa: BLE001 - load is best effort; reported
                    self.error, self.supported = str(e)[:200], False
                    return
                if not r["supported"]:
                    self.supported = False
                    return
                self.gbps[f"{s}-{d}"] = round(r["gbps"], 1)

    def start(self) -> "LinkLoad":
        if self.pairs:
            self._t = threading.Thread(target=self._run, name="xgmi-load", daemon=True)
            self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(60)


def fake_backend(gpus: int, loads: Sequence[tuple[int, int, float]]):
    from ..sniffer.collector import FakeBackend
    be = FakeBackend(gpus=gpus, node="validate")
    for a, b, ld in loads:
        be.state[a].link_load[b] = ld
        be.state[b].link_load[a] = ld
    return be


def sample_scv(backend, settle_s: float = 0.5):
    """Two samples (link load is a counter delta between them) → the node's Scv."""
    from ..sniffer.collector import samples_to_scv
    backend.sample()
    time.sleep(settle_s)
    return samples_to_scv("validate", backend.sample(), sniffer=getattr(backend, "name", "amd-smi"))


def choose_sets(scv, k: int, memory_mb: int = 0) -> dict:
    """Best set = the native engine's placement of a k-GPU pod on this node (the scheduler's
    own path); worst = the k-subset with the largest reference objective. Card indices are
    Scv card positions; ``ranks`` maps them to HIP ordinals."""
    from ..models.pod import PodInfo
    from ..ops.native import core, link_matrix, pod_req, push_scv
    from .gang import GangWeights, GpuView, objective
    eng = core().Engine(False, 1)
    idx = eng.upsert_node("validate")
    eng.set_node_meta(idx, False, [], [], 1 << 20, 1 << 50, 110)
    push_scv(eng, idx, scv, compat=False)
    labels = {"scv/number": str(k)}
    if memory_mb:
        labels["scv/memory"] = str(memory_mb)
    pi = PodInfo.from_obj({"metadata": {"name": "gang", "uid": "validate-gang", "labels": labels}, "spec": {}})
    res = eng.schedule(pi.num_id, pod_req(eng, pi), False)
    if res[0] < 0:
        raise RuntimeError(f"no {k}-GPU set fits this node: reasons {res[5]}")
    best = sorted(res[3])
    cards = scv.status.card_list
    nphys, lq = link_matrix(scv)
    views = [GpuView(c.free_memory, c.total_memory, c.phys, c.numa_node, int(round(c.cu_occupancy * 100)))
             for c in cards]
    w = GangWeights()
    elig = [i for i, c in enumerate(cards) if c.health == "Healthy" and c.free_memory >= memory_mb]
    scored = [(objective(views, lq, nphys, s, memory_mb, w), list(s)) for s in itertools.combinations(elig, k)]
    (best_obj, best_link), spec_best = min(scored, key=lambda x: (x[0][0], x[1]))
    (worst_obj, worst_link), worst = max(scored, key=lambda x: (x[0][0], [-i for i in x[1]]))
    obj_of = {tuple(s): o for o, s in scored}
    rank = [c.hip_id if c.hip_id >= 0 else c.id for c in cards]
    # the two objectives the busbw measurement arbitrates: mean pair quality only (rounds 1-2)
    # vs mean + bottleneck pair (a ring all-reduce runs at its slowest link)
    mean_only = GangWeights(minlink=0)
    order = {name: [list(s) for _, s in sorted(((objective(views, lq, nphys, s, memory_mb, ww)[0], list(s))
                                                  for s in itertools.combinations(elig, k)))[:5]]
             for name, ww in (("mean_only", mean_only), ("mean_plus_bottleneck", w))}
    return {"best": best, "worst": worst, "best_ranks": sorted(rank[i] for i in best),
            "predicted_order_top5": order,
            "worst_ranks": sorted(rank[i] for i in worst),
            "best_objective": obj_of[tuple(best)][0], "best_link_bad": obj_of[tuple(best)][1],
            "worst_objective": worst_obj, "worst_link_bad": worst_link,
            "engine_matches_spec": best == spec_best, "gang_quality": res[6]}


def measure(sets: dict, sizes: Sequence[int], iters: int) -> dict:
    """Every rank: all-reduce over each set's ranks (subgroups); returns rank 0's view."""
    import torch.distributed as dist
    from .rccl_probe import allreduce_bandwidth
    out = {}
    for name in ("best", "worst"):
        ranks = sets[f"{name}_ranks"]
        grp = dist.new_group(ranks=ranks)
        rows = None
        if dist.get_rank() in ranks:
            rows = allreduce_bandwidth(sizes, iters=iters, group=grp)
        holder = [rows]
        dist.broadcast_object_list(holder, src=ranks[0])
        out[name] = holder[0]
        dist.barrier()
    return out


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--k", type=int, default=4, help="GPUs of the gang")
    ap.add_argument("--memory", type=int, default=0, help="scv/memory per GPU (MB)")
    ap.add_argument("--load-pairs", default="", help="xGMI links to load during the test, e.g. 0-1,2-3 (HIP ordinals)")
    ap.add_argument("--sizes", default="16M,256M")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--fake", action="store_true", help="FakeBackend telemetry instead of amd-smi (CPU rehearsal)")
    ap.add_argument("--fake-load", default="", help="a-b:load,... link loads injected into FakeBackend")
    ap.add_argument("--out", default="", help="also write rank 0's JSON here")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist
    from .rccl_probe import parse_size
    local = int(os.environ.get("LOCAL_RANK", 0))
    cuda = torch.cuda.is_available() and not a.fake
    if cuda:
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    else:
        dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    if a.k > world:
        raise SystemExit(f"--k {a.k} needs at least {a.k} ranks (one per GPU), have {world}")

    load = None
    info: dict = {}
    if rank == 0:
        if a.fake:
            loads = []
            for p in filter(None, a.fake_load.split(",")):
                ab, ld = p.split(":")
                x, y = ab.split("-")
                loads.append((int(x), int(y), float(ld)))
            backend = fake_backend(world, loads)
            info["telemetry"] = "FakeBackend"
            info["injected_link_load"] = {f"{x}-{y}": ld for x, y, ld in loads}
        else:
            from ..sniffer.collector import AmdSmiBackend
            backend = AmdSmiBackend()
            info["telemetry"] = "amd-smi (C++ collector)"
            load = LinkLoad(_pairs(a.load_pairs)).start()
            time.sleep(1.0 if load.pairs else 0.0)
        scv = sample_scv(backend)
        sets = choose_sets(scv, a.k, a.memory)
        info["sampled_link_load"] = {f"{c.id}-{l.peer}": round(l.load, 3) for c in scv.status.card_list
                                     for l in c.xgmi if l.load > 0}
    else:
        sets = None
    holder = [sets]
    dist.broadcast_object_list(holder, src=0)
    sets = holder[0]
    bw = measure(sets, [parse_size(s) for s in a.sizes.split(",")], a.iters)
    if load is not None:
        load.stop()
        info["xgmi_load"] = {"pairs": [f"{s}-{d}" for s, d in load.pairs], "supported": load.supported,
                             "peer_write_gbps": load.gbps, **({"error": load.error} if load.error else {})}
    if rank == 0:
        big_b, big_w = bw["best"][-1], bw["worst"][-1]
        out = {"k": a.k, "world": world, "backend": "nccl (RCCL over xGMI)" if cuda else "gloo (CPU rehearsal, no xGMI)",
               **sets, **info, "busbw_best": bw["best"], "busbw_worst": bw["worst"],
               "busbw_ratio_best_over_worst": round(big_b["busbw_gbps"] / big_w["busbw_gbps"], 3)
               if big_w["busbw_gbps"] else None}
        if not cuda:
            out["note"] = "CPU rehearsal: the sets are chosen from injected telemetry; gloo bandwidth says nothing about xGMI"
        line = json.dumps(out)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
