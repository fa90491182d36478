"""gfx950 device placement scorer — enabling it on an engine, and the smoke/parity helpers.

The native engine ``dlopen``s ``libyoda_hip.so`` itself and calls ``yoda_dev_schedule`` from
C++ inside ``Engine::schedule`` whenever the cluster has at least ``min_nodes`` nodes and
the pod is representable on the device (see ``Engine::device_eligible``), so the Python
control plane never touches the device on the hot path. Node records are mirrored
incrementally: every engine mutation marks its node dirty and dirty rows are scattered
into the device table before the next device cycle.
"""
from __future__ import annotations

import ctypes
import random

from .hip import PATH, lib as hip_lib


def declare(lib: ctypes.CDLL) -> None:
    lib.yoda_dev_last_us.argtypes = [ctypes.c_void_p]
    lib.yoda_dev_last_us.restype = ctypes.c_float
    lib.yoda_dev_batch_trace.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    lib.yoda_dev_batch_trace.restype = ctypes.c_int
    lib.yoda_dev_counters.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.yoda_dev_counters.restype = ctypes.c_int
    lib.yoda_dev_set_pairs.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.yoda_dev_set_pairs.restype = None


def set_pairs(engine, on: bool) -> None:
    """k_batch with two pods in flight (PAIRS, the default where twice the grid fits) or one
    at a time, for the next batches of ``engine``'s device scorer."""
    lib = hip_lib()
    declare(lib)
    lib.yoda_dev_set_pairs(engine.device_ctx, 1 if on else 0)


# k_batch phases (block 0's stamps): filter → record 1 out; part A of scoring (gang search,
# maxima-free terms) while record 1 travels; gather 1 (maxima); part B (normalised metrics)
# → record 2 out; gather 2 (raw lo/hi); select → record 3 out; gather 3 (winner); publish
TRACE_PHASES = ("filter", "score_a", "gather1", "score_b", "gather2", "select", "gather3", "publish")
# PAIRS, the block that owns the other set's last winner (stamps 13, 9..12): record 3 gathered →
# winner known and assumed, → record 1 sent (re-filtered group), → the group scored, → gather 1 done
OWNER_PHASES = (("own_winner", 13, 9), ("own_filter_rec1", 9, 10), ("own_score_a", 9, 11),
                ("own_gather1", 11, 12), ("own_to_gather1", 13, 12),
                # wave 1 (scoring replica 0): the group's filter verdict, then score A
                ("own_sa_filter", 9, 14), ("own_sa_score", 14, 15), ("own_sa_to_merge", 15, 11),
                # inside wave 1's score A: node tables loaded, GPU set chosen, default scores
                ("own_sa_tables", 14, 16), ("own_sa_gang", 16, 17), ("own_sa_defaults", 17, 15),
                # wave 0's early gather 1: record 1 sent → every record 1 of the set in hand
                ("own_early_g1", 10, 18),
                # the block-wide gather 1 (G > 128): records in hand, transposed, reduced
                ("own_g1_load", 11, 19), ("own_g1_transpose", 19, 20), ("own_g1_reduce", 20, 21),
                ("own_g1_barrier", 21, 12),
                # the fix-up's block barrier: the scoring wave done → every wave there → the group finished
                ("own_to_barrier", 15, 23), ("own_finish", 23, 11), ("own_w0_to_barrier", 10, 23),
                ("own_barrier_at", 9, 23))


def batch_trace(engine, on: bool = True) -> None:
    """Record block 0's phase stamps in every persistent k_batch launch (benchmarks only)."""
    lib = hip_lib()
    declare(lib)
    if lib.yoda_dev_batch_trace(engine.device_ctx, 1 if on else 0, None, 0) < 0:
        raise RuntimeError("yoda_dev_batch_trace failed")


def batch_geometry(engine) -> tuple[int, int]:
    """(grid, nodes per block) of the last k_batch launch; (0, 0) if none ran."""
    lib = hip_lib()
    declare(lib)
    v = lib.yoda_dev_batch_trace(engine.device_ctx, 1, None, 0)
    return v >> 16, v & 0xFFFF


def read_batch_trace(engine, max_pods: int = 256) -> list[dict]:
    """Per pod of the last k_batch chunk: µs spent in each phase (block 0's view)."""
    lib = hip_lib()
    declare(lib)
    W = 24
    buf = (ctypes.c_ulonglong * (max_pods * W))()
    m = lib.yoda_dev_batch_trace(engine.device_ctx, 1, buf, max_pods)
    out = []
    for b in range(max(m, 0)):
        t = [buf[b * W + k] for k in range(W)]
        d = {ph: (t[k + 1] - t[k]) / 100.0 for k, ph in enumerate(TRACE_PHASES)}
        if t[22]:   # SPEC kernels: 1 = the speculated maxima held (no record 2), 2 = record 2 exchanged
            d["spec_hit"] = 1.0 if t[22] == 1 else 0.0
        if t[13] and t[9] and t[12]:   # PAIRS: the fix-up owner's stamps (a pod with one)
            d.update({ph: (t[hi] - t[lo]) / 100.0 for ph, lo, hi in OWNER_PHASES if t[lo] and t[hi]})
        out.append(d)
    return out


COUNTERS = ("dispatches", "kbatch_dispatches", "kbatch_pods", "abandoned", "busy_refusals", "kbatch_us",
            "drain_queries", "drain_query_us", "abandon_wait_us", "presleeps", "wait_us_per_pod", "last_pairs")


def counters(engine) -> dict:
    """The device context's counters: every kernel dispatch, k_batch dispatches and the pods
    they placed, calls abandoned at the host deadline, calls refused while an abandoned one
    drained, k_batch GPU time in µs (accumulated while ``engine.device_set_timing(True)``), and
    the host's batch wait: pre-sleeps taken and the smoothed wall µs per pod they are sized by."""
    lib = hip_lib()
    declare(lib)
    buf = (ctypes.c_double * len(COUNTERS))()
    if lib.yoda_dev_counters(engine.device_ctx, buf, len(COUNTERS)) != 0:
        raise RuntimeError("yoda_dev_counters failed (device scorer not enabled?)")
    return {k: (buf[i] if k.endswith("_us") or k.endswith("_per_pod") else int(buf[i])) for i, k in enumerate(COUNTERS)}


def enable(engine, device: int = 0, capacity: int = 65536, min_nodes: int = 256) -> None:
    """Attach the device scorer to ``engine``; raises if the GPU path cannot start."""
    hip_lib()          # builds the library if needed; shares torch's HIP runtime if loaded
    ok, err = engine.enable_device(str(PATH), device, capacity, min_nodes)
    if not ok:
        raise RuntimeError(f"device scorer unavailable: {err}")


def synthetic_cluster(engine, n_nodes: int, seed: int = 0, compat: bool = False, busy: float = 0.5,
                      labels_fn=None):
    """Populate ``engine`` with ``n_nodes`` random MI355X/MI350X nodes (8 GPUs each);
    ``labels_fn(i)``: extra node labels (e.g. a zone)."""
    from ..models.device import MI350X, MI355X, make_node
    from ..models.pod import NodeInfo
    from ..models.scv import Card, Scv, ScvStatus, XgmiLink
    from .native import push_node, push_scv
    rng = random.Random(seed)
    for i in range(n_nodes):
        spec = MI355X if rng.random() < 0.75 else MI350X
        info = NodeInfo.from_obj(make_node(f"node-{i}", cpu=str(rng.choice([96, 192])),
                                           memory=rng.choice(["1Ti", "2Ti"]),
                                           labels=labels_fn(i) if labels_fn else None))
        idx = push_node(engine, info)
        cards = []
        for g in range(8):
            used = rng.randint(0, int(spec.hbm_mb * busy))
            cards.append(Card(id=g, health="Healthy" if rng.random() > 0.02 else "Unhealthy",
                              total_memory=spec.hbm_mb, free_memory=spec.hbm_mb - used, clock=spec.max_sclk_mhz,
                              bandwidth=spec.hbm_bw_gbps, core=spec.cus, power=spec.power_w, physical_id=g,
                              numa_node=int(g >= 4), cu_occupancy=rng.randint(0, 100)))
        for c in cards:
            c.xgmi = [XgmiLink(peer=d.phys, load=rng.choice([0.0, 0.0, 0.1, 0.5, 0.9])) for d in cards if d is not c]
        st = ScvStatus(card_list=cards, update_time=0.0)
        st.recompute_sums()
        push_scv(engine, idx, Scv(name=f"node-{i}", status=st), compat,
                 stale=rng.random() < 0.01)


def random_request(engine, rng: random.Random, uid: str):
    from ..models.pod import PodInfo
    from .native import pod_req
    lab = {}
    r = rng.random()
    if r < 0.5:
        lab["scv/memory"] = str(rng.choice([1024, 4096, 65536, 200000]))
    elif r < 0.8:
        lab.update({"scv/number": str(rng.choice([2, 4, 8])), "scv/memory": str(rng.choice([1024, 16384]))})
    elif r < 0.9:
        lab.update({"scv/clock": str(rng.choice([2400, 2200])), "scv/memory": "2048"})
    else:
        lab["scv/number"] = str(rng.choice([1, 3, 9]))
    pi = PodInfo.from_obj({"metadata": {"name": uid, "uid": uid, "labels": lab},
                           "spec": {"containers": [{"name": "c", "resources": {"requests": {
                               "cpu": rng.choice(["1", "8"]), "memory": "16Gi"}}}]}})
    return pi, pod_req(engine, pi)


def cloud_cluster(engine, n_nodes: int, seed: int = 0) -> None:
    """A zoned cloud pool on ``engine``: ``synthetic_cluster`` nodes with
    topology.kubernetes.io/zone (3 zones), the hot image on ~30 % of the nodes at varying sizes, a
    Service + ReplicaSet selecting app=trainer, the System default spreading, and trainer pods
    already running on a third of the nodes (so spreading is a real per-node term)."""
    from ..framework.scheduler import push_spread_source
    from ..models.pod import PodInfo
    from ..plugins.spread_affinity import PodTopologySpread
    from .native import core, pod_req
    C = core()
    engine.set_percentage_of_nodes_to_score(100)
    synthetic_cluster(engine, n_nodes, seed=seed, labels_fn=lambda i: {"topology.kubernetes.io/zone": f"zone-{i % 3}"})
    rng = random.Random(seed)
    gi = 1 << 30
    for i in range(n_nodes):
        imgs = [("registry.k8s.io/pause:3.9", 1 << 20)]
        if rng.random() < 0.3:
            imgs.append(("docker.io/rocm/vllm:v0.6.4", (600 + 250 * rng.randrange(5)) << 20))
        engine.set_node_extras(i, imgs, [("ephemeral-storage", rng.choice([2, 5, 100]) * gi)], [])
    engine.filters = engine.filters | C.F_SPREAD
    engine.set_score_weight(C.S_IMAGE_LOCALITY, 1)
    engine.set_score_weight(C.S_PREFER_AVOID, 10000)
    engine.set_score_weight(C.S_SPREAD, 2)
    engine.set_spread_defaults(PodTopologySpread({}, None).engine_defaults())
    push_spread_source(engine, "services", {"metadata": {"name": "trainer", "namespace": "default"},
                                            "spec": {"selector": {"app": "trainer"}}}, False)
    push_spread_source(engine, "replicasets", {"metadata": {"name": "trainer-rs", "namespace": "default"},
                                               "spec": {"selector": {"matchLabels": {"app": "trainer"}}}}, False)
    for k in range(n_nodes // 3):        # trainer pods already running (no GPU reservation)
        pi = PodInfo.from_obj({"metadata": {"name": f"old-{k}", "uid": f"old-{seed}-{k}", "namespace": "default",
                                            "labels": {"app": "trainer"}}, "spec": {}})
        engine.reserve(pi.num_id, pod_req(engine, pi), rng.randrange(n_nodes), [])


def cloud_pod(engine, rng: random.Random, uid: str, image: str | None = None, trainer: float = 0.3):
    """A pod for ``cloud_cluster``: ``random_request``'s GPU labels, an image (the hot one the
    nodes partly hold, or one none holds; ``image`` fixes it), sometimes ephemeral storage, and
    with probability ``trainer`` a trainer ReplicaSet pod (System default spreading applies)."""
    from ..models.pod import PodInfo
    base, _ = random_request(engine, rng, uid)
    obj = {"metadata": {"name": uid, "uid": uid, "namespace": "default", "labels": dict(base.labels)},
           "spec": {"containers": [{"name": "c", "image": image or rng.choice(["docker.io/rocm/vllm:v0.6.4", "rocm/pytorch"]),
                                    "resources": {"requests": {"cpu": "1", "memory": "16Gi"}}}]}}
    if rng.random() < 0.2:
        obj["spec"]["containers"][0]["resources"]["requests"]["ephemeral-storage"] = rng.choice(["1Gi", "3Gi"])
    if rng.random() < trainer:
        obj["metadata"]["labels"]["app"] = "trainer"
        obj["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "trainer-rs",
                                               "uid": "rs-1", "controller": True}]
    return PodInfo.from_obj(obj)


def compare_cycle(engine, req) -> dict:
    """Run one device cycle and the CPU reference on the same state; return a diff dict
    (empty = bit-exact). Ties may pick different nodes; the device's node must be one of
    the CPU's argmax set, and its GPU set must equal the CPU's choice on that node."""
    dev = engine.device_cycle(req)
    if dev is None:
        return {"skipped": True}
    feas, reasons = engine.feasible_nodes(req, [])
    diffs = {}
    if dev[1] != len(feas):
        diffs["feasible"] = (dev[1], len(feas))
    if list(dev[5]) != list(reasons):
        diffs["reasons"] = (list(dev[5]), list(reasons))
    if feas:
        if len(feas) == 1:
            best, arg = 0, {feas[0]}
        else:
            sc = engine.score_nodes(req, feas)
            best = max(sc)
            arg = {n for n, s in zip(feas, sc) if s == best}
        if dev[4] != best:
            diffs["score"] = (dev[4], best)
        if dev[0] not in arg:
            diffs["node"] = (dev[0], sorted(arg)[:5])
        ok, cards, q = engine.select_gpus(req, dev[0])
        if list(dev[3]) != list(cards) or (ok and dev[6] != q):
            diffs["cards"] = (list(dev[3]), list(cards), dev[6], q)
    elif dev[0] != -1:
        diffs["node"] = (dev[0], -1)
    return diffs


def compare_batch(dev, ref, pods, reqs_dev, reqs_ref) -> list:
    """One k_batch run on ``dev`` against a CPU replay on ``ref`` (same cluster, no device):
    for each pod in order, the device's node must be in the CPU's argmax set with the CPU's best
    score, feasible count and reason histogram, and its GPU set the CPU's choice on that node;
    the replay then reserves the device's choice, so every later pod is compared on the same
    state. Returns the diffs (empty: bit-exact up to tie-breaks) — the PodTopologySpread and
    ImageLocality score columns included."""
    res = dev.schedule_batch([p.num_id for p in pods], reqs_dev)
    diffs = []
    for k, (p, r) in enumerate(zip(pods, res)):
        req = reqs_ref[k]
        feas, reasons = ref.feasible_nodes(req, [])
        d = {}
        if r[1] != len(feas):
            d["feasible"] = (r[1], len(feas))
        if list(r[5]) != list(reasons):
            d["reasons"] = (list(r[5]), list(reasons))
        if feas:
            if len(feas) == 1:
                best, arg = 0, {feas[0]}
            else:
                sc = ref.score_nodes(req, feas)
                best = max(sc)
                arg = {n for n, s in zip(feas, sc) if s == best}
            if r[4] != best:
                d["score"] = (r[4], best)
            if r[0] not in arg:
                d["node"] = (r[0], sorted(arg)[:5])
            ok, cards, _q = ref.select_gpus(req, r[0] if r[0] >= 0 else 0)
            if r[0] >= 0 and list(r[3]) != list(cards):
                d["cards"] = (list(r[3]), list(cards))
        elif r[0] != -1:
            d["node"] = (r[0], -1)
        if d:
            diffs.append((k, d))
        if r[0] >= 0:
            ref.reserve(p.num_id, req, r[0], list(r[3]))
    return diffs


def smoke(device: int = 0, n_nodes: int = 512, pods: int = 32) -> dict:
    """Device vs CPU parity on a synthetic cluster (used by ``__graft_entry__.smoke``)."""
    from .native import core
    eng = core().Engine(False, 1)
    eng.set_percentage_of_nodes_to_score(100)
    synthetic_cluster(eng, n_nodes, seed=1)
    enable(eng, device, capacity=max(1024, n_nodes), min_nodes=1)
    rng = random.Random(7)
    bad = []
    for k in range(pods):
        pi, req = random_request(eng, rng, f"smoke-{k}")
        d = compare_cycle(eng, req)
        if d:
            bad.append(d)
        res = eng.schedule(pi.num_id, req, True)      # device path + reserve → next pod sees it
    if bad:
        raise AssertionError(f"device scorer mismatch: {bad[:3]}")
    # one persistent k_batch dispatch over a batch, then the device table must still agree
    from .native import pod_req
    batch = [random_request(eng, rng, f"smoke-b{k}")[0] for k in range(pods)]
    before = eng.device_cycles
    eng.schedule_batch([p.num_id for p in batch], [pod_req(eng, p) for p in batch])
    if eng.device_cycles - before != len(batch) or eng.device_fallbacks:
        raise AssertionError(f"k_batch did not run: {eng.device_cycles - before} cycles, {eng.device_fallbacks} fallbacks")
    pi, req = random_request(eng, rng, "smoke-after")
    d = compare_cycle(eng, req)
    if d:
        raise AssertionError(f"device table diverged after k_batch: {d}")
    return {"device_cycles": eng.device_cycles, "fallbacks": eng.device_fallbacks,
            "last_us": round(eng.device_last_us(), 1), "batch_grid_npb": batch_geometry(eng)}
