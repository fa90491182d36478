"""Native DefaultPreemption (``Engine::preempt``) ≡ its Python spec (``plugins.defaults.preempt_spec``)
on random clusters with priorities, PodDisruptionBudgets, unschedulable / tainted / Scv-less
nodes, and candidate caps. Both follow upstream v1.20: potential nodes are
the ones whose first failing filter is not UnschedulableAndUnresolvable, at most
max(pct % of them, abs) candidates are dry-run from an offset, victims are reprieved PDB-violating
first and then by importance, and candidates are ranked by pickOneNodeForPreemption's keys.
"""
import time

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from yoda_scheduler_amd.framework.cache import SchedulerCache
from yoda_scheduler_amd.models.device import make_node, make_scv
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.models.selectors import LabelSelector
from yoda_scheduler_amd.ops.native import core, pod_req
from yoda_scheduler_amd.plugins.defaults import preempt_spec

C = core()
CARD_MB = 294912
_uid = iter(range(10 ** 9))


def _cluster(nodes, placed):
    eng = C.Engine(False, 1)
    cache = SchedulerCache(eng)
    for name, gpus, kind in nodes:
        taints = [{"key": "dedicated", "value": "x", "effect": "NoSchedule"}] if kind == "tainted" else None
        cache.add_node(make_node(name, unschedulable=kind == "cordoned", taints=taints))
        if kind != "noscv":
            cache.set_scv(make_scv(name, gpus=gpus))
    for node, prio, mb, cards, app in placed:
        cache.add_pod({"metadata": {"name": f"v{next(_uid)}", "namespace": "default", "uid": f"pv-{next(_uid)}",
                                    "labels": {"app": app, "scv/memory": str(mb)},
                                    "annotations": {"scv.amd.com/gpus": ",".join(map(str, cards)),
                                                    "scv.amd.com/reserved-mb": str(mb)}},
                       "spec": {"nodeName": node, "priority": prio,
                                "containers": [{"name": "c", "resources": {"requests": {"cpu": "1"}}}]}})
        time.sleep(0.0002)          # distinct reservation times (MoreImportantPod's start-time key)
    return eng, cache


@st.composite
def _cases(draw):
    n = draw(st.integers(1, 6))
    nodes = [(f"n{i}", draw(st.integers(1, 4)),
              draw(st.sampled_from(["ok", "ok", "ok", "cordoned", "tainted", "noscv"]))) for i in range(n)]
    placed = []
    for name, gpus, _kind in nodes:
        used = [0] * gpus
        for _ in range(draw(st.integers(0, 5))):
            mb = draw(st.sampled_from([60000, 100000, 140000]))
            k = draw(st.integers(1, min(2, gpus)))
            free = [c for c in range(gpus) if used[c] + mb <= CARD_MB]
            if len(free) < k:
                continue
            cards = free[:k]
            for c in cards:
                used[c] += mb
            placed.append((name, draw(st.integers(-3, 8)), mb, cards, draw(st.sampled_from(["a", "b", "c"]))))
    pdbs = [(draw(st.sampled_from([{"matchLabels": {"app": "a"}}, {"matchLabels": {"app": "b"}}, {}, None])),
             draw(st.integers(0, 2))) for _ in range(draw(st.integers(0, 2)))]
    pod = (draw(st.integers(0, 10)), draw(st.sampled_from([150000, 200000, 294912])), draw(st.integers(1, 2)))
    return nodes, placed, pdbs, pod, draw(st.sampled_from([(10, 100), (0, 1), (50, 2)])), draw(st.integers(0, 9))


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_cases())
def test_native_preemption_equals_python_spec(case):
    nodes, placed, pdb_specs, (prio, mb, number), (pct, absolute), offset = case
    eng, cache = _cluster(nodes, placed)
    pod = PodInfo.from_obj({"metadata": {"name": "hi", "namespace": "default", "uid": f"hi-{next(_uid)}",
                                         "labels": {"scv/memory": str(mb), "scv/number": str(number)}},
                            "spec": {"priority": prio, "containers": [{"name": "c"}]}})
    req = pod_req(eng, pod)
    pdbs = [("default", LabelSelector(sel), allowed) for sel, allowed in pdb_specs]
    before = {n: cache.node_gpu_state(n) for n, _g, _k in nodes}
    node_idx, ids, cards, _viol, _pot, _ev, _c = eng.preempt(
        req, prio, [(ns, sel.native(), a) for ns, sel, a in pdbs], pct, absolute, offset)
    assert {n: cache.node_gpu_state(n) for n, _g, _k in nodes} == before     # ledger restored
    spec = preempt_spec(eng, cache, pod, req, pdbs, pct, absolute, offset)
    assert {n: cache.node_gpu_state(n) for n, _g, _k in nodes} == before
    if spec is None:
        assert node_idx < 0
        return
    node, victims, spec_cards = spec
    assert eng.node_name(node_idx) == node
    assert sorted(ids) == sorted(v.info.num_id for v in victims)
    assert list(cards) == list(spec_cards)


def test_candidate_cap_and_unresolvable_nodes_are_skipped():
    """300 nodes where a preemptor fits after one eviction each, plus 100 cordoned ones: the
    cordoned nodes are not potential nodes, and with minCandidateNodesAbsolute 100 the search
    stops after 100 dry runs (upstream calculateNumCandidates: max(10 % of 300, 100))."""
    nodes = [(f"n{i}", 1, "ok") for i in range(300)] + [(f"c{i}", 1, "cordoned") for i in range(100)]
    placed = [(f"n{i}", 1, 200000, [0], "a") for i in range(300)]
    eng, cache = _cluster(nodes, placed)
    pod = PodInfo.from_obj({"metadata": {"name": "hi", "namespace": "default", "uid": "hi-cap",
                                         "labels": {"scv/memory": "200000"}},
                            "spec": {"priority": 5, "containers": [{"name": "c"}]}})
    node_idx, ids, _cards, _v, potential, evaluated, cands = eng.preempt(pod_req(eng, pod), 5, [], 10, 100, 17)
    assert potential == 300 and evaluated == 100 and cands == 100
    assert node_idx >= 0 and len(ids) == 1


def test_preemption_cost_at_4096_nodes():
    """an attempt at 4096 nodes × 8 low-priority single-GPU pods costs ≤ 5 ms
    in this container (the Python what-if over every node took ~120 ms)."""
    nodes = [(f"n{i}", 8, "ok") for i in range(4096)]
    placed = [(f"n{i}", 1, CARD_MB, [g], "a") for i in range(4096) for g in range(8)]
    eng, cache = _cluster_fast(nodes, placed)
    pod = PodInfo.from_obj({"metadata": {"name": "hi", "namespace": "default", "uid": "hi-big",
                                         "labels": {"scv/memory": str(CARD_MB), "scv/number": "8"}},
                            "spec": {"priority": 10, "containers": [{"name": "c"}]}})
    req = pod_req(eng, pod)
    best = None
    for _ in range(5):
        t = time.perf_counter()
        node_idx, ids, _c, _v, potential, evaluated, _n = eng.preempt(req, 10, [], 10, 100, -1)
        best = min(best or 1e9, time.perf_counter() - t)
    assert node_idx >= 0 and len(ids) == 8 and potential == 4096 and evaluated == 409
    assert best < 0.005, f"{best * 1e3:.2f} ms per attempt"


def _cluster_fast(nodes, placed):
    """As ``_cluster`` without the per-pod sleep (reservation times are not compared here)."""
    eng = C.Engine(False, 1)
    cache = SchedulerCache(eng)
    for name, gpus, _kind in nodes:
        cache.add_node(make_node(name))
        cache.set_scv(make_scv(name, gpus=gpus))
    for k, (node, prio, mb, cards, app) in enumerate(placed):
        cache.add_pod({"metadata": {"name": f"f{k}", "namespace": "default", "uid": f"pf-{k}",
                                    "labels": {"app": app, "scv/memory": str(mb)},
                                    "annotations": {"scv.amd.com/gpus": ",".join(map(str, cards)),
                                                    "scv.amd.com/reserved-mb": str(mb)}},
                       "spec": {"nodeName": node, "priority": prio,
                                "containers": [{"name": "c", "resources": {"requests": {"cpu": "1"}}}]}})
    return eng, cache
