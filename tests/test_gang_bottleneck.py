"""Bottleneck xGMI term of the gang objective.

A ring all-reduce over a GPU set runs at the speed of its slowest link, so a set with one
saturated link must lose to a set whose links are all mildly loaded, even though its mean
pair quality is higher. The term is ``w_minlink × (10000 − min pair q) × 100`` on top of the
mean (engine.cpp Engine::gang_objective, scorer.hip gang search, parallel/gang.py) — Python
spec ≡ C++ engine here; the device kernel is pinned by tests/test_gpu_device_scorer.py.
"""
from yoda_scheduler_amd.models.device import make_scv
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.models.scv import XgmiLink
from yoda_scheduler_amd.ops.native import core, link_matrix, pod_req, push_scv
from yoda_scheduler_amd.parallel.gang import GangWeights, GpuView, objective, select


def _node(loads: dict):
    """An 8-GPU node, all on one NUMA node, with per-pair xGMI loads."""
    s = make_scv("n", gpus=8)
    for c in s.status.card_list:
        c.numa_node = 0
        c.xgmi = [XgmiLink(peer=p, load=loads.get((min(c.phys, p), max(c.phys, p)), 0.0)) for p in range(8)
                  if p != c.phys]
    return s


def _engine_pick(scv, k: int, minlink: int):
    eng = core().Engine(False, 1)
    idx = eng.upsert_node("n")
    eng.set_node_meta(idx, False, [], [], 1 << 20, 1 << 50, 110)
    eng.set_gang_weights(minlink=minlink)
    push_scv(eng, idx, scv, compat=False)
    pi = PodInfo.from_obj({"metadata": {"name": "g", "uid": "g", "labels": {"scv/number": str(k)}}, "spec": {}})
    ok, cards, q = eng.select_gpus(pod_req(eng, pi), idx)
    assert ok
    return sorted(cards)


def _spec_pick(scv, k: int, minlink: int):
    nphys, lq = link_matrix(scv)
    views = [GpuView(c.free_memory, c.total_memory, c.phys, c.numa_node, 0) for c in scv.status.card_list]
    ok, cards, _ = select(views, list(range(8)), k, 0, lq, nphys, GangWeights(minlink=minlink))
    assert ok
    return sorted(cards)


def test_one_hot_link_loses_to_uniformly_mild_links():
    # set A = {0,1,2,3}: five idle links and one saturated (0-1); set B = {4,5,6,7}: six links
    # at 30 % load. Every other pair (between the sets) is saturated, so only A and B compete.
    loads = {}
    for a in range(8):
        for b in range(a + 1, 8):
            loads[(a, b)] = 1.0
    for a, b in [(0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]:
        loads[(a, b)] = 0.0
    for a in range(4, 8):
        for b in range(a + 1, 8):
            loads[(a, b)] = 0.3
    scv = _node(loads)
    # the mean alone prefers A (higher average quality) ...
    assert _spec_pick(scv, 4, 0) == _engine_pick(scv, 4, 0) == [0, 1, 2, 3]
    # ... the bottleneck term moves the gang to B, whose slowest link is far faster
    assert _spec_pick(scv, 4, 2) == _engine_pick(scv, 4, 2) == [4, 5, 6, 7]
    nphys, lq = link_matrix(scv)
    views = [GpuView(c.free_memory, c.total_memory, c.phys, c.numa_node, 0) for c in scv.status.card_list]
    a_obj, a_link = objective(views, lq, nphys, [0, 1, 2, 3], 0, GangWeights())
    b_obj, b_link = objective(views, lq, nphys, [4, 5, 6, 7], 0, GangWeights())
    assert a_link < b_link and b_obj < a_obj


def test_bottleneck_term_is_neutral_on_uniform_links_and_single_gpu():
    scv = _node({})
    for k in (1, 2, 4, 8):
        assert _spec_pick(scv, k, 2) == _engine_pick(scv, k, 2) == _engine_pick(scv, k, 0)
