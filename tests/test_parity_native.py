"""Property tests: the native engine is bit-exact with the Python policy spec (filter,
cluster maxima, raw yoda score, normalisation, gang selection) on random MI355X-like
clusters, with and without scheduler reservations."""
import random

from hypothesis import given, settings
from hypothesis import strategies as st

from yoda_scheduler_amd.models.labels import parse_gpu_request
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.models.scv import Card, Scv, ScvStatus, XgmiLink
from yoda_scheduler_amd.ops.native import core, link_matrix, pod_req, push_scv
from yoda_scheduler_amd.parallel.gang import GangWeights, GpuView, select
from yoda_scheduler_amd.plugins import yoda_policy as P

CLOCKS = [2100, 2200, 2400]


def rand_cluster(rng: random.Random, n_nodes: int) -> list[Scv]:
    out = []
    for n in range(n_nodes):
        g = rng.choice([0, 1, 2, 4, 8])
        cards = []
        for i in range(g):
            total = rng.choice([294912, 147456, 1000])
            cards.append(Card(id=i, health="Healthy" if rng.random() > 0.1 else "Unhealthy",
                              total_memory=total, free_memory=rng.randint(0, total),
                              clock=rng.choice(CLOCKS), bandwidth=rng.choice([8000, 6000]),
                              core=rng.choice([256, 128]), power=rng.choice([1400, 1000]),
                              physical_id=i, numa_node=int(i >= g // 2), cu_occupancy=rng.randint(0, 100)))
        for c in cards:
            c.xgmi = [XgmiLink(peer=d.phys, load=rng.choice([0.0, 0.25, 0.5, 0.9])) for d in cards if d is not c]
        st_ = ScvStatus(card_list=cards)
        st_.recompute_sums()
        if rng.random() < 0.1:
            st_.free_memory_sum = rng.randint(0, 10**6)   # sums need not agree with the list
        out.append(Scv(name=f"n{n}", status=st_))
    return out


def rand_labels(rng: random.Random) -> dict:
    lab = {}
    if rng.random() < 0.7:
        lab["scv/memory"] = str(rng.choice([0, 100, 1000, 5000, 100000, 200000, 300000]))
    if rng.random() < 0.5:
        lab["scv/number"] = str(rng.choice([0, 1, 2, 3, 4, 8, 9]))
    if rng.random() < 0.3:
        lab["scv/clock"] = str(rng.choice(CLOCKS))
    if rng.random() < 0.05:
        lab["scv/number"] = rng.choice(["-1", "abc", ""])
    return lab


def build(scvs, compat, reserved=None):
    e = core().Engine(compat, 1)
    for i, s in enumerate(scvs):
        idx = e.upsert_node(s.name)
        e.set_node_meta(idx, False, [], [], 10**6, 10**15, 10**6)
        push_scv(e, idx, s, compat)
    views = []
    for i, s in enumerate(scvs):
        res = (reserved or {}).get(i, [0] * len(s.status.card_list))
        st_ = s.status
        views.append(P.NodeView(s.name, st_.card_list, st_.card_number, st_.free_memory_sum, st_.total_memory_sum,
                                reserved_mb=res if not compat else ()))
    return e, views


@settings(max_examples=150, deadline=None)
@given(seed=st.integers(0, 2**32 - 1), compat=st.booleans())
def test_policy_parity(seed, compat):
    rng = random.Random(seed)
    scvs = rand_cluster(rng, rng.randint(1, 5))
    e, views = build(scvs, compat)
    # optionally put reservations on the native ledger and mirror them in the views
    if not compat:
        for k in range(rng.randint(0, 6)):
            ni = rng.randrange(len(scvs))
            ncards = len(scvs[ni].status.card_list)
            if not ncards:
                continue
            cards = sorted(rng.sample(range(ncards), rng.randint(1, ncards)))
            mb = rng.choice([0, 1000, 50000])
            pi = PodInfo.from_obj({"metadata": {"name": f"r{k}", "uid": f"res-{seed}-{k}",
                                                "labels": {"scv/memory": str(mb)}}, "spec": {}})
            assert e.reserve(pi.num_id, pod_req(e, pi), ni, cards)
            rv = list(views[ni].reserved_mb) or [0] * ncards
            for c in cards:
                rv[c] += mb
            views[ni].reserved_mb = rv
            views[ni].pending_mb = rv      # sample time 0: nothing reserved is in the sample yet
    for _ in range(4):
        lab = rand_labels(rng)
        req = parse_gpu_request(lab)
        pi = PodInfo.from_obj({"metadata": {"name": "q", "uid": f"q{seed}", "labels": lab}, "spec": {}})
        r = pod_req(e, pi)
        feas_py = [i for i, v in enumerate(views) if P.filter_node(req, v, compat)[0]]
        feas_nat = [i for i in range(len(views)) if e.filter_node(r, i) == 0]
        assert feas_py == feas_nat, lab
        scope = list(range(len(views))) if compat else feas_nat
        mv = P.collect_max(req, [views[i] for i in scope], compat)
        mx = e.collect_max(r, scope)
        assert mx == (mv.bandwidth, mv.clock, mv.core, mv.free_memory, mv.power, mv.total_memory)
        for i in feas_nat:
            want = P.calculate_score(mv, req, views[i], compat)
            if not compat:
                nphys, q = link_matrix(scvs[i])
                want_u = want + P.gang_bonus(req, views[i], q, nphys)
                want = want_u if want_u <= 2**63 - 1 else 0
            assert e.yoda_raw_score(r, i, mx) == want, (lab, i)


@settings(max_examples=200, deadline=None)
@given(seed=st.integers(0, 2**32 - 1), binpack=st.booleans())
def test_gang_selection_parity(seed, binpack):
    rng = random.Random(seed)
    g = rng.choice([2, 4, 8, 16])
    cards = [Card(id=i, total_memory=294912, free_memory=rng.randint(0, 294912), clock=2400,
                  physical_id=i % 8, numa_node=int((i % 8) >= 4), cu_occupancy=rng.randint(0, 100))
             for i in range(g)]
    for c in cards:
        c.xgmi = [XgmiLink(peer=p, load=rng.random()) for p in range(8) if p != c.phys and p < min(g, 8)]
    s = Scv(name="g", status=ScvStatus(card_list=cards))
    s.status.recompute_sums()
    k = rng.randint(1, g)
    m = rng.choice([0, 1000, 100000])
    w = GangWeights(binpack=binpack, enum_limit=rng.choice([5000, 10]))
    e, _ = build([s], False)
    e.set_gang_weights(link=w.link, numa=w.numa, fit=w.fit, occ=w.occ, binpack=binpack, gang_score=w.gang_score,
                       enum_limit=w.enum_limit)
    pi = PodInfo.from_obj({"metadata": {"name": "g", "uid": f"g{seed}",
                                        "labels": {"scv/number": str(k), "scv/memory": str(m)}}, "spec": {}})
    ok_n, sel_n, q_n = e.select_gpus(pod_req(e, pi), 0)
    nphys, lq = link_matrix(s)
    views = [GpuView(c.free_memory, c.total_memory, c.phys, c.numa_node, int(round(c.cu_occupancy * 100)))
             for c in cards]
    elig = [i for i, c in enumerate(cards) if c.free_memory >= m]
    ok_p, sel_p, q_p = select(views, elig, k, m, lq, nphys, w)
    assert (ok_n, list(sel_n), q_n) == (ok_p, sel_p, q_p)


def test_pending_reservations_vs_samples():
    """A reservation is subtracted from the sniffed free HBM until a sample taken
    ``settle`` seconds later is expected to contain its usage; never both."""
    s = Scv(name="n", status=ScvStatus(card_list=[Card(id=0, total_memory=100_000, free_memory=100_000, clock=2400)]))
    s.status.recompute_sums()
    s.status.update_time = 100.0
    e, _ = build([s], False)
    push_scv(e, 0, s, False)
    e.settle_seconds = 30.0
    e.set_fixed_now(120.0)
    pi = PodInfo.from_obj({"metadata": {"name": "a", "uid": "pend-a", "labels": {"scv/memory": "40000"}}, "spec": {}})
    assert e.reserve(pi.num_id, pod_req(e, pi), 0, [0])
    (total, free, reserved, pods, _c, _h, _p, pending), = e.node_cards(0)
    assert (reserved, pending) == (40_000, 40_000)
    # a sample at t=130 is still within the settle window of the t=120 reservation
    s.status.update_time = 130.0
    s.status.card_list[0].free_memory = 60_000       # the pod already allocated
    push_scv(e, 0, s, False)
    assert e.node_cards(0)[0][7] == 40_000            # conservative: still pending
    # a sample at t=200 is trusted to contain it
    s.status.update_time = 200.0
    push_scv(e, 0, s, False)
    assert e.node_cards(0)[0][7] == 0
    big = PodInfo.from_obj({"metadata": {"name": "b", "uid": "pend-b", "labels": {"scv/memory": "60000"}},
                            "spec": {}})
    assert e.filter_node(pod_req(e, big), 0) == 0      # 60 000 sampled free, 60 000 unreserved
    assert e.release(pi.num_id)
    assert e.node_cards(0)[0][2] == 0 and e.node_cards(0)[0][7] == 0


def test_ledger_reserve_release_roundtrip():
    rng = random.Random(1)
    scvs = rand_cluster(rng, 1)
    while not scvs[0].status.card_list:
        scvs = rand_cluster(rng, 1)
    e, _ = build(scvs, False)
    before = e.node_cards(0)
    pis = []
    for k in range(20):
        pi = PodInfo.from_obj({"metadata": {"name": f"x{k}", "uid": f"ledger-{k}",
                                            "labels": {"scv/memory": "10"}}, "spec": {}})
        res = e.schedule(pi.num_id, pod_req(e, pi), True)
        if res[0] >= 0:
            pis.append(pi)
    assert e.ledger_size == len(pis)
    for pi in pis:
        assert e.release(pi.num_id)
    assert e.node_cards(0) == before and e.ledger_size == 0


def test_nonzero_requests_feed_allocation_scores():
    """upstream NonZeroRequested: an absent cpu/memory request counts as 100m / 200 MiB
    per container for Least/Most/Balanced scoring (an explicit 0 stays 0), while the
    resource fit uses the plain requests."""
    from yoda_scheduler_amd.models.pod import PodInfo, _requests
    mi = 1024 * 1024
    assert _requests({"containers": [{}, {}]}) == (0, 0, 200, 400 * mi)
    assert _requests({"containers": [{"resources": {"requests": {"cpu": "0", "memory": "1Gi"}}}]}) == \
        (0, 1024 * mi, 0, 1024 * mi)
    assert _requests({"containers": [{}], "initContainers": [{"resources": {"requests": {"cpu": "2"}}}]}) == \
        (2000, 0, 2000, 200 * mi)
    assert _requests({"containers": [{}], "overhead": {"cpu": "50m"}}) == (50, 0, 150, 200 * mi)
    c = core()
    eng = c.Engine(False, 1)
    for name in ("busy", "idle"):
        idx = eng.upsert_node(name)
        eng.set_node_meta(idx, False, [], [], 4000, 8 << 30, 110)
    eng.filters = 0
    for i in range(6):
        eng.set_score_weight(i, 0)
    eng.set_score_weight(c.S_LEAST_ALLOCATED, 1)
    plain = PodInfo.from_obj({"metadata": {"name": "p", "uid": "u-p"}, "spec": {"containers": [{}]}})
    assert (plain.cpu_m, plain.mem, plain.nz_cpu_m, plain.nz_mem) == (0, 0, 100, 200 * mi)
    busy = eng.node_index("busy")
    for i in range(10):      # ten request-less pods: 1000m / 2000 MiB non-zero on "busy"
        pi = PodInfo.from_obj({"metadata": {"name": f"b{i}", "uid": f"u-b{i}"}, "spec": {"containers": [{}]}})
        assert eng.reserve(pi.num_id, pod_req(eng, pi), busy, [])
    assert eng.node_usage(busy)[:2] == (0, 0) and eng.node_usage(busy)[4:6] == (1000, 2000 * mi)
    s = eng.score_nodes(pod_req(eng, plain), [busy, eng.node_index("idle")])
    # busy: cpu (4000−1100)/4000 → 72, mem (8192−2200)/8192 → 73 → 72; idle: 97, 97 → 97
    assert s == [72, 97]
