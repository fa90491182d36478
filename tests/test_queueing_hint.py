"""Scv queueing hint (yodaRuntime.scvQueueingHint): telemetry updates requeue parked pods
only when the node's filter-visible GPU capacity grew — verdict r1 'change-driven
telemetry plus event-aware requeue'. A load-only update (less free HBM, link load, CU
busy) leaves the parked pods alone; freed HBM, a recovered card or a changed clock moves
them back at once (not after the unschedulable-queue flush timer)."""
import asyncio
import time

from yoda_scheduler_amd.models.device import make_scv
from yoda_scheduler_amd.models.scv import Scv
from yoda_scheduler_amd.testing import FakeCluster, yoda_config


def run(coro):
    return asyncio.run(coro)


def _publish(c: FakeCluster, node: str, used_mb: list, health: str = "Healthy", clock: int | None = None) -> None:
    s = make_scv(node, update_time=time.time(), used_mb=used_mb)
    for card in s.status.card_list:
        card.health = health if card.id == 0 else card.health
        if clock is not None:
            card.clock = clock
    s.status.recompute_sums()
    obj = s.to_json()
    obj["metadata"]["resourceVersion"] = c.server.get("scvs", node)["metadata"]["resourceVersion"]
    c.server.update("scvs", obj, status_only=True)


async def _parked(c: FakeCluster, sched, name: str, labels: dict) -> None:
    c.add_pod(name, labels)
    assert await c.wait(lambda: any(p.name == name for p, _ in sched.queue._unsched.values()), 3.0), "pod not parked"


def _attempts(sched, name: str) -> int:
    return next(p.attempts for p, _ in sched.queue._unsched.values() if p.name == name)


def test_load_only_scv_updates_do_not_requeue_parked_pods():
    async def go():
        cfg = yoda_config(backoff=0.01, max_backoff=0.02)
        c = FakeCluster(cfg)
        c.add_node("n0", used_mb=[200_000] * 8)           # ~94 GB free per card
        sched = await c.start()
        await _parked(c, sched, "big", {"scv/memory": "150000"})
        a0 = _attempts(sched, "big")
        for k in range(20):                                # tenants grow: capacity only shrinks
            _publish(c, "n0", [200_000 + 100 * k] * 8)
            await asyncio.sleep(0.005)
        await asyncio.sleep(0.1)
        skips, moves = sched.scv_requeue_skips, sched.scv_requeues
        attempts = _attempts(sched, "big")
        await c.stop()
        return a0, attempts, skips, moves
    a0, attempts, skips, moves = run(go())
    assert skips == 20 and moves == 0
    assert attempts == a0          # no retry of the parked pod


def test_freed_hbm_requeues_and_binds_immediately():
    async def go():
        cfg = yoda_config(backoff=0.01, max_backoff=0.02)
        c = FakeCluster(cfg)
        c.add_node("n0", used_mb=[200_000] * 8)
        sched = await c.start()
        await _parked(c, sched, "big", {"scv/memory": "150000"})
        t0 = time.monotonic()
        _publish(c, "n0", [200_000] * 7 + [10_000])         # one card frees up
        ok = await c.wait_bound(1, 3.0)
        dt = time.monotonic() - t0
        node, moves = c.node_of("big"), sched.scv_requeues
        await c.stop()
        return ok, dt, node, moves
    ok, dt, node, moves = run(go())
    assert ok and node == "n0" and moves == 1
    assert dt < 1.0               # the flush timer (60 s) was not needed


def test_recovered_card_and_clock_change_requeue():
    async def go():
        cfg = yoda_config(backoff=0.01, max_backoff=0.02)
        c = FakeCluster(cfg)
        c.add_node("n0")
        _publish(c, "n0", [0] * 8, health="Unhealthy")
        sched = await c.start()
        await _parked(c, sched, "all8", {"scv/number": "8"})          # card 0 unhealthy → 7 fit
        await _parked(c, sched, "clk", {"scv/clock": "2000"})         # no card at 2000 MHz
        m0 = sched.scv_requeues
        _publish(c, "n0", [0] * 8, health="Healthy")                  # card 0 recovers
        ok8 = await c.wait(lambda: c.node_of("all8") == "n0", 3.0)
        m1 = sched.scv_requeues
        _publish(c, "n0", [0] * 8, clock=2000)                        # clock pinned to 2000
        okc = await c.wait(lambda: c.node_of("clk") == "n0", 3.0)
        m2 = sched.scv_requeues
        await c.stop()
        return ok8, okc, m1 - m0, m2 - m1
    ok8, okc, d1, d2 = run(go())
    assert ok8 and okc and d1 == 1 and d2 == 1


def test_hint_disabled_requeues_on_every_update():
    async def go():
        cfg = yoda_config(backoff=0.01, max_backoff=0.02)
        cfg["yodaRuntime"]["scvQueueingHint"] = False
        c = FakeCluster(cfg)
        c.add_node("n0", used_mb=[200_000] * 8)
        sched = await c.start()
        await _parked(c, sched, "big", {"scv/memory": "150000"})
        for k in range(5):
            _publish(c, "n0", [200_000 + 100 * k] * 8)
            await asyncio.sleep(0.02)
        await asyncio.sleep(0.1)
        moves, skips = sched.scv_requeues, sched.scv_requeue_skips
        await c.stop()
        return moves, skips
    moves, skips = run(go())
    assert moves == 5 and skips == 0


def test_capacity_grew_rules():
    from yoda_scheduler_amd.framework.scheduler import Scheduler
    base = (False, 8, ((True, 100, 90, 2400),) * 2)
    g = Scheduler._capacity_grew
    assert not g(base, base)
    assert not g(base, (False, 8, ((True, 90, 80, 2400),) * 2))      # less free
    assert g(base, (False, 8, ((True, 100, 95, 2400), (True, 100, 90, 2400))))   # effective free up
    assert g(base, (False, 8, ((True, 100, 90, 2200), (True, 100, 90, 2400))))   # clock changed
    assert g((True,) + base[1:], base)                                 # stale → fresh
    assert g(base, (False, 9, base[2]))                                # CardNumber up
    assert g((False, 8, ((False, 100, 90, 2400),) * 2), base)          # card healthy again
    assert Scv is not None


def test_hint_moves_only_pods_the_new_capacity_fits():
    """Per-pod hint: capacity grows on the node (one card frees 40 GB) — the parked pod
    asking 60 GB per card for 1 card is moved back and binds; the one asking 150 GB stays
    parked (its attempt count does not move)."""
    async def go():
        cfg = yoda_config(backoff=0.01, max_backoff=0.02)
        c = FakeCluster(cfg)
        c.add_node("n0", used_mb=[250_000] * 8)            # ~44 GB free per card
        sched = await c.start()
        await _parked(c, sched, "mid", {"scv/memory": "60000"})
        await _parked(c, sched, "big", {"scv/memory": "150000"})
        a_big = _attempts(sched, "big")
        _publish(c, "n0", [250_000] * 7 + [210_000])        # card 7: ~84 GB free
        ok = await c.wait(lambda: c.node_of("mid") == "n0", 3.0)
        await asyncio.sleep(0.05)
        still = [p.name for p, _ in sched.queue._unsched.values()]
        a_big2 = _attempts(sched, "big")
        await c.stop()
        return ok, still, a_big, a_big2
    ok, still, a0, a1 = run(go())
    assert ok and still == ["big"] and a0 == a1


def test_gpu_fits_rules():
    from yoda_scheduler_amd.framework.scheduler import Scheduler
    from yoda_scheduler_amd.models.pod import PodInfo

    def pod(lab):
        return PodInfo.from_obj({"metadata": {"name": "p", "uid": f"u{sorted(lab.items())}", "labels": lab}, "spec": {}})
    cap = (False, 2, ((True, 100, 80, 2400), (True, 100, 40, 2200)))
    f = Scheduler._gpu_fits
    assert f(pod({"scv/memory": "80"}), cap, False)
    assert not f(pod({"scv/memory": "90"}), cap, False)
    assert f(pod({"scv/memory": "90"}), cap, True)               # compat: sampled free, no ledger
    assert f(pod({"scv/number": "2", "scv/memory": "40"}), cap, False)
    assert not f(pod({"scv/number": "3"}), cap, False)            # > CardNumber
    assert f(pod({"scv/clock": "2200"}), cap, False)
    assert not f(pod({"scv/clock": "2300"}), cap, False)
    assert not f(pod({}), (True,) + cap[1:], False)                # stale
    assert not f(pod({}), (False, 0, ()), False)                   # no cards


def test_hint_reads_the_engines_filter_inputs():
    """the hint's capacity view is the engine's own filter input
    (`Engine::filter_view`, next to `yoda_filter`), not a Python-side copy: it follows the
    engine's reservations (effective free HBM), CardNumber and staleness, and a node the
    engine does not know has none."""
    async def go():
        c = FakeCluster(yoda_config())
        c.add_node("n0", used_mb=[0] * 8)
        sched = await c.start()
        cap = sched._capacity("n0")
        idx = sched.engine.node_index("n0")
        has_scv, stale, cn, cards = sched.engine.filter_view(idx)
        assert cap == (bool(stale or not has_scv), cn, tuple(tuple(x) for x in cards))
        assert cap[0] is False and cap[1] == 8 and len(cap[2]) == 8
        c.add_pod("p", {"scv/memory": "100000", "scv/number": "2"})
        assert await c.wait_bound(1, 5.0)
        after = sched._capacity("n0")
        # the reservation lowered two cards' effective free HBM; sampled free is unchanged
        lowered = [i for i in range(8) if after[2][i][2] < cap[2][i][2]]
        assert len(lowered) == 2 and all(after[2][i][1] == cap[2][i][1] for i in range(8))
        assert sched._capacity("nope") is None
        await c.stop()
    run(go())
