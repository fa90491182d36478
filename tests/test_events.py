"""Scheduler events through events.k8s.io/v1 (upstream v1.20 EventBroadcasterAdapter) and
the core/v1 fallback: reportingController = profile name, action Binding / Scheduling /
Preempting, series on repeats, the preemptor as ``related``."""
import asyncio

from yoda_scheduler_amd.testing import FakeCluster, yoda_config


def run(c):
    return asyncio.run(c)


def _events(c, res):
    return [o for o in c.server._objs[res].values()]


def test_events_v1_binding_scheduling_series():
    async def go():
        c = FakeCluster(yoda_config(backoff=0.01, max_backoff=0.02))
        c.add_node("n", gpus=1)
        await c.start()
        c.add_pod("ok", {"scv/memory": "1000"})
        c.add_pod("big", {"scv/memory": "999999"})          # never fits: retried → series
        await c.wait_bound(1)
        await c.wait(lambda: c.sched.recorder.recorded["FailedScheduling"] >= 1, 5)
        await asyncio.sleep(0.05)
        c.server.patch("nodes", "n", {"metadata": {"labels": {"tick": "1"}}})   # NodeUpdate: retry "big"
        await c.wait(lambda: any((e.get("series") or {}).get("count", 1) >= 2
                                 for e in _events(c, "events.k8s.io")), 5)
        evs = _events(c, "events.k8s.io")
        core = _events(c, "events")
        await c.stop()
        return evs, core
    evs, core = run(go())
    assert core == []
    by_reason = {e["reason"]: e for e in evs}
    s = by_reason["Scheduled"]
    assert s["apiVersion"] == "events.k8s.io/v1" and s["action"] == "Binding" and s["type"] == "Normal"
    assert s["reportingController"] == "yoda-scheduler" and s["reportingInstance"].startswith("yoda-scheduler-")
    assert s["regarding"]["name"] == "ok" and s["regarding"]["kind"] == "Pod" and "to n" in s["note"]
    assert s["eventTime"].endswith("Z") and "." in s["eventTime"]
    f = by_reason["FailedScheduling"]
    assert f["action"] == "Scheduling" and f["type"] == "Warning" and f["series"]["count"] >= 2
    assert len([e for e in evs if e["reason"] == "FailedScheduling"]) == 1      # aggregated, not duplicated


def test_events_core_v1_fallback_and_preempted_related():
    async def go():
        cfg = yoda_config()
        cfg["yodaRuntime"]["eventsAPI"] = "v1"
        c = FakeCluster(cfg)
        c.add_node("n", gpus=1, used_mb=[294912 - 10000])
        await c.start()
        c.add_pod("low", {"scv/memory": "8000"}, priority=1)
        await c.wait_bound(1)
        await c.wait(lambda: _events(c, "events"), 5)
        core = _events(c, "events")
        await c.stop()

        c2 = FakeCluster()
        c2.add_node("n", gpus=1, used_mb=[294912 - 10000])
        await c2.start()
        c2.add_pod("low", {"scv/memory": "8000"}, priority=1)
        await c2.wait_bound(1)
        c2.add_pod("high", {"scv/memory": "8000"}, priority=100)
        await c2.wait(lambda: any(e["reason"] == "Preempted" for e in _events(c2, "events.k8s.io")), 5)
        evs = _events(c2, "events.k8s.io")
        await c2.stop()
        return core, evs
    core, evs = run(go())
    sched = [e for e in core if e["reason"] == "Scheduled"][0]
    assert sched["apiVersion"] == "v1" and sched["source"]["component"] == "yoda-scheduler"
    assert sched["involvedObject"]["name"] == "low" and sched["count"] == 1
    pre = [e for e in evs if e["reason"] == "Preempted"][0]
    assert pre["action"] == "Preempting" and pre["regarding"]["name"] == "low"
    assert pre["related"]["name"] == "high" and pre["related"]["kind"] == "Pod"


def test_micro_time_matches_datetime():
    import random
    from datetime import datetime, timezone
    from yoda_scheduler_amd.framework.events import micro_time
    rng = random.Random(1)
    for _ in range(20000):
        ts = rng.uniform(0, 2e9)
        assert micro_time(ts) == datetime.fromtimestamp(ts, timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")
