"""Coscheduling: all-or-nothing placement of a pod group through Permit WAIT (waiting
pods held assumed, released together, rejected together on timeout)."""
import asyncio

from yoda_scheduler_amd.testing import FakeCluster, yoda_config

G = "pod-group.scheduling.sigs.k8s.io"


def run(c):
    return asyncio.run(c)


def cfg(timeout=0.5):
    c = yoda_config(backoff=0.05, max_backoff=0.1)
    plugins = c["profiles"][0]["plugins"]
    for point in ("preFilter", "permit", "reserve"):
        plugins[point] = {"enabled": [{"name": "Coscheduling"}]}
    c["profiles"][0]["pluginConfig"].append({"name": "Coscheduling", "args": {"permitWaitingTimeSeconds": timeout}})
    c["yodaRuntime"]["unschedulableFlushSeconds"] = 0.3
    return c


def member(c, name, group, n, mem="200000"):
    c.add_pod(name, {"scv/memory": mem, "scv/number": "1", G: group, f"{G}/min-available": str(n)})


def test_group_waits_for_all_members_then_binds_together():
    async def go():
        c = FakeCluster(cfg(timeout=5))
        for i in range(3):
            c.add_node(f"n{i}", gpus=1)
        await c.start()
        member(c, "w0", "job", 3)
        member(c, "w1", "job", 3)
        await asyncio.sleep(0.3)
        early = len(c.server.bind_log)                # too few members exist: nothing binds
        plain_native = c.sched.frameworks["yoda-scheduler"].native_for(
            __import__("yoda_scheduler_amd.models.pod", fromlist=["PodInfo"]).PodInfo.from_obj(
                {"metadata": {"name": "x", "uid": "x", "labels": {"scv/memory": "1"}}, "spec": {}}))
        member(c, "w2", "job", 3)
        ok = await c.wait_bound(3, 5)
        nodes = sorted(c.node_of(f"w{i}") for i in range(3))
        await c.stop()
        return early, ok, nodes, plain_native
    early, ok, nodes, plain_native = run(go())
    assert early == 0 and ok and nodes == ["n0", "n1", "n2"]
    assert plain_native                                # pods outside groups keep the native cycle


def test_partial_group_times_out_releases_gpus_and_retries():
    async def go():
        c = FakeCluster(cfg(timeout=0.4))
        for i in range(2):                             # room for 2 of the 3 members (200 GB each)
            c.add_node(f"n{i}", gpus=1)
        await c.start()
        for i in range(3):
            member(c, f"w{i}", "job", 3)
        await asyncio.sleep(1.2)
        partial = len(c.server.bind_log)
        held = [g["reserved"] for n in ("n0", "n1") for g in c.sched.cache.node_gpu_state(n)]
        c.add_node("n2", gpus=1)                       # capacity arrives: the group goes through
        ok = await c.wait_bound(3, 8)
        await c.stop()
        return partial, held, ok
    partial, held, ok = run(go())
    assert partial == 0                                # never a partial gang
    assert ok
