"""The in-process (Python cycle) path's plumbing: batched watch reads, direct in-process
Bindings, and PodReq sharing between pods of one template."""
from __future__ import annotations

import asyncio

from yoda_scheduler_amd.bench.workloads import pod_object
from yoda_scheduler_amd.fakeapi.client import InProcessClient
from yoda_scheduler_amd.fakeapi.server import FakeApiServer, Faults
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.ops.native import core, pod_req


def run(coro):
    return asyncio.run(coro)


def _pod(i, labels=None, **spec):
    o = pod_object(i, labels or {"scv/number": "1"}, "yoda-scheduler", spec=spec or None)
    return o


def test_watch_batches_deliver_every_queued_event_then_end():
    async def go():
        srv = FakeApiServer()
        cl = InProcessClient(srv)
        got = []
        agen = cl.watch_batches("pods", "0")
        first = asyncio.ensure_future(agen.__anext__())
        await asyncio.sleep(0)              # the watch is registered and parked
        for i in range(5):
            srv.create("pods", _pod(i))
        got.append([e[1]["metadata"]["name"] for e in await first])
        srv.create("pods", _pod(9))
        got.append([e[1]["metadata"]["name"] for e in await agen.__anext__()])
        srv.close_watches()
        try:
            await agen.__anext__()
            ended = False
        except StopAsyncIteration:
            ended = True
        return got, ended
    got, ended = run(go())
    assert got == [[f"burst-{i}" for i in range(5)], ["burst-9"]]
    assert ended


def test_watch_get_and_batches_agree_on_close_and_replay():
    async def go():
        srv = FakeApiServer(faults=Faults(drop_watch_every=3))
        for i in range(2):
            srv.create("pods", _pod(i))
        w = srv.watch("pods", "1")          # replays the event after rv 1, then live
        first = await w.get()
        srv.create("pods", _pod(2))
        srv.create("pods", _pod(3))
        srv.create("pods", _pod(4))         # the third live event closes the watch
        srv.create("pods", _pod(5))         # not delivered
        rest = await w.next_batch()
        return first, rest, await w.next_batch(), await w.get()
    first, rest, after, end = run(go())
    assert first[1]["metadata"]["name"] == "burst-1"
    assert [e[1]["metadata"]["name"] for e in rest] == ["burst-2", "burst-3", "burst-4"]
    assert after is None and end is None


def test_direct_binds_report_status_like_the_native_transport():
    async def go():
        srv = FakeApiServer()
        cl = InProcessClient(srv)
        for i in range(3):
            srv.create("pods", _pod(i))
        uid0 = srv.get("pods", "burst-0")["metadata"]["uid"]
        out = []
        db = cl.direct_binds()
        db.bind_many([("default", "burst-0", uid0, "n1", [("a", "1")]),
                      ("default", "burst-0", uid0, "n2", None),          # already bound: 409
                      ("default", "nope", "", "n1", None)],               # 404
                     [lambda s, b, k=k: out.append((k, s, b)) for k in range(3)])
        assert out == []                    # completions run on a later loop iteration
        await asyncio.sleep(0)
        srv.faults.latency_s = 0.01
        db.bind("default", "burst-1", "", "n1", None, lambda s, b: out.append((3, s, b)))
        await asyncio.sleep(0)
        early = len(out)
        await asyncio.sleep(0.05)
        return out, early, srv.get("pods", "burst-0"), srv.get("pods", "burst-1")
    out, early, p0, p1 = run(go())
    codes = {k: s for k, s, _ in out}
    assert codes == {0: 201, 1: 409, 2: 404, 3: 201}
    assert early == 3                       # the latency-delayed bind completed later
    assert p0["spec"]["nodeName"] == "n1" and p0["metadata"]["annotations"] == {"a": "1"}
    assert p1["spec"]["nodeName"] == "n1"
    assert b"Conflict" in next(b for k, s, b in out if k == 1)


def test_pods_of_one_template_share_a_podreq_and_others_do_not():
    e = core().Engine(False, 1)
    mk = lambda i, labels=None, **spec: PodInfo.from_obj(  # noqa: E731
        dict(_pod(i, labels, **spec), metadata={"name": f"p{i}", "namespace": "default", "uid": f"u{i}",
                                                "labels": labels or {"scv/number": "1"}}))
    a, b = mk(1), mk(2)
    assert pod_req(e, a) is pod_req(e, b)
    c = mk(3, {"scv/number": "2"})
    assert pod_req(e, c) is not pod_req(e, a)
    d = mk(4, tolerations=[{"key": "k", "operator": "Exists"}])
    f = mk(5, tolerations=[{"key": "k", "operator": "Exists"}])
    assert pod_req(e, d) is not pod_req(e, f)   # node-side constraints: never shared
    g = mk(6, topologySpreadConstraints=[{"maxSkew": 1, "topologyKey": "kubernetes.io/hostname",
                                          "whenUnsatisfiable": "DoNotSchedule",
                                          "labelSelector": {"matchLabels": {"scv/number": "1"}}}])
    assert pod_req(e, g) is not pod_req(e, a) and g.native_req.n_spread == 1
    e2 = core().Engine(False, 1)
    assert pod_req(e2, mk(7)) is not pod_req(e, a)   # per engine
