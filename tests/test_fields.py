"""Field selectors on lists and watches (apiserver semantics) and the scheduler's pod
informer filter ``status.phase!=Succeeded,status.phase!=Failed`` (upstream v1.20)."""
import asyncio

import pytest

from yoda_scheduler_amd.fakeapi.http import FakeApiHttp
from yoda_scheduler_amd.fakeapi.server import FakeApiServer
from yoda_scheduler_amd.kube.client import KubeClient, KubeConfig
from yoda_scheduler_amd.kube.fields import FieldSelector, filter_event, parse
from yoda_scheduler_amd.testing import FakeCluster

TERMINAL = "status.phase!=Succeeded,status.phase!=Failed"


def run(c):
    return asyncio.run(c)


def pod(name, phase=None, node=None):
    o = {"metadata": {"name": name, "namespace": "default"}, "spec": {}}
    if phase:
        o["status"] = {"phase": phase}
    if node:
        o["spec"]["nodeName"] = node
    return o


def test_selector_parse_and_match():
    s = FieldSelector(TERMINAL)
    assert s.matches(pod("a")) and s.matches(pod("a", "Running")) and not s.matches(pod("a", "Failed"))
    unassigned = FieldSelector("spec.nodeName=")
    assert unassigned.matches(pod("a")) and not unassigned.matches(pod("a", node="n1"))
    assert FieldSelector("metadata.name==b,spec.nodeName=n1").matches(pod("b", node="n1"))
    assert not FieldSelector("metadata.name=a,metadata.name=b").matches(pod("a"))
    assert parse("") is None and parse(None) is None
    with pytest.raises(ValueError):
        FieldSelector("status.phase")


def test_watch_event_transitions():
    s = FieldSelector(TERMINAL)
    run_, done = pod("a", "Running"), pod("a", "Succeeded")
    assert filter_event(s, "MODIFIED", done, run_) == ("DELETED", done)       # stops matching
    assert filter_event(s, "MODIFIED", run_, done) == ("ADDED", run_)         # starts matching
    assert filter_event(s, "MODIFIED", run_, pod("a", "Pending")) == ("MODIFIED", run_)
    assert filter_event(s, "MODIFIED", done, pod("a", "Failed")) is None
    assert filter_event(s, "ADDED", done, None) is None and filter_event(s, "DELETED", done, None) is None


def test_field_selector_over_http_list_and_watch():
    async def go():
        srv = FakeApiServer()
        api = FakeApiHttp(srv)
        url = await api.start()
        cl = KubeClient(KubeConfig(url))
        try:
            srv.create("pods", pod("done", "Succeeded"))
            srv.create("pods", pod("live"))
            items, rv = await cl.list("pods", field_selector=TERMINAL)
            events = []

            async def watcher():
                async for typ, obj in cl.watch("pods", rv, field_selector=TERMINAL):
                    if typ == "BOOKMARK":
                        continue
                    events.append((typ, obj["metadata"]["name"]))
                    if len(events) == 3:
                        return
            t = asyncio.get_event_loop().create_task(watcher())
            await asyncio.sleep(0.05)
            srv.create("pods", pod("new"))
            srv.create("pods", pod("born-dead", "Failed"))                  # never seen
            srv.patch("pods", "live", {"status": {"phase": "Succeeded"}}, "default")
            srv.patch("pods", "new", {"status": {"phase": "Running"}}, "default")
            await asyncio.wait_for(t, 5)
            page, _rv, _c = srv.list_page("pods", None, 10, "", TERMINAL)
            return [o["metadata"]["name"] for o in items], events, [o["metadata"]["name"] for o in page]
        finally:
            await cl.close()
            await api.stop()
    listed, events, page = run(go())
    assert listed == ["live"]
    assert events == [("ADDED", "new"), ("DELETED", "live"), ("MODIFIED", "new")]
    assert page == ["new"]


def test_completed_pod_frees_its_gpu_through_the_filtered_informer():
    async def go():
        c = FakeCluster()
        c.add_node("n", gpus=1)
        await c.start()
        c.add_pod("a", {"scv/memory": "200000"})
        assert await c.wait_bound(1)
        c.add_pod("b", {"scv/memory": "200000"})
        await asyncio.sleep(0.2)
        blocked = c.node_of("b") == ""
        c.server.patch("pods", "a", {"status": {"phase": "Succeeded"}}, "default")
        ok = await c.wait(lambda: c.node_of("b") == "n", 5)
        gone_from_store = "default/a" not in c.sched.informers["pods"].store
        await c.stop()
        return blocked, ok, gone_from_store
    blocked, ok, gone_from_store = run(go())
    assert blocked and ok and gone_from_store
