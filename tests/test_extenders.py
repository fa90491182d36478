"""HTTP scheduler extenders (KubeSchedulerConfiguration.extenders): filter, prioritize
and bind verbs over real HTTP, ignorable failures, managedResources interest."""
import asyncio

from aiohttp import web

from yoda_scheduler_amd.framework.config import parse_config
from yoda_scheduler_amd.testing import FakeCluster, yoda_config


def run(c):
    return asyncio.run(c)


class ExtenderServer:
    def __init__(self, api_server=None):
        self.calls = {"filter": 0, "prioritize": 0, "bind": 0, "broken": 0}
        self.api = api_server
        self.app = web.Application()
        self.app.router.add_post("/filter", self.filter)
        self.app.router.add_post("/prioritize", self.prioritize)
        self.app.router.add_post("/bind", self.bind)
        self.app.router.add_post("/broken", self.broken)

    async def filter(self, req):
        self.calls["filter"] += 1
        a = await req.json()
        names = a.get("NodeNames") or [n["metadata"]["name"] for n in a["Nodes"]["items"]]
        keep = [n for n in names if not n.endswith("0")]
        return web.json_response({"NodeNames": keep, "FailedNodes": {n: "extender says no" for n in names
                                                                     if n not in keep}})

    async def prioritize(self, req):
        self.calls["prioritize"] += 1
        a = await req.json()
        names = a.get("NodeNames") or [n["metadata"]["name"] for n in a["Nodes"]["items"]]
        return web.json_response([{"Host": n, "Score": 10 if n == "n2" else 0} for n in names])

    async def bind(self, req):
        self.calls["bind"] += 1
        a = await req.json()
        self.api.bind(a["PodNamespace"], a["PodName"], a["PodUID"], a["Node"], {"bound-by": "extender"})
        return web.json_response({})

    async def broken(self, req):
        self.calls["broken"] += 1
        return web.Response(status=500, text="boom")

    async def start(self):
        self.runner = web.AppRunner(self.app)
        await self.runner.setup()
        site = web.TCPSite(self.runner, "127.0.0.1", 0)
        await site.start()
        return f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"

    async def stop(self):
        await self.runner.cleanup()


def test_config_parses_extenders():
    cfg = yoda_config()
    cfg["extenders"] = [{"urlPrefix": "http://x/sched/", "filterVerb": "filter", "prioritizeVerb": "prio",
                         "weight": 3, "httpTimeout": "2s", "nodeCacheCapable": True, "ignorable": True,
                         "managedResources": [{"name": "example.com/fpga", "ignoredByScheduler": True}]}]
    c = parse_config(cfg)
    e = c.extenders[0]
    assert (e.url_prefix, e.filter_verb, e.prioritize_verb, e.weight, e.http_timeout) == \
        ("http://x/sched", "filter", "prio", 3, 2.0)
    assert e.node_cache_capable and e.ignorable and e.managed_resources == [("example.com/fpga", True)]


def test_extender_filter_prioritize_bind_and_ignorable():
    async def go():
        c = FakeCluster(yoda_config())
        ext = ExtenderServer(c.server)
        url = await ext.start()
        cfg = yoda_config()
        cfg["extenders"] = [
            {"urlPrefix": url, "filterVerb": "filter", "prioritizeVerb": "prioritize", "weight": 1000,
             "nodeCacheCapable": True},
            {"urlPrefix": url, "filterVerb": "broken", "ignorable": True},
            {"urlPrefix": url, "bindVerb": "bind",
             "managedResources": [{"name": "example.com/fpga", "ignoredByScheduler": True}]},
        ]
        c.config = parse_config(cfg)
        for i in range(4):
            c.add_node(f"n{i}")
        await c.start()
        for i in range(3):
            c.add_pod(f"p{i}", {"scv/memory": "1000"})
        c.server.create("pods", {"metadata": {"name": "fpga", "namespace": "default", "labels": {}},
                                 "spec": {"schedulerName": "yoda-scheduler", "containers": [
                                     {"name": "c", "image": "x",
                                      "resources": {"requests": {"example.com/fpga": "1"}}}]}})
        ok = await c.wait_bound(4)
        out = ({f"p{i}": c.node_of(f"p{i}") for i in range(3)}, c.node_of("fpga"),
               (c.pod("fpga")["metadata"].get("annotations") or {}).get("bound-by"), dict(ext.calls), ok)
        await c.stop()
        await ext.stop()
        return out
    placed, fpga_node, bound_by, calls, ok = run(go())
    assert ok
    assert all(n != "n0" for n in placed.values())          # filtered by the extender
    assert set(placed.values()) == {"n2"}                  # prioritize 1000 × 10 × 10 outweighs yoda (300 × 100)
    assert fpga_node != "n0" and bound_by == "extender"    # managedResources → extender binds
    assert calls["bind"] == 1 and calls["broken"] >= 4      # ignorable failure did not block


def test_non_ignorable_extender_failure_fails_the_cycle():
    async def go():
        c = FakeCluster(yoda_config(backoff=0.05, max_backoff=0.1))
        ext = ExtenderServer(c.server)
        url = await ext.start()
        cfg = yoda_config(backoff=0.05, max_backoff=0.1)
        cfg["extenders"] = [{"urlPrefix": url, "filterVerb": "broken"}]
        c.config = parse_config(cfg)
        c.add_node("n1")
        await c.start()
        c.add_pod("p", {"scv/memory": "1000"})
        await c.wait(lambda: c.sched.failed >= 2, 3.0)
        out = c.node_of("p"), c.sched.failed
        await c.stop()
        await ext.stop()
        return out
    node, failed = run(go())
    assert node == "" and failed >= 2
