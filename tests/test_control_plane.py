"""HTTP Kubernetes client ↔ fake apiserver HTTP front, scheduling over HTTP, Lease leader
election (single leader, failover, release), sniffer publishing, CLI entry points."""
import asyncio
import json
import os
import subprocess
import sys
import time

import pytest

from yoda_scheduler_amd.fakeapi.http import FakeApiHttp
from yoda_scheduler_amd.fakeapi.server import FakeApiServer
from yoda_scheduler_amd.kube.client import KubeClient, KubeConfig
from yoda_scheduler_amd.kube.errors import ApiError
from yoda_scheduler_amd.models.device import make_node, make_scv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(coro):
    return asyncio.run(coro)


def test_http_client_crud_watch_bind():
    async def go():
        api = FakeApiHttp()
        url = await api.start()
        cl = KubeClient(KubeConfig(url))
        try:
            n = await cl.create("nodes", make_node("n1"))
            assert n["metadata"]["resourceVersion"]
            items, rv = await cl.list("nodes")
            assert [i["metadata"]["name"] for i in items] == ["n1"]
            got = []

            async def watcher():
                async for typ, obj in cl.watch("pods", rv):
                    got.append((typ, obj["metadata"]["name"], (obj.get("spec") or {}).get("nodeName")))
                    if len(got) == 3:
                        return

            t = asyncio.get_event_loop().create_task(watcher())
            await asyncio.sleep(0.05)
            p = await cl.create("pods", {"metadata": {"name": "p", "namespace": "default"}, "spec": {}})
            await cl.bind("default", "p", p["metadata"]["uid"], "n1", {"scv.amd.com/gpus": "0,1"})
            with pytest.raises(ApiError) as ei:
                await cl.bind("default", "p", p["metadata"]["uid"], "n1")
            assert ei.value.code == 409
            await cl.patch("pods", "p", {"metadata": {"labels": {"a": "b"}}}, "default")
            await asyncio.wait_for(t, 3)
            pod = await cl.get("pods", "p", "default")
            assert pod["spec"]["nodeName"] == "n1" and pod["metadata"]["annotations"]["scv.amd.com/gpus"] == "0,1"
            assert pod["metadata"]["labels"] == {"a": "b"}
            stale = dict(pod)
            stale["metadata"] = dict(pod["metadata"], resourceVersion="1")
            with pytest.raises(ApiError) as ei:
                await cl.update("pods", stale, "default")
            assert ei.value.code == 409
            await cl.delete("pods", "p", "default")
            with pytest.raises(ApiError) as ei:
                await cl.get("pods", "p", "default")
            assert ei.value.code == 404
            return got
        finally:
            await cl.close()
            await api.stop()
    got = run(go())
    assert got[0] == ("ADDED", "p", None) and got[1] == ("MODIFIED", "p", "n1")


def test_watch_too_old_resource_version_is_gone():
    async def go():
        srv = FakeApiServer(history=4)
        api = FakeApiHttp(srv)
        url = await api.start()
        cl = KubeClient(KubeConfig(url))
        for i in range(10):
            srv.create("nodes", make_node(f"n{i}"))
        try:
            with pytest.raises(ApiError) as ei:
                async for _ in cl.watch("nodes", "1"):
                    pass
            return ei.value.code
        finally:
            await cl.close()
            await api.stop()
    assert run(go()) == 410


def test_chunked_list_and_expired_continue_over_http():
    """client-go pager semantics: ``limit`` chunks joined through ``continue`` tokens; a
    token older than the apiserver's history window is 410 Expired."""
    async def go():
        srv = FakeApiServer(history=50)
        api = FakeApiHttp(srv)
        url = await api.start()
        cl = KubeClient(KubeConfig(url))
        try:
            for i in range(1234):
                srv.create("nodes", make_node(f"n{i:04d}"))
            before = srv.calls["list"]
            items, rv = await cl.list("nodes", resource_version="", limit=500)
            pages = srv.calls["list"] - before
            first, _rv, cont = srv.list_page("nodes", None, 10, "")
            for i in range(60):                          # push the token's RV out of the window
                srv.create("nodes", make_node(f"late{i}"))
            with pytest.raises(ApiError) as ei:
                srv.list_page("nodes", None, 10, cont)
            return [o["metadata"]["name"] for o in items], rv, pages, ei.value.code, len(first)
        finally:
            await cl.close()
            await api.stop()
    names, rv, pages, code, first = run(go())
    assert names == sorted(f"n{i:04d}" for i in range(1234)) and rv == "1234"
    assert pages == 3 and code == 410 and first == 10


def test_informer_bookmarks_and_consistent_relist_after_gone():
    """BOOKMARK events advance the informer's resourceVersion without touching the store;
    after a 410 the relist is a consistent, paged read."""
    from yoda_scheduler_amd.fakeapi.client import InProcessClient
    from yoda_scheduler_amd.kube.informer import Informer

    async def go():
        srv = FakeApiServer(history=5)
        adds = []
        inf = Informer(InProcessClient(srv), "nodes", on_add=lambda o: adds.append(o["metadata"]["name"]))
        inf.page_size = 2
        srv.create("nodes", make_node("a"))
        task = asyncio.get_event_loop().create_task(inf.run())
        await asyncio.wait_for(inf.synced.wait(), 5)
        srv.create("scvs", make_scv("a", update_time=time.time()).to_json())   # RV moves, no node change
        srv.bookmark("nodes")
        for _ in range(200):
            if inf.bookmarks:
                break
            await asyncio.sleep(0.005)
        rv_after_bookmark = inf.resource_version
        # force a 410: the watch drops, history moves past the informer's RV
        srv.close_watches()
        for i in range(8):
            srv.create("nodes", make_node(f"b{i}"))
        lists0 = srv.calls["list"]
        for _ in range(400):
            if len(inf.store) == 9:
                break
            await asyncio.sleep(0.005)
        inf.stop()
        srv.close_watches()
        task.cancel()
        await asyncio.gather(task, return_exceptions=True)
        return rv_after_bookmark, inf.bookmarks, sorted(inf.store), srv.calls["list"] - lists0, adds
    rv, bookmarks, store, lists, adds = run(go())
    assert bookmarks == 1 and rv == "2"
    assert store == ["a"] + [f"b{i}" for i in range(8)] and sorted(adds) == store
    assert lists >= 5            # 9 nodes in pages of 2


def test_schedule_over_http_with_informer_relist():
    from yoda_scheduler_amd.framework.config import parse_config
    from yoda_scheduler_amd.framework.scheduler import Scheduler
    from yoda_scheduler_amd.testing import yoda_config

    async def go():
        srv = FakeApiServer()
        srv.create("nodes", make_node("n1"))
        s = make_scv("n1", update_time=time.time())
        s.update_interval_ms = 600_000
        srv.create("scvs", s.to_json())
        api = FakeApiHttp(srv)
        url = await api.start()
        cl = KubeClient(KubeConfig(url))
        sched = Scheduler(cl, parse_config(yoda_config()))
        await sched.start()
        loop_t = asyncio.get_event_loop().create_task(sched.scheduling_loop())
        for i in range(20):
            srv.create("pods", {"metadata": {"name": f"p{i}", "namespace": "default", "labels": {"scv/memory": "100"}},
                                "spec": {"schedulerName": "yoda-scheduler"}})
            if i == 10:
                srv.close_watches()          # informers must resume from their resourceVersion
        t0 = time.time()
        while len(srv.bind_log) < 20 and time.time() - t0 < 10:
            await asyncio.sleep(0.01)
        n = len(srv.bind_log)
        await sched.shutdown()
        loop_t.cancel()
        await cl.close()
        await api.stop()
        return n
    assert run(go()) == 20


def test_leader_election_single_leader_and_failover():
    from yoda_scheduler_amd.fakeapi.client import InProcessClient
    from yoda_scheduler_amd.framework.leader import LeaderElector

    async def go():
        srv = FakeApiServer()
        cl = InProcessClient(srv)
        a = LeaderElector(cl, identity="a", lease_duration=0.6, renew_deadline=0.4, retry_period=0.1)
        b = LeaderElector(cl, identity="b", lease_duration=0.6, renew_deadline=0.4, retry_period=0.1)
        await a.acquire()
        tb = asyncio.get_event_loop().create_task(b.acquire())
        await asyncio.sleep(0.8)
        assert a.is_leader and not b.is_leader and not tb.done()
        # a stops renewing (crash): b takes over after the lease expires
        a._task.cancel()
        await asyncio.wait_for(tb, 3)
        assert b.is_leader
        lease = srv.get("leases", "yoda-scheduler", "kube-system")
        assert lease["spec"]["holderIdentity"] == "b" and lease["spec"]["leaseTransitions"] == 1
        # clean release lets a standby in immediately
        await b.release()
        c = LeaderElector(cl, identity="c", lease_duration=5, renew_deadline=4, retry_period=0.1)
        await asyncio.wait_for(c.acquire(), 2)
        await c.release()
        return True
    assert run(go())


@pytest.mark.parametrize("lock", ["endpoints", "configmaps", "endpointsleases"])
def test_leader_election_legacy_and_multi_locks(lock):
    """client-go EndpointsLock / ConfigMapLock (record in the leader annotation) and the
    endpointsleases multilock (legacy primary + Lease kept in step)."""
    from yoda_scheduler_amd.fakeapi.client import InProcessClient
    from yoda_scheduler_amd.framework.leader import LEADER_ANNOTATION, LeaderElector

    async def go():
        srv = FakeApiServer()
        cl = InProcessClient(srv)
        kw = dict(lease_duration=0.6, renew_deadline=0.4, retry_period=0.1, resource_lock=lock)
        a = LeaderElector(cl, identity="a", **kw)
        b = LeaderElector(cl, identity="b", **kw)
        await a.acquire()
        tb = asyncio.get_event_loop().create_task(b.acquire())
        await asyncio.sleep(0.5)
        assert a.is_leader and not tb.done()
        a._task.cancel()
        await asyncio.wait_for(tb, 3)
        res = "configmaps" if lock == "configmaps" else "endpoints"
        rec = json.loads(srv.get(res, "yoda-scheduler", "kube-system")["metadata"]["annotations"][LEADER_ANNOTATION])
        lease = srv.get("leases", "yoda-scheduler", "kube-system") if lock.endswith("leases") else None
        await b.release()
        return rec, lease
    rec, lease = run(go())
    assert rec["holderIdentity"] == "b" and rec["leaderTransitions"] == 1
    if lock.endswith("leases"):
        assert lease["spec"]["holderIdentity"] == "b"


def test_unknown_lock_type_rejected():
    from yoda_scheduler_amd.framework.leader import LeaderElector
    with pytest.raises(ValueError):
        LeaderElector(object(), resource_lock="etcd")


def test_leader_loses_lease_when_apiserver_unreachable():
    from yoda_scheduler_amd.framework.leader import LeaderElector

    class Flaky:
        def __init__(self, inner):
            self.inner, self.down = inner, False

        def __getattr__(self, n):
            f = getattr(self.inner, n)

            async def w(*a, **k):
                if self.down:
                    raise ApiError(503, "ServiceUnavailable", "down")
                return await f(*a, **k)
            return w

    from yoda_scheduler_amd.fakeapi.client import InProcessClient

    async def go():
        cl = Flaky(InProcessClient(FakeApiServer()))
        a = LeaderElector(cl, identity="a", lease_duration=0.5, renew_deadline=0.3, retry_period=0.05)
        await a.acquire()
        cl.down = True
        await asyncio.wait_for(a.lost.wait(), 3)
        return a.is_leader
    assert run(go()) is False


def test_sniffer_agent_publishes_and_updates():
    from yoda_scheduler_amd.fakeapi.client import InProcessClient
    from yoda_scheduler_amd.sniffer.collector import FakeBackend
    from yoda_scheduler_amd.sniffer.publisher import SnifferAgent

    async def go():
        srv = FakeApiServer()
        be = FakeBackend(8)
        agent = SnifferAgent(InProcessClient(srv), "node-x", be, interval=0.01)
        await agent.run(count=3)
        be.state[3].ecc_uncorrectable = 2          # fault injection: ECC error on GPU 3
        be.state[0].used_mb = 100_000
        be.state[1].link_load = {2: 0.8}
        await agent.publish_once()
        return srv.get("scvs", "node-x")
    obj = run(go())
    from yoda_scheduler_amd.models.scv import Scv
    s = Scv.from_json(obj)
    assert s.status.card_number == 8 and s.status.card_list[3].health == "Unhealthy"
    assert s.status.card_list[0].free_memory == 294912 - 100_000
    assert any(l.peer == 2 and l.load == pytest.approx(0.8) for l in s.status.card_list[1].xgmi)
    assert int(obj["metadata"]["resourceVersion"]) > 1


def test_cli_write_config_and_sniffer_print():
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-m", "yoda_scheduler_amd.cmd.scheduler", "--config",
                          os.path.join(ROOT, "deploy", "yoda-scheduler.yaml"), "--v=3", "--write-config-to", "-",
                          "--authentication-kubeconfig=/x"],
                         capture_output=True, text=True, env=env, timeout=60)
    assert out.returncode == 0, out.stderr
    cfg = json.loads(out.stdout)
    assert [p["scheduler_name"] for p in cfg["profiles"]] == ["yoda-scheduler2", "yoda-scheduler"]
    out = subprocess.run([sys.executable, "-m", "yoda_scheduler_amd.cmd.sniffer", "--print", "--backend", "fake",
                          "--node", "n0", "--fake-gpus", "4"], capture_output=True, text=True, env=env, timeout=60)
    assert out.returncode == 0, out.stderr
    scv = json.loads(out.stdout)
    assert scv["metadata"]["name"] == "n0" and scv["status"]["cardNumber"] == 4


def test_cli_fake_cluster_serves_health_and_schedules():
    """End-to-end process test: yoda-scheduler --fake-cluster with its fake apiserver on
    HTTP; a pod posted over HTTP gets bound; /healthz and /metrics answer."""
    import socket

    def free_port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    api_port, status_port = free_port(), free_port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    proc = subprocess.Popen([sys.executable, "-m", "yoda_scheduler_amd.cmd.scheduler", "--fake-cluster", "2",
                             "--fake-apiserver-port", str(api_port), "--port", str(status_port),
                             "--bind-address", "127.0.0.1", "--device-scorer", "off"],
                            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)

    async def go():
        cl = KubeClient(KubeConfig(f"http://127.0.0.1:{api_port}"))
        try:
            for _ in range(200):
                try:
                    await cl.list("nodes")
                    break
                except Exception:
                    await asyncio.sleep(0.05)
            await cl.create("pods", {"metadata": {"name": "cli", "namespace": "default",
                                                  "labels": {"scv/memory": "1000"}},
                                     "spec": {"schedulerName": "yoda-scheduler", "priority": 7, "containers": [
                                         {"name": "c", "resources": {"requests": {"cpu": "250m"}}}]}})
            for _ in range(200):
                pod = await cl.get("pods", "cli", "default")
                if pod["spec"].get("nodeName"):
                    break
                await asyncio.sleep(0.05)
            import aiohttp
            async with aiohttp.ClientSession() as s:
                async with s.get(f"http://127.0.0.1:{status_port}/healthz") as r:
                    health = await r.text()
                async with s.get(f"http://127.0.0.1:{status_port}/metrics") as r:
                    metrics = await r.text()
                async with s.get(f"http://127.0.0.1:{status_port}/debug/pprof/profile?seconds=0.3&limit=5") as r:
                    prof = await r.text()
                async with s.get(f"http://127.0.0.1:{status_port}/debug/pprof/goroutine") as r:
                    stacks = await r.text()
                async with s.get(f"http://127.0.0.1:{status_port}/debug/pprof/heap") as r:
                    heap = await r.json()
                async with s.get(f"http://127.0.0.1:{status_port}/configz") as r:
                    configz = await r.json()
                async with s.get(f"http://127.0.0.1:{status_port}/metrics/resources") as r:
                    resources = await r.text()
                async with s.get(f"http://127.0.0.1:{status_port}/debug/cache") as r:
                    cache = await r.json()
                proc.send_signal(__import__("signal").SIGUSR2)      # cache comparer + dump to the log
                await asyncio.sleep(0.3)
            return pod, health, metrics, (prof, stacks, heap, configz, resources, cache)
        finally:
            await cl.close()

    try:
        pod, health, metrics, (prof, stacks, heap, configz, resources, cache) = run(go())
    finally:
        proc.terminate()
        try:
            out, _ = proc.communicate(timeout=10)
        except subprocess.TimeoutExpired:
            proc.kill()
            out = ""
    assert pod["spec"]["nodeName"].startswith("mi355x-")
    assert health == "ok"
    assert "scheduler_schedule_attempts_total" in metrics
    assert "function calls" in prof and "asyncio task(s)" in stacks and heap["objects"] > 0
    assert "componentconfig" in configz
    node = pod["spec"]["nodeName"]
    assert (f'kube_pod_resource_request{{namespace="default",node="{node}",pod="cli",priority="7",resource="cpu",'
            f'scheduler="yoda-scheduler",unit="cores"}} 0.25') in resources
    assert all(not v for section in cache["comparison"].values() for v in section.values()), cache["comparison"]
    assert cache["dump"]["nodes"][node]["pods"] == ["default/cli"]
    assert "cache comparer: cache matches the informers" in out


def test_tracer_chrome_trace():
    from yoda_scheduler_amd.testing import FakeCluster, yoda_config

    async def go():
        cfg = yoda_config()
        cfg["yodaRuntime"]["trace"] = True
        c = FakeCluster(cfg)
        c.add_node("n")
        await c.start()
        for i in range(5):
            c.add_pod(f"p{i}", {"scv/memory": "1"})
        await c.wait_bound(5)
        await asyncio.sleep(0.02)
        tr = c.sched.tracer.chrome_trace()
        await c.stop()
        return tr
    tr = run(go())
    names = {e["name"] for e in tr["traceEvents"]}
    assert "bind" in names and ({"cycle", "native_batch"} & names)


def test_https_kubeconfig_with_ca_data_and_token(tmp_path):
    """The production client path: HTTPS with the cluster CA from a kubeconfig's
    ``certificate-authority-data`` and a bearer token; a wrong token is rejected (401) and
    an unknown CA fails the TLS handshake. A scheduler over that client binds a pod."""
    import base64
    import shutil
    import ssl

    if not shutil.which("openssl"):
        pytest.skip("openssl not available")
    d = tmp_path
    sh = lambda *a: subprocess.run(a, check=True, capture_output=True)  # noqa: E731
    sh("openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "1", "-subj", "/CN=yoda-test-ca",
       "-keyout", str(d / "ca.key"), "-out", str(d / "ca.crt"))
    sh("openssl", "req", "-newkey", "rsa:2048", "-nodes", "-subj", "/CN=127.0.0.1",
       "-keyout", str(d / "srv.key"), "-out", str(d / "srv.csr"))
    (d / "ext.cnf").write_text("subjectAltName=IP:127.0.0.1\n")
    sh("openssl", "x509", "-req", "-in", str(d / "srv.csr"), "-CA", str(d / "ca.crt"), "-CAkey", str(d / "ca.key"),
       "-CAcreateserial", "-days", "1", "-extfile", str(d / "ext.cnf"), "-out", str(d / "srv.crt"))
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(str(d / "srv.crt"), str(d / "srv.key"))

    async def go():
        from yoda_scheduler_amd.framework.config import parse_config
        from yoda_scheduler_amd.framework.scheduler import Scheduler
        from yoda_scheduler_amd.testing import yoda_config
        srv = FakeApiServer()
        srv.create("nodes", make_node("n0"))
        scv = make_scv("n0", update_time=time.time())
        scv.update_interval_ms = 60_000
        srv.create("scvs", scv.to_json())
        api = FakeApiHttp(srv, ssl_context=ctx, token="s3cret")
        url = await api.start()
        ca_b64 = base64.b64encode((d / "ca.crt").read_bytes()).decode()
        kc = {"apiVersion": "v1", "kind": "Config", "current-context": "t",
              "clusters": [{"name": "c", "cluster": {"server": url, "certificate-authority-data": ca_b64}}],
              "users": [{"name": "u", "user": {"token": "s3cret"}}],
              "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}
        import yaml
        (d / "kubeconfig").write_text(yaml.safe_dump(kc))
        good = KubeClient(KubeConfig.load(str(d / "kubeconfig")))
        bad_token = KubeClient(KubeConfig(url, token="nope", ca_file=str(d / "ca.crt")))
        no_ca = KubeClient(KubeConfig(url, token="s3cret"))
        errors = []
        try:
            nodes, _ = await good.list("nodes")
            for cl in (bad_token, no_ca):
                try:
                    await cl.list("nodes")
                    errors.append("accepted")
                except ApiError as e:
                    errors.append(e.code)
                except Exception as e:  # noqa: BLE001 - TLS verification failure
                    errors.append(type(e).__name__)
            sched = Scheduler(good, parse_config(yoda_config()))
            await sched.start()
            loop_t = asyncio.get_event_loop().create_task(sched.scheduling_loop())
            await good.create("pods", {"metadata": {"name": "tls", "namespace": "default",
                                                    "labels": {"scv/memory": "1000"}},
                                       "spec": {"schedulerName": "yoda-scheduler"}})
            for _ in range(400):
                if srv.bind_log:
                    break
                await asyncio.sleep(0.01)
            await sched.shutdown()
            loop_t.cancel()
            return len(nodes), errors, dict(srv.bind_node)
        finally:
            for cl in (good, bad_token, no_ca):
                await cl.close()
            await api.stop()

    n, errors, bound = run(go())
    assert n == 1
    assert errors[0] == 401 and errors[1] != "accepted"
    assert bound == {"default/tls": "n0"}


def test_bench_http_transport_contract():
    """bench.py --transport http: apiserver in its own process, scheduler over the HTTP
    client; every pod of a config-2 burst is bound and the JSON line follows the contract."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--transport", "http", "--config", "2",
                        "--steps", "2", "--warmup", "1"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["transport"] == "http" and d["pods_bound"] == 200 and d["pods_unschedulable"] == 0
    assert d["value"] > 0 and d["p99_latency_ms"] > 0 and d["e2e_scheduling_p99_ms"] is not None
    # the harness's own bound is reported, and the scheduler process ran with its malloc
    # tunable (bench.py re-executed itself; the environment here did not set one)
    assert 0.0 < d["apiserver_busy_share_of_bursts"] <= 1.5
    if "GLIBC_TUNABLES" not in os.environ:
        assert d["malloc"] == "glibc.malloc.tcache_count=2048"


def test_bench_malloc_opt_out_keeps_glibc_defaults():
    env = dict(os.environ, PYTHONPATH=ROOT, YODA_BENCH_MALLOC="default")
    env.pop("GLIBC_TUNABLES", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "1", "--steps", "1",
                        "--warmup", "0", "--alt", "none"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["malloc"] == "glibc defaults"


def test_fastbind_pipelining_errors_chunked_and_reconnect():
    """The pipelined binding client: many binds in flight over a few connections against
    the fake apiserver (404 / 409 surface as ApiError), and against a raw server that
    answers with a chunked body and then closes the connection (the client reconnects)."""
    from yoda_scheduler_amd.kube.fastbind import FastBinder

    async def go():
        srv = FakeApiServer()
        srv.create("nodes", make_node("n0"))
        for i in range(300):
            srv.create("pods", {"metadata": {"name": f"p{i}", "namespace": "default"}, "spec": {}})
        api = FakeApiHttp(srv)
        url = await api.start()
        fb = FastBinder(url, conns=3, max_inflight=8)
        await asyncio.gather(*(fb.bind("default", f"p{i}", "", "n0") for i in range(300)))
        codes = []
        for name in ("p0", "missing"):
            try:
                await fb.bind("default", name, "", "n0")
            except ApiError as e:
                codes.append(e.code)
        await fb.close()
        await api.stop()

        # raw server: chunked 201, then "Connection: close"
        served = []

        async def handle(r, w):
            while True:
                line = await r.readline()
                if not line:
                    break
                length = 0
                while True:
                    h = await r.readline()
                    if h in (b"\r\n", b""):
                        break
                    if h.lower().startswith(b"content-length:"):
                        length = int(h.split(b":")[1])
                await r.readexactly(length)
                served.append(1)
                close = len(served) % 2 == 0
                w.write(b"HTTP/1.1 201 Created\r\nTransfer-Encoding: chunked\r\n" +
                        (b"Connection: close\r\n" if close else b"") + b"\r\n4\r\n{\"a\"\r\n3\r\n:1}\r\n0\r\n\r\n")
                await w.drain()
                if close:
                    w.close()
                    return
        raw = await asyncio.start_server(handle, "127.0.0.1", 0)
        port = raw.sockets[0].getsockname()[1]
        fb2 = FastBinder(f"http://127.0.0.1:{port}", conns=1)
        for i in range(6):
            await fb2.bind("default", f"x{i}", "", "n0")
        await fb2.close()
        raw.close()
        await raw.wait_closed()
        return len(srv.bind_log), codes, len(served)

    bound, codes, served = run(go())
    assert bound == 300
    assert codes == [409, 404]
    assert served == 6


def test_bench_node_gpus_sweep_option():
    """BASELINE protocol item 5 (every config at 1/2/4/8 GPUs per node): ``--node-gpus``
    resizes the synthetic nodes; pods asking for more GPUs than a node has are reported as
    unschedulable, everything else binds."""
    from yoda_scheduler_amd.bench.workloads import make_workload
    w = make_workload(5, node_gpus=2)
    assert [g for _n, _s, g in w.nodes] == [2, 2, 2, 2] and "4 nodes x 2 MI355X" in w.name
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "2", "--node-gpus", "4",
                        "--steps", "1", "--warmup", "0"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["node_gpus"] == 4 and d["pods_bound"] == 100 and "1 node x 4 MI355X" in d["config"]["model"]
    # a burst that leaves pods unschedulable (config 3's 2/4/8-GPU pods on a 1-GPU node) ends
    # once every pod is bound or parked, and the next burst's reset waits for the mirror of
    # lane pods the Python path read to empty (both used to hang)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "3", "--node-gpus", "1",
                        "--steps", "1", "--warmup", "1", "--alt", "none"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["pods_bound"] > 0 and d["pods_unschedulable"] > 0
    assert d["pods_bound"] + d["pods_unschedulable"] == 1000


def test_bench_headline_reset_stays_small_and_mirror_off():
    """Guard of the driver's headline: the driver's command on config 3
    binds every pod, the lane's change log (the Python mirror of lane pods) never switches on
    in an all-native burst, and the reset between bursts (deleting the previous burst and
    waiting for the releases, inside the timed step) stays well below the burst itself.
    Syncing the mirror from the reset loop broke all three in round 3 (≈30 % of the headline)."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    # the timing bound is a ratio of medians on a shared CPU (a loaded test runner can stretch
    # one reset): a second run decides; the mirror/log checks are exact on every run
    for attempt in range(2):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                            "--alt", "none"], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
        assert d["pods_bound"] == 3000 and d["pods_unschedulable"] == 0
        assert d["lane_log_on"] is False
        bursts = sorted(s - rs for s, rs in zip(d["step_ms"], d["reset_ms"]))
        # absolute: against the host's single-thread calibration loop (a
        # ratio to the burst let a +55 % reset pass). MI355X boxes: 0.26-0.29x with the fix,
        # 0.39x at round 5's regression; this container runs ~2x slower per event and noisier
        calib = d["host"]["calib_loop_ms"]
        if d["reset_ms_median"] <= 1.0 * calib or attempt == 1:
            break
    assert d["reset_ms_median"] <= 0.5 * bursts[len(bursts) // 2], (d["reset_ms"], d["step_ms"])
    assert d["reset_ms_median"] <= 1.0 * calib, (d["reset_ms"], calib)
    assert d["burst_only_pods_per_s"] >= d["value"]
    # the engine's share of a lane pod stays a small part of the scheduler's CPU per pod
    assert d["lane_engine_us_per_pod"]["cpu"] <= 0.5 * d["cpu_us_per_pod"]


def test_bench_nodes_option_resizes_config_6_only():
    """``--nodes`` (the CPU/device crossover end to end) resizes config 6's cluster and is
    refused for the BASELINE configs, whose cluster shapes are fixed by BASELINE.json."""
    from yoda_scheduler_amd.bench.workloads import make_workload
    w = make_workload(6, nodes=64)
    assert len(w.nodes) == 64 and "64 nodes x 8 MI355X" in w.name and w.n_pods == 1000
    assert len({n for n, _s, _g in w.nodes}) == 64
    with pytest.raises(ValueError):
        make_workload(3, nodes=64)


def test_wait_for_propagates_cancellation_and_fastbind_timeout():
    """``utils.aio.wait_for`` keeps a caller's cancellation even when the inner awaitable
    finishes in the same loop iteration (asyncio.wait_for on Python < 3.12 returns the
    result instead, which left a bind worker running after scheduler shutdown); the
    pipelined binder times out a request the server never answers."""
    from yoda_scheduler_amd.kube.fastbind import FastBinder
    from yoda_scheduler_amd.utils import aio

    async def race():
        fut = asyncio.get_event_loop().create_future()

        async def inner():
            return await fut
        t = asyncio.ensure_future(aio.wait_for(inner(), 10))
        await asyncio.sleep(0)
        await asyncio.sleep(0)
        fut.set_result(1)
        t.cancel()
        try:
            await t
            return "result"
        except asyncio.CancelledError:
            return "cancelled"

    async def timeout():
        with pytest.raises(asyncio.TimeoutError):
            await aio.wait_for(asyncio.sleep(5), 0.05)

        async def silent(r, w):
            await r.read(1 << 16)            # accept the request, never answer
            await asyncio.sleep(5)
        srv = await asyncio.start_server(silent, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        fb = FastBinder(f"http://127.0.0.1:{port}", conns=1, timeout=0.1)
        t0 = time.monotonic()
        try:
            with pytest.raises(asyncio.TimeoutError):
                await fb.bind("default", "p", "u", "n")
            return time.monotonic() - t0
        finally:
            await fb.close()
            srv.close()
    assert run(race()) == "cancelled"
    assert run(timeout()) < 2.0


def test_scv_engine_view_matches_dataclass_path():
    """ops.native.scv_engine_view (engine input computed straight from the Scv JSON, the
    scheduler's per-update path) equals Scv.from_json → card_tuples / compat_card_tuples +
    link_matrix + the status sums, over randomised objects: missing fields, absent amd
    blocks, physical ids (partitions), link loads/downs, ECC, health strings, Go-style
    negative numbers; LazyScv decodes to the same Scv."""
    import random as _r

    from yoda_scheduler_amd.models.device import make_scv
    from yoda_scheduler_amd.models.scv import LazyScv, Scv, XgmiLink
    from yoda_scheduler_amd.ops.native import card_tuples, compat_card_tuples, link_matrix, scv_engine_view

    rng = _r.Random(11)
    for trial in range(300):
        s = make_scv(f"n{trial}", update_time=1.7e9 + trial, used_mb=[rng.randint(0, 200_000) for _ in range(8)])
        for c in s.status.card_list:
            c.health = rng.choice(["Healthy", "Healthy", "Unhealthy", ""])
            c.ecc_uncorrectable = rng.choice([0, 0, 0, 2])
            c.xgmi_links_up = rng.random() > 0.1
            c.cu_occupancy = rng.choice([0.0, 12.345, 99.99])
            c.numa_node = rng.choice([0, 1, 3])
            c.uuid = rng.choice(["", f"uuid-{c.id}"])
            c.hip_uuid = rng.choice(["", f"GPU-{trial:04d}{c.id}"])
            c.hip_id = rng.choice([-1, 7 - c.id])
            if trial % 3 == 0:
                c.physical_id = c.id // 2          # partitions
            c.xgmi = [XgmiLink(peer=p, load=rng.choice([0.0, 0.2, 0.95, 1.4, -0.1]), up=rng.random() > 0.05)
                      for p in range(8) if p != c.phys and rng.random() > 0.2]
        s.status.recompute_sums()
        obj = s.to_json()
        if trial % 7 == 0:
            del obj["status"]["amd"]
        if trial % 11 == 0:
            for cj in obj["status"]["cardList"]:
                cj.pop(rng.choice(list(cj)), None)
        if trial % 13 == 0:
            obj["status"]["cardList"][0]["freeMemory"] = -5
        ref = Scv.from_json(obj)
        for compat in (False, True):
            view = scv_engine_view(obj, compat)
            cards = compat_card_tuples(ref) if compat else card_tuples(ref)
            st = ref.status
            want = (cards, st.card_number & (2**64 - 1), st.free_memory_sum & (2**64 - 1),
                    st.total_memory_sum & (2**64 - 1), float(st.update_time or 0.0), *link_matrix(ref))
            assert view == want, (trial, compat)
        lz = LazyScv(obj, scv_engine_view(obj, False))
        want_ids = [(c.id, c.uuid, c.hip_uuid, c.hip_id) for c in ref.status.card_list]
        assert lz.card_idents() == want_ids
        assert lz._scv is None                     # identities read without decoding
        ids: list = []                             # ... or taken in the engine-view pass
        assert LazyScv(obj, scv_engine_view(obj, False, ids), ids).card_idents() == want_ids
        assert lz.is_stale(1.7e9 + trial + 100, 3.0) == ref.is_stale(1.7e9 + trial + 100, 3.0)
        assert lz.card_number == ref.status.card_number and lz.status.card_list == ref.status.card_list


def test_cpu_affinity_spec_and_l3_grouping(monkeypatch):
    """--cpu-affinity: `none` leaves the mask alone, `l3:<i>` pins to the i-th last-level-cache
    domain of the allowed CPUs (modulo their number), a single domain is left alone."""
    import os

    from yoda_scheduler_amd.utils import affinity
    assert affinity.apply("none") is None
    with pytest.raises(ValueError):
        affinity.apply("numa")
    shared = {0: "0-1,4-5", 1: "0-1,4-5", 4: "0-1,4-5", 5: "0-1,4-5", 2: "2-3,6-7", 3: "2-3,6-7", 6: "2-3,6-7",
              7: "2-3,6-7"}
    real_open = open

    def fake_open(path, *a, **k):
        if path.startswith("/sys/devices/system/cpu/cpu") and path.endswith("shared_cpu_list"):
            import io
            return io.StringIO(shared[int(path.split("/cpu/cpu")[1].split("/")[0])])
        return real_open(path, *a, **k)
    got = []
    monkeypatch.setattr("builtins.open", fake_open)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(8)))
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: got.append(list(cpus)))
    assert affinity.l3_cpu_sets() == [[0, 1, 4, 5], [2, 3, 6, 7]]
    # `l3` takes the least busy domain (other tenants), `l3:<i>` the i-th
    monkeypatch.setattr(affinity, "_busy_fractions", lambda cpus: {c: (0.9 if c in (0, 1, 4, 5) else 0.1) for c in cpus})
    assert affinity.apply("l3") == [2, 3, 6, 7] and affinity.apply("l3:2") == [0, 1, 4, 5]
    assert got == [[2, 3, 6, 7], [0, 1, 4, 5]]
    # several bench ranks: rank 0 ranks the domains most idle first, rank r takes the r-th
    assert affinity.ranked_l3_sets() == [[2, 3, 6, 7], [0, 1, 4, 5]]
    monkeypatch.setattr(affinity, "_busy_fractions", lambda cpus: {c: 0.0 for c in cpus})
    assert affinity.ranked_l3_sets() == [[0, 1, 4, 5], [2, 3, 6, 7]]     # ties keep CPU order
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: {0, 1})
    assert affinity.apply("l3") is None


def test_parallelism_sets_engine_threads_unless_engine_threads_is_given():
    """Upstream `parallelism` (v1beta2+) sizes the C++ engine's node fan-out when the yoda
    runtime block does not; neither set keeps one thread (the reference's v1beta1 documents)."""
    from yoda_scheduler_amd.framework.config import parse_config
    base = {"apiVersion": "kubescheduler.config.k8s.io/v1beta2", "kind": "KubeSchedulerConfiguration"}
    assert parse_config(dict(base)).engine_threads == 1
    assert parse_config(dict(base, parallelism=8)).engine_threads == 8
    assert parse_config(dict(base, parallelism=8, yodaRuntime={"engineThreads": 2})).engine_threads == 2
    with pytest.raises(ValueError):
        parse_config(dict(base, parallelism=0))


def test_cli_serves_healthz_on_its_own_bind_address(tmp_path):
    """v1beta1 `healthzBindAddress` different from `metricsBindAddress`: /healthz answers on
    its own listener, /metrics on the metrics one (upstream serves two listeners then)."""
    import socket
    import time
    import urllib.request

    def free_port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    mport, hport = free_port(), free_port()
    cfg = tmp_path / "sched.yaml"
    cfg.write_text("apiVersion: kubescheduler.config.k8s.io/v1beta1\nkind: KubeSchedulerConfiguration\n"
                   "leaderElection:\n  leaderElect: false\n"
                   f"metricsBindAddress: 127.0.0.1:{mport}\nhealthzBindAddress: 127.0.0.1:{hport}\n"
                   "profiles:\n- schedulerName: yoda-scheduler\n")
    env = dict(os.environ, PYTHONPATH=ROOT)
    proc = subprocess.Popen([sys.executable, "-m", "yoda_scheduler_amd.cmd.scheduler", "--config", str(cfg),
                             "--fake-cluster", "1", "--device-scorer", "off"],
                            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        def get(port, path):
            for _ in range(200):
                try:
                    with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=2) as r:
                        return r.status, r.read().decode()
                except OSError:
                    if proc.poll() is not None:
                        raise AssertionError(proc.stdout.read()[-3000:])
                    time.sleep(0.05)
            raise AssertionError("no answer")
        assert get(hport, "/healthz") == (200, "ok")
        status, body = get(mport, "/metrics")
        assert status == 200 and "scheduler_" in body
    finally:
        proc.terminate()
        proc.wait(timeout=30)


def test_kind_cluster_keeps_the_native_lane_on():
    """in a realistic cluster — every node reports ``status.images`` and
    allocatable ``ephemeral-storage``, the ``default/kubernetes`` and ``kube-system/kube-dns``
    Services exist, 30 % of the burst belongs to a Service-selected ReplicaSet and 20 % requests
    ``ephemeral-storage`` — every profile stays on the native lane and every pod of the burst is
    placed there: none is forwarded to or handed over to the Python path."""
    from yoda_scheduler_amd.bench.harness import HttpShard
    from yoda_scheduler_amd.bench.workloads import make_workload

    async def go():
        w = make_workload(3, cluster="kind")
        assert w.cluster == "kind" and any(w.metas.values())
        assert sum("ephemeral-storage" in str(s) for s in w.specs.values()) >= 100
        sh = HttpShard(w, events=False)
        try:
            await sh.start()
            s = sh.sched
            assert s.lane is not None
            fw = s.frameworks[w.scheduler_name]
            assert s.lane.eligible_mask(fw) is not None, "the profile left the lane"
            assert s.cache.image_nodes and s.engine.image_nodes("docker.io/rocm/vllm:v0.6.4") == 1
            r1 = await sh.burst("a")
            r2 = await sh.burst("b")
            st = s.lane.lane.stats()
            return r1, r2, st, s.lane.handoffs, s.lane.forwarded, None
        finally:
            await sh.stop()

    r1, r2, st, handoffs, forwarded, _ = run(go())
    assert r1.bound == r2.bound == 1000 and r1.unschedulable == r2.unschedulable == 0
    assert st["admitted"] >= 2000 and st["scheduled"] >= 2000
    assert handoffs == 0 and st["unschedulable"] == 0
    # bound pods' echoes of other schedulers aside, nothing of the burst reached Python
    assert forwarded == 0, forwarded


def test_spread_and_anti_affinity_bursts_stay_on_the_native_lane():
    """a 1000-pod burst where every pod has a hostname DoNotSchedule
    topologySpreadConstraint, and a burst with required-anti-affinity pods mixed in, are placed
    entirely by the native lane (native PodTopologySpread / InterPodAffinity): nothing is handed
    to or forwarded to the Python path."""
    from yoda_scheduler_amd.bench.harness import HttpShard
    from yoda_scheduler_amd.bench.workloads import make_workload

    async def go(w):
        sh = HttpShard(w, events=False)
        try:
            await sh.start()
            r = await sh.burst("a")
            st = sh.sched.lane.lane.stats()
            return r, st, sh.sched.lane.handoffs, sh.sched.lane.forwarded
        finally:
            await sh.stop()

    for w in (make_workload(3, mix_spread=1000), make_workload(3, mix_anti=10)):
        r, st, handoffs, forwarded = run(go(w))
        assert r.bound == 1000 and r.unschedulable == 0, w.name
        assert st["admitted"] == 1000 and handoffs == 0 and forwarded == 0, (w.name, st["admitted"], forwarded)
