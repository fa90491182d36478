"""Native Kubernetes transport (native/kube): JSON codec, quantity + pod projection parity
with the Python decoders, the C++ transport against both fake apiservers (Python aiohttp
and the native epoll one), and reflector robustness (backoff, handler isolation, token
rotation)."""
from __future__ import annotations

import asyncio
import json
import os
import subprocess
import tempfile
import time

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from yoda_scheduler_amd.fakeapi.http import FakeApiHttp
from yoda_scheduler_amd.fakeapi.server import FakeApiServer, _merge
from yoda_scheduler_amd.kube import native as nat
from yoda_scheduler_amd.kube.client import KubeClient, KubeConfig
from yoda_scheduler_amd.kube.errors import ApiError
from yoda_scheduler_amd.models.device import make_node, make_scv
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.utils.quantity import bytes_of, cpu_millis

K = nat.module()


def run(coro):
    return asyncio.run(coro)


# ============================================================== codec
def test_json_codec_roundtrip_escapes_unicode_numbers():
    doc = {"s": "a\"b\\c\n\t\u0001é漢🚀", "n": [0, -1, 12345678901234567890, 1.5e-7, 3.25],
           "o": {"x": None, "t": True, "f": False, "e": {}, "a": []}}
    raw = json.dumps(doc)
    assert json.loads(K.canonical(raw)) == doc
    # surrogate-pair escapes decode to one code point; numbers keep their source text
    assert json.loads(K.canonical('{"k":"\\ud83d\\ude80","big":12345678901234567890}')) == \
        {"k": "🚀", "big": 12345678901234567890}
    assert K.canonical('{"v": 1.50}') == b'{"v":1.50}'
    for bad in ('{"a":}', '[1,2', '{"a" 1}', '"\x01"', 'nul', '{"a":1}x'):
        with pytest.raises(ValueError):
            K.canonical(bad)


_json_leaf = st.one_of(st.none(), st.booleans(), st.integers(-10**6, 10**6), st.text(max_size=6))
_json = st.recursive(_json_leaf, lambda ch: st.one_of(st.lists(ch, max_size=3),
                                                      st.dictionaries(st.text(max_size=4), ch, max_size=4)),
                     max_leaves=12)


@settings(max_examples=150, deadline=None)
@given(_json, _json)
def test_merge_patch_matches_python(target, patch):
    if not isinstance(target, dict):
        target = {"v": target}
    got = json.loads(K.merge_patch(json.dumps(target), json.dumps(patch)))
    assert got == _merge(target, patch)


# ============================================================== quantities
_qty = st.builds(lambda num, frac, suf: f"{num}{'.' + frac if frac else ''}{suf}",
                 st.integers(0, 10**7), st.one_of(st.just(""), st.from_regex(r"[0-9]{1,4}", fullmatch=True)),
                 st.sampled_from(["", "m", "k", "M", "G", "Ki", "Mi", "Gi", "Ti", "n", "u", "e3", "E2"]))


@settings(max_examples=300, deadline=None)
@given(_qty)
def test_quantity_matches_python_decimal(q):
    # exact where the value fits int64; beyond that the projection defers to Python (None)
    for got, want in ((K.quantity(q, 3), cpu_millis(q)), (K.quantity(q, 0), bytes_of(q))):
        if abs(want) < 2**63:
            assert got == want
        else:
            assert got is None


def test_quantity_rejects_what_python_decides():
    for q in ("1.2.3", "abc", "5x", "--1"):
        assert K.quantity(q, 0) is None


# ============================================================== pod projection
_labels = st.dictionaries(st.sampled_from(["scv/number", "scv/memory", "scv/clock", "scv/priority", "app",
                                           "pod-group.scheduling.sigs.k8s.io"]),
                          st.sampled_from(["1", "2", "512", "x", "-3", "2400"]), max_size=4)
_expr = st.fixed_dictionaries({"key": st.sampled_from(["zone", "gpu", "kubernetes.io/hostname"]),
                               "operator": st.sampled_from(["In", "NotIn", "Exists", "Gt"]),
                               "values": st.lists(st.sampled_from(["a", "b", "3"]), max_size=2)})
_term = st.fixed_dictionaries({}, optional={
    "matchExpressions": st.lists(_expr, max_size=2),
    "matchFields": st.lists(st.fixed_dictionaries({"key": st.sampled_from(["metadata.name", "spec.x"]),
                                                    "operator": st.just("In"),
                                                    "values": st.lists(st.just("n1"), max_size=1)}), max_size=1)})
_container = st.fixed_dictionaries({"name": st.just("c")}, optional={
    "image": st.sampled_from(["rocm/pytorch", "rocm/pytorch:7.0", "registry:5000/x", "img@sha256:ab", ""]),
    "resources": st.fixed_dictionaries({}, optional={"requests": st.fixed_dictionaries({}, optional={
        "cpu": st.sampled_from(["100m", "1", "0.5", "2500m", 2]),
        "memory": st.sampled_from(["128Mi", "1Gi", "1e3", "512", "1.5Gi"]),
        "ephemeral-storage": st.sampled_from(["1Gi", "0", "500M"]),
        "amd.com/gpu": st.sampled_from(["1", "8", 2])})}),
    "ports": st.lists(st.fixed_dictionaries({"containerPort": st.just(80)}, optional={
        "hostPort": st.sampled_from([0, 8080]), "protocol": st.sampled_from(["TCP", "UDP"]),
        "hostIP": st.just("0.0.0.0")}), max_size=2)})
_spec = st.fixed_dictionaries({"containers": st.lists(_container, min_size=1, max_size=3)}, optional={
    "schedulerName": st.sampled_from(["yoda-scheduler", "default-scheduler"]),
    "nodeName": st.sampled_from(["", "n1"]),
    "priority": st.sampled_from([0, 5, -2, 1000000000]),
    "nodeSelector": st.dictionaries(st.sampled_from(["zone", "gpu"]), st.sampled_from(["a", "b"]), max_size=2),
    "initContainers": st.lists(_container, max_size=2),
    "overhead": st.fixed_dictionaries({}, optional={"cpu": st.just("50m"), "memory": st.just("64Mi")}),
    "tolerations": st.lists(st.fixed_dictionaries({}, optional={
        "key": st.sampled_from(["", "gpu", "node.kubernetes.io/not-ready"]),
        "operator": st.sampled_from(["Exists", "Equal", ""]), "value": st.sampled_from(["", "x"]),
        "effect": st.sampled_from(["", "NoSchedule", "NoExecute"]),
        "tolerationSeconds": st.just(300)}), max_size=3),
    "affinity": st.fixed_dictionaries({}, optional={
        "nodeAffinity": st.fixed_dictionaries({}, optional={
            "requiredDuringSchedulingIgnoredDuringExecution": st.fixed_dictionaries(
                {"nodeSelectorTerms": st.lists(_term, max_size=2)}),
            "preferredDuringSchedulingIgnoredDuringExecution": st.lists(st.fixed_dictionaries(
                {"weight": st.integers(1, 100), "preference": _term}), max_size=2)}),
        "podAntiAffinity": st.fixed_dictionaries({}, optional={
            "requiredDuringSchedulingIgnoredDuringExecution": st.lists(st.just({"topologyKey": "zone"}),
                                                                       max_size=1)}),
        "podAffinity": st.fixed_dictionaries({}, optional={
            "preferredDuringSchedulingIgnoredDuringExecution": st.lists(st.just({"weight": 1}), max_size=1)})}),
    "topologySpreadConstraints": st.lists(st.fixed_dictionaries({"topologyKey": st.sampled_from(["zone", "h"])}, optional={
        "maxSkew": st.integers(1, 3), "whenUnsatisfiable": st.sampled_from(["DoNotSchedule", "ScheduleAnyway"]),
        "labelSelector": st.one_of(st.none(), st.fixed_dictionaries({}, optional={
            "matchLabels": st.dictionaries(st.sampled_from(["app", "tier"]), st.sampled_from(["a", "b"]), max_size=2),
            "matchExpressions": st.lists(st.fixed_dictionaries({
                "key": st.sampled_from(["app", "tier"]), "operator": st.sampled_from(["In", "NotIn", "Exists"]),
                "values": st.lists(st.sampled_from(["a", "b"]), max_size=2)}), max_size=2)}))}), max_size=2),
    "volumes": st.lists(st.sampled_from([{"name": "v", "persistentVolumeClaim": {"claimName": "c"}},
                                         {"name": "e", "emptyDir": {}}, {"name": "d", "rbd": {}},
                                         {"name": "g", "ephemeral": {}}]), max_size=2)})
_pod = st.fixed_dictionaries({
    "metadata": st.fixed_dictionaries({"name": st.sampled_from(["p1", "p2"])}, optional={
        "namespace": st.sampled_from(["default", "ml"]), "uid": st.sampled_from(["u1", "u2"]),
        "labels": _labels, "annotations": st.dictionaries(st.sampled_from(["a", "scv.amd.com/gpus"]),
                                                          st.sampled_from(["0,1", "x"]), max_size=2),
        "creationTimestamp": st.just("2026-01-01T00:00:00Z"),
        "ownerReferences": st.lists(st.fixed_dictionaries({"kind": st.sampled_from(["ReplicaSet", "Job",
                                                                                     "ReplicationController"]),
                                                           "name": st.just("o")},
                                                          optional={"controller": st.booleans(),
                                                                    "apiVersion": st.sampled_from(["apps/v1", "v1"]),
                                                                    "uid": st.sampled_from(["o-1", "o-2"])}),
                                    max_size=2),
        "deletionTimestamp": st.sampled_from([None, "2026-01-01T00:00:00Z"])}),
    "spec": _spec})

_FIELDS = ("uid", "namespace", "name", "labels", "gpu", "scheduler_name", "node_name", "cpu_m", "mem", "priority",
           "node_selector", "required_terms", "preferred_terms", "tolerations", "annotations", "host_ports", "flags",
           "ext", "nz_cpu_m", "nz_mem", "images", "containers", "owner", "avoid", "spread", "deleting")


def _norm(v):
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_norm(x) for x in v)
    return v


@settings(max_examples=250, deadline=None)
@given(_pod)
def test_pod_projection_matches_from_obj(pod):
    raw = json.dumps(pod)
    ev = K.project(raw)
    want = PodInfo.from_obj(json.loads(raw))
    got = PodInfo.from_native(ev)
    for f in _FIELDS:
        assert _norm(getattr(got, f)) == _norm(getattr(want, f)), f
    assert ev.ok, "the generated pods are all within the projection's coverage"
    # lazy object decodes to the same pod
    assert got.obj == json.loads(raw)
    key, uid, node, sched, phase, h = ev.ident()
    assert (key, uid, node, sched) == (want.key, want.uid, want.node_name, want.scheduler_name)


@settings(max_examples=250, deadline=None)
@given(_pod, st.sampled_from([{}, {"phase": "Pending"}, {"phase": "Running", "podIP": "10.0.0.1"}]),
       st.booleans())
def test_flat_projection_equals_dom_projection(pod, status, pretty):
    """The watch stream decodes pods with the flat document (flatjson.hpp); every field of
    its projection — including the spec/metadata hash and the fallback decision — equals the
    DOM projection's, on compact and indented JSON and with escaped strings."""
    pod = dict(pod, status=status)
    pod["metadata"] = dict(pod["metadata"], annotations={**(pod["metadata"].get("annotations") or {}),
                                                         "note": "tab\there \"q\" \u00e9\u2603"})
    raw = json.dumps(pod, indent=2 if pretty else None, ensure_ascii=pretty)
    a, b = K.project(raw), K.project_flat(raw)
    assert a.ident() == b.ident() and a.ok == b.ok and a.flags == b.flags and a.rv == b.rv
    assert a.info_args() == b.info_args()
    assert a.hash == b.hash


@settings(max_examples=300, deadline=None)
@given(_pod, st.sampled_from(["MODIFIED", "DELETED", "ADDED"]),
       st.sampled_from([None, {}, {"phase": "Running"}, {"phase": 3}, [], "x"]),
       st.sampled_from([None, "", "2026-01-01T00:00:00Z", 0, 1, 0.5, {}, {"a": 1}, [], [0], True, False]),
       st.booleans(), st.booleans())
def test_watch_identity_scan_equals_the_parser(pod, typ, status, deletion, pretty, escaped):
    """The transport reads echo and delete events of a lane-attached pod watch with a skipping
    scan instead of the flat parser: type, object span and every identity field agree with
    the parser path; a field with escapes makes the scan defer (None), never disagree."""
    pod = dict(pod)
    if status is not None:
        pod["status"] = status
    meta = dict(pod["metadata"], resourceVersion="17")
    if deletion is not None:
        meta["deletionTimestamp"] = deletion
    if escaped:
        meta["name"] = 'p\\"1'
    pod["metadata"] = meta
    line = json.dumps({"type": typ, "object": pod}, indent=2 if pretty else None).replace("\n", " ")
    want = K.flat_identity(line)
    got = K.scan_identity(line)
    if escaped:
        assert got is None
    else:
        assert got[:3] == want and got[3] is False
        assert json.loads(got[1]) == pod
    # the transport's mode: only echoes and deletions are scanned, any other type stops at
    # the type member (the line then goes to the full parser). A deletion is scanned to its
    # metadata only; the rest of its identity (scheduler, node, phase) is filled on first use
    # and equals the full scan's
    md = K.scan_identity(line, True)
    if typ in ("MODIFIED", "DELETED") and not escaped:
        assert md[:3] == got[:3] and md[3] == (typ == "DELETED")
    else:
        assert md == (got if typ in ("MODIFIED", "DELETED") else None)


def test_flat_projection_rejects_malformed_json_like_the_dom():
    for bad in ['{"metadata": {"name": "p"}', '{"a": tru}', '{"a": "x\\q"}', '[1, 2,]', '{"a": 01}', '"\x01"']:
        with pytest.raises(ValueError):
            K.project_flat(bad)
        with pytest.raises(ValueError):
            K.project(bad)


def test_projection_hash_ignores_volatile_metadata_and_status():
    base = {"metadata": {"name": "p", "resourceVersion": "1", "labels": {"a": "b"}},
            "spec": {"containers": [{"name": "c"}]}, "status": {"phase": "Pending"}}
    h0 = K.project(json.dumps(base)).hash
    moved = json.loads(json.dumps(base))
    moved["metadata"]["resourceVersion"] = "9"
    moved["metadata"]["managedFields"] = [{"x": 1}]
    moved["status"] = {"phase": "Pending", "conditions": [{"type": "PodScheduled", "status": "False"}]}
    assert K.project(json.dumps(moved)).hash == h0
    relabel = json.loads(json.dumps(base))
    relabel["metadata"]["labels"] = {"a": "c"}
    assert K.project(json.dumps(relabel)).hash != h0


def test_projection_covers_extended_resources():
    """Extended resources are projected natively (the native NodeResourcesFit reads them), so
    such pods no longer fall back to a Python decode of the object."""
    pod = {"metadata": {"name": "p"}, "spec": {"containers": [{"name": "c", "resources": {"requests": {
        "amd.com/gpu": "2", "cpu": "1", "ephemeral-storage": "1Gi"}}}]}}
    ev = K.project(json.dumps(pod))
    assert ev.ok and ev.info_args() is not None
    pi = PodInfo.from_native(ev)
    assert pi.ext == {"amd.com/gpu": 2, "ephemeral-storage": 1 << 30} and pi.cpu_m == 1000
    assert pi.flags & 64                                 # PF_EXTENDED


# ============================================================== native fake apiserver
from yoda_scheduler_amd.testing import NativeApiServerProcess as NativeApi  # noqa: E402


@pytest.fixture
def native_api():
    a = NativeApi(history=50)
    yield a
    a.stop()


def test_native_apiserver_crud_watch_bind_and_selectors(native_api):
    async def go():
        cl = KubeClient(KubeConfig(native_api.url), native=True)
        try:
            await cl.create("nodes", make_node("n1"))
            with pytest.raises(ApiError) as ei:
                await cl.create("nodes", make_node("n1"))
            assert ei.value.code == 409
            _, rv = await cl.list("nodes")
            got = []

            async def watcher():
                async for typ, obj in cl.watch("pods", rv, field_selector="spec.nodeName="):
                    got.append((typ, obj["metadata"]["name"]))
                    if len(got) == 2:
                        return
            t = asyncio.get_event_loop().create_task(watcher())
            await asyncio.sleep(0.05)
            p = await cl.create("pods", {"metadata": {"name": "p"}, "spec": {"schedulerName": "x"}})
            assert p["metadata"]["namespace"] == "default" and p["metadata"]["uid"]
            with pytest.raises(ApiError) as ei:
                await cl.bind("default", "p", "wrong-uid", "n1")
            assert ei.value.code == 409
            await cl.bind("default", "p", p["metadata"]["uid"], "n1", {"scv.amd.com/gpus": "0"})
            await asyncio.wait_for(t, 5)
            # leaving the selector (bound) reaches a field-selected watch as DELETED
            assert got == [("ADDED", "p"), ("DELETED", "p")]
            pod = await cl.get("pods", "p", "default")
            assert pod["spec"]["nodeName"] == "n1" and pod["metadata"]["annotations"] == {"scv.amd.com/gpus": "0"}
            assert [c["type"] for c in pod["status"]["conditions"]] == ["PodScheduled"]
            with pytest.raises(ApiError) as ei:
                await cl.bind("default", "p", p["metadata"]["uid"], "n1")
            assert ei.value.code == 409
            stale = dict(pod, metadata=dict(pod["metadata"], resourceVersion="1"))
            with pytest.raises(ApiError) as ei:
                await cl.update("pods", stale, "default")
            assert ei.value.code == 409
            upd = await cl.update_status("pods", dict(pod, status={"phase": "Running"}), "default")
            assert upd["status"] == {"phase": "Running"} and upd["spec"]["nodeName"] == "n1"
            pt = await cl.patch("pods", "p", {"metadata": {"labels": {"a": "b"}, "uid": "hijack"}}, "default")
            assert pt["metadata"]["labels"] == {"a": "b"} and pt["metadata"]["uid"] == p["metadata"]["uid"]
            sel, _ = await cl.list("pods", field_selector="status.phase!=Running")
            assert sel == []
            await cl.delete("pods", "p", "default")
            with pytest.raises(ApiError) as ei:
                await cl.get("pods", "p", "default")
            assert ei.value.code == 404
            scv = await cl.create("scvs", make_scv("n1").to_json())
            assert scv["kind"] == "Scv" and scv["apiVersion"] == "core.run-linux.com/v1"
        finally:
            await cl.close()
    run(go())


def test_native_apiserver_bind_and_delete_edit_the_stored_text(native_api):
    """The fake apiserver binds and deletes pods by editing the stored JSON text (no DOM copy):
    the Binding's annotations merge into existing ones (same key replaced), other conditions
    survive while PodScheduled is replaced, status/spec members the edit does not touch stay,
    a field selector on an untouched path keeps matching through bind and delete, and every
    version carries its own resourceVersion."""
    async def go():
        cl = KubeClient(KubeConfig(native_api.url), native=True)
        try:
            await cl.create("nodes", make_node("n1"))
            _, rv = await cl.list("pods")
            got = []

            async def watcher():
                async for typ, obj in cl.watch("pods", rv, field_selector="status.phase!=Succeeded"):
                    got.append((typ, obj["metadata"]["resourceVersion"], obj["spec"].get("nodeName")))
                    if len(got) == 3:
                        return
            t = asyncio.get_event_loop().create_task(watcher())
            await asyncio.sleep(0.05)
            p = await cl.create("pods", {
                "metadata": {"name": "q", "annotations": {"keep": "1", "scv.amd.com/gpus": "old"}},
                "spec": {"schedulerName": "x", "nodeName": ""},
                "status": {"phase": "Pending", "conditions": [
                    {"type": "Initialized", "status": "True"},
                    {"type": "PodScheduled", "status": "False", "reason": "Unschedulable"}]}})
            await cl.bind("default", "q", p["metadata"]["uid"], "n1",
                          {"scv.amd.com/gpus": "0,1", "scv.amd.com/reserved-mb": "512"})
            pod = await cl.get("pods", "q", "default")
            assert pod["spec"] == {"schedulerName": "x", "nodeName": "n1"}
            assert pod["metadata"]["annotations"] == {"keep": "1", "scv.amd.com/gpus": "0,1",
                                                     "scv.amd.com/reserved-mb": "512"}
            conds = pod["status"]["conditions"]
            assert [c["type"] for c in conds] == ["Initialized", "PodScheduled"] and conds[1]["status"] == "True"
            assert pod["status"]["phase"] == "Pending"
            assert int(pod["metadata"]["resourceVersion"]) > int(p["metadata"]["resourceVersion"])
            await cl.delete("pods", "q", "default")
            await asyncio.wait_for(t, 5)
            assert [g[0] for g in got] == ["ADDED", "MODIFIED", "DELETED"]
            rvs = [int(g[1]) for g in got]
            assert rvs == sorted(rvs) and len(set(rvs)) == 3 and got[1][2] == "n1" and got[2][2] == "n1"
        finally:
            await cl.close()
    run(go())


def test_transport_bind_many_routes_each_answer_to_its_callback(native_api):
    """A run of Bindings handed over in one call: each pod gets its own answer (201 for the
    good ones, 409 for a wrong uid) through its own callback, with its annotations applied."""
    async def go():
        cl = KubeClient(KubeConfig(native_api.url), native=True)
        try:
            await cl.create("nodes", make_node("n1"))
            uids = []
            for k in range(5):
                p = await cl.create("pods", {"metadata": {"name": f"p{k}"}, "spec": {"schedulerName": "x"}})
                uids.append(p["metadata"]["uid"])
            uids[3] = "wrong-uid"
            loop = asyncio.get_event_loop()
            futs = [loop.create_future() for _ in uids]
            binds = [("default", f"p{k}", u, "n1", [("scv.amd.com/gpus", str(k))]) for k, u in enumerate(uids)]
            cbs = [(lambda f: (lambda st, body: f.set_result((st, body))))(f) for f in futs]
            cl.native.bind_many(binds, cbs, 5.0)
            got = await asyncio.wait_for(asyncio.gather(*futs), 5)
            assert [st for st, _ in got] == [201, 201, 201, 409, 201]
            for k in (0, 4):
                pod = await cl.get("pods", f"p{k}", "default")
                assert pod["spec"]["nodeName"] == "n1"
                assert pod["metadata"]["annotations"] == {"scv.amd.com/gpus": str(k)}
            cl.native.bind_many([], [], 5.0)          # nothing to hand over: no-op
        finally:
            await cl.close()
    run(go())


def test_native_apiserver_paging_history_410_and_bookmarks(native_api):
    async def go():
        cl = KubeClient(KubeConfig(native_api.url), native=True)
        try:
            for i in range(7):
                await cl.create("nodes", make_node(f"n{i}"))
            pages = []
            async for items, rv in cl.list_pages("nodes", resource_version="", limit=3):
                pages.append([i["metadata"]["name"] for i in items])
            assert [len(p) for p in pages] == [3, 3, 1] and sum(pages, []) == sorted(f"n{i}" for i in range(7))
            for i in range(60):                         # history is 50 events: RV 1 is compacted
                await cl.patch("nodes", "n0", {"metadata": {"labels": {"i": str(i)}}})
            with pytest.raises(ApiError) as ei:
                async for _ in cl.watch("nodes", "1"):
                    pass
            assert ei.value.code == 410
            # bookmarks advance the RV without an object
            _, rv = await cl.list("nodes")
            seen = []

            async def watcher():
                async for typ, obj in cl.watch("nodes", rv):
                    seen.append((typ, obj["metadata"]["resourceVersion"]))
                    return
            t = asyncio.get_event_loop().create_task(watcher())
            await asyncio.sleep(0.05)
            st, _ = await cl.native.request("GET", "/debug/bookmark?resource=nodes")
            assert st == 200
            await asyncio.wait_for(t, 5)
            assert seen == [("BOOKMARK", rv)]
        finally:
            await cl.close()
    run(go())


def test_native_apiserver_token_auth_and_client_rotation(tmp_path):
    api = NativeApi(token="tok-2")
    tf = tmp_path / "token"
    tf.write_text("tok-1")

    async def go():
        cfg = KubeConfig(api.url, token="tok-1", token_file=str(tf))
        cl = KubeClient(cfg, native=True)
        try:
            # the file still holds the old token: 401 → re-read → still 401 → error
            with pytest.raises(ApiError) as ei:
                await cl.list("nodes")
            assert ei.value.code == 401
            tf.write_text("tok-2")                         # the kubelet rotated the projected token
            items, _ = await cl.list("nodes")              # 401 → forced re-read → retry succeeds
            assert items == [] and cl.retried_401 >= 2
            await cl.create("nodes", make_node("n1"))
        finally:
            await cl.close()
    try:
        run(go())
    finally:
        api.stop()


# ============================================================== transport
def test_transport_rate_limit_timeouts_and_refused_connection():
    async def go():
        srv = FakeApiServer()
        srv.faults.latency_s = 0.0
        api = FakeApiHttp(srv)
        url = await api.start()
        cl = KubeClient(KubeConfig(url), native=True)
        try:
            await cl.create("nodes", make_node("n1"))
            cl.set_rate(20.0, 1)                           # 20 QPS, burst 1
            t0 = time.perf_counter()
            res = await asyncio.gather(*(cl.native.request("GET", "/api/v1/nodes", limited=True) for _ in range(6)))
            dt = time.perf_counter() - t0
            assert all(s == 200 for s, _ in res)
            assert dt >= 0.2, dt                           # 5 waits of 50 ms
            cl.set_rate(0, 0)
            st = cl.native.stats()
            assert st["throttled"] >= 5 and st["errors"] == 0
        finally:
            await cl.close()
            await api.stop()
        # nothing listens: the request fails with a connection error, not a hang. The port is
        # held bound (not listening) so a parallel test cannot start a server on it.
        import socket
        hold = socket.socket()
        hold.bind(("127.0.0.1", 0))
        dead = KubeClient(KubeConfig(f"http://127.0.0.1:{hold.getsockname()[1]}"), native=True, timeout=2.0)
        try:
            with pytest.raises((ConnectionError, asyncio.TimeoutError)):
                await dead.get("nodes", "n1")
        finally:
            await dead.close()
            hold.close()
    run(go())


def test_transport_request_timeout_against_silent_server():
    """A server that accepts and never answers: the request fails with a timeout (-2 →
    asyncio.TimeoutError) after its deadline instead of hanging the caller."""
    import socket

    async def go():
        ls = socket.socket()
        ls.bind(("127.0.0.1", 0))
        ls.listen(8)
        port = ls.getsockname()[1]
        t = nat.NativeTransport(KubeConfig(f"http://127.0.0.1:{port}"), conns=1)
        try:
            t0 = time.perf_counter()
            st, body = await t.request("GET", "/api/v1/nodes", timeout=0.2)
            dt = time.perf_counter() - t0
            assert st == -2 and b"timed out" in body and 0.15 <= dt < 2.0
            assert isinstance(nat.api_error(st, body), asyncio.TimeoutError)
            assert t.stats()["timeouts"] == 1
        finally:
            t.close()
            ls.close()
    run(go())


def test_transport_closes_connection_when_oldest_request_times_out():
    """a black-holed connection must not keep its pool slot. The oldest request
    times out (-2); everything pipelined behind it fails at once (-1, connection closed)
    instead of each waiting out its own deadline, and the connection is reopened."""
    import socket

    async def go():
        ls = socket.socket()
        ls.bind(("127.0.0.1", 0))
        ls.listen(8)
        port = ls.getsockname()[1]
        t = nat.NativeTransport(KubeConfig(f"http://127.0.0.1:{port}"), conns=1, max_inflight=8)
        try:
            t0 = time.perf_counter()
            first = asyncio.ensure_future(t.request("GET", "/api/v1/nodes", timeout=0.2))
            await asyncio.sleep(0.02)
            later = [asyncio.ensure_future(t.request("GET", "/api/v1/nodes", timeout=30.0)) for _ in range(3)]
            st0, _ = await first
            rest = await asyncio.wait_for(asyncio.gather(*later), 5.0)
            dt = time.perf_counter() - t0
            assert st0 == -2
            assert all(st == -1 and b"timed out" in body for st, body in rest), rest
            assert dt < 2.0                                   # not the 30 s deadlines
            conns0 = t.stats()["connects"]
            st2, _ = await t.request("GET", "/api/v1/nodes", timeout=0.1)
            assert st2 == -2 and t.stats()["connects"] == conns0 + 1    # a fresh connection
        finally:
            t.close()
            ls.close()
    run(go())


def test_native_watch_idle_timeout_ends_a_silent_stream():
    """A watch on a connection that delivers nothing ends after its idle timeout (status -1)
    so the reflector re-watches, instead of waiting forever for the server's own end."""
    import socket

    async def go():
        ls = socket.socket()
        ls.bind(("127.0.0.1", 0))
        ls.listen(8)
        port = ls.getsockname()[1]
        t = nat.NativeTransport(KubeConfig(f"http://127.0.0.1:{port}"), conns=1)
        done = asyncio.get_event_loop().create_future()
        try:
            t0 = time.perf_counter()
            t.watch("/api/v1/pods?watch=1", True, lambda evs: None,
                    lambda st, body: done.done() or done.set_result((st, body)), idle_timeout=0.3)
            st, body = await asyncio.wait_for(done, 5.0)
            assert st == -1 and b"idle" in body and time.perf_counter() - t0 >= 0.25
        finally:
            t.close()
            ls.close()
    run(go())


# ============================================================== reflector robustness
def test_informer_handler_exception_is_isolated_no_relist():
    from yoda_scheduler_amd.fakeapi.client import InProcessClient
    from yoda_scheduler_amd.kube.informer import Informer

    async def go():
        srv = FakeApiServer()
        seen = []

        def on_add(o):
            seen.append(o["metadata"]["name"])
            if o["metadata"]["name"] == "bad":
                raise RuntimeError("handler bug")
        inf = Informer(InProcessClient(srv), "nodes", on_add=on_add)
        task = asyncio.get_event_loop().create_task(inf.run())
        await asyncio.wait_for(inf.synced.wait(), 5)
        lists0 = srv.calls["list"]
        for n in ("a", "bad", "c"):
            srv.create("nodes", make_node(n))
        for _ in range(200):
            if len(seen) == 3:
                break
            await asyncio.sleep(0.005)
        await asyncio.sleep(0.05)
        inf.stop()
        srv.close_watches()
        task.cancel()
        await asyncio.gather(task, return_exceptions=True)
        return seen, inf.handler_errors, srv.calls["list"] - lists0, sorted(inf.store)
    seen, errs, relists, store = run(go())
    assert seen == ["a", "bad", "c"] and errs == 1
    assert relists == 0 and store == ["a", "bad", "c"]


def test_informer_backoff_bounds_requests_while_apiserver_down():
    from yoda_scheduler_amd.kube.informer import Backoff, Informer

    class Down:
        def __init__(self):
            self.calls = 0

        async def list(self, *a, **k):
            self.calls += 1
            raise ConnectionError("connection refused")

    async def go():
        c = Down()
        inf = Informer(c, "nodes", relist_backoff=0.01, max_backoff=0.08)
        task = asyncio.get_event_loop().create_task(inf.run())
        await asyncio.sleep(0.6)
        inf.stop()
        task.cancel()
        await asyncio.gather(task, return_exceptions=True)
        return c.calls
    calls = run(go())
    # 0.01, 0.02, 0.04, 0.08, 0.08, ... each stretched by up to 2× jitter: ≤ 12 in 0.6 s
    # (a fixed 0.01 s retry would be ~60)
    assert 3 <= calls <= 12, calls
    b = Backoff(1.0, 8.0, jitter=0.0, reset_after=1e9)
    assert [b.next() for _ in range(5)] == [1.0, 2.0, 4.0, 8.0, 8.0]
    b.reset()
    assert b.next() == 1.0


# ============================================================== scheduler over the native stack
@pytest.mark.parametrize("server,lane", [("native", "on"), ("python", "on"), ("native", "off")])
def test_scheduler_binds_over_native_transport(server, lane):
    from yoda_scheduler_amd.framework.config import parse_config
    from yoda_scheduler_amd.framework.scheduler import Scheduler
    from yoda_scheduler_amd.kube.informer import NativePodInformer
    from yoda_scheduler_amd.testing import yoda_config

    async def go():
        api = NativeApi() if server == "native" else None
        papi = None
        if api is None:
            papi = FakeApiHttp(FakeApiServer())
            url = await papi.start()
        else:
            url = api.url
        cl = KubeClient(KubeConfig(url), native=True)
        try:
            await cl.create("nodes", make_node("n1"))
            s = make_scv("n1", update_time=time.time())
            s.update_interval_ms = 600_000
            await cl.create("scvs", s.to_json())
            cfg = yoda_config()
            cfg["yodaRuntime"]["nativeLane"] = lane
            sched = Scheduler(cl, parse_config(cfg))
            assert isinstance(sched.make_informers()["pods"], NativePodInformer)
            assert (sched.lane is not None) == (lane == "on")
            await sched.start()
            loop_t = asyncio.get_event_loop().create_task(sched.scheduling_loop())
            for i in range(30):
                await cl.create("pods", {"metadata": {"name": f"p{i}", "labels": {"scv/memory": "1000",
                                                                                   "scv/number": str(1 + i % 2)}},
                                         "spec": {"schedulerName": "yoda-scheduler",
                                                  "tolerations": [{"key": "node.kubernetes.io/not-ready",
                                                                   "operator": "Exists", "effect": "NoExecute"}]}})
            t0 = time.time()
            while sched.scheduled < 30 and time.time() - t0 < 10:
                await asyncio.sleep(0.01)
            items, _ = await cl.list("pods")
            cards = {i["metadata"]["name"]: i["metadata"].get("annotations", {}).get("scv.amd.com/gpus")
                     for i in items}
            # the bind echo confirmed every assumed pod; the lazy store decodes on demand
            await asyncio.sleep(0.1)
            assumed = [p for p in sched.cache.pods.values() if p.assumed]
            stored = sched.informers["pods"].store.get("default/p3")
            await cl.delete("pods", "p3", "default")
            await asyncio.sleep(0.1)
            gone = "default/p3" in sched.informers["pods"].store
            await sched.shutdown()
            loop_t.cancel()
            return sched.scheduled, cards, assumed, stored, gone
        finally:
            await cl.close()
            if api:
                api.stop()
            if papi:
                await papi.stop()
    n, cards, assumed, stored, gone = run(go())
    assert n == 30 and all(cards.values()) and not assumed and not gone
    assert len(cards["p1"].split(",")) == 2 and len(cards["p0"].split(",")) == 1
    assert stored["spec"]["nodeName"] == "n1"


def test_bounded_drain_keeps_order_and_yields_between_chunks():
    """NativeTransport dispatches at most DRAIN_BUDGET watch events per loop turn: a large
    event batch is split, the rest stays first in line, completions queued behind it run
    after it, and a continuation is scheduled with call_soon so other tasks (the scheduling
    loop) run between chunks."""
    class FakeT:
        def __init__(self, items):
            self.items = items

        def drain(self):
            out, self.items = self.items, []
            return out

    tr = nat.NativeTransport.__new__(nat.NativeTransport)
    tr._cbs, tr._watches, tr.callback_errors = {}, {}, 0
    import collections
    tr._backlog, tr._continue_pending = collections.deque(), False
    seen: list = []
    tr._watches[7] = nat.WatchHandle(7, lambda evs: seen.append(("ev", [e[1] for e in evs])),
                                     lambda st, b: seen.append(("end", st)))
    tr._cbs[3] = lambda st, body: seen.append(("bind", st))
    big = [("ADDED", str(i), None) for i in range(1200)]
    tr.t = FakeT([(1, 7, big), (0, 3, 201, b""), (1, 7, [("MODIFIED", "x", None)]), (2, 7, 200, b"")])

    async def go():
        tr._loop = asyncio.get_event_loop()
        other = []

        async def scheduler_like():
            for _ in range(5):
                other.append(len([s for s in seen if s[0] == "ev"]))
                await asyncio.sleep(0)
        task = asyncio.ensure_future(scheduler_like())
        tr._drain()
        for _ in range(10):
            await asyncio.sleep(0)
        await task
        return other
    other = asyncio.run(go())
    evs = [x for kind, v in seen if kind == "ev" for x in v]
    assert evs == [str(i) for i in range(1200)] + ["x"]          # order kept across splits
    chunks = [len(v) for kind, v in seen if kind == "ev"]
    assert chunks[:3] == [512, 512, 176] and max(chunks) <= nat.NativeTransport.DRAIN_BUDGET
    kinds = [k for k, _ in seen]
    assert kinds.index("bind") > 2 and kinds[-1] == "end"         # completion after the big batch
    assert other[0] >= 1 and other[-1] <= len(chunks)             # the other task ran between chunks


def test_failed_bind_handoff_requeues_the_run():
    """If handing a run's Bindings to the transport raises, every pod of the run takes the
    bind-failure path (forgotten, retried from backoff) instead of staying assumed; once the
    transport accepts again they bind. (The Python runner's path: native lane off.)"""
    from yoda_scheduler_amd.framework.config import parse_config
    from yoda_scheduler_amd.framework.scheduler import Scheduler
    from yoda_scheduler_amd.testing import yoda_config

    async def go():
        api = NativeApi()
        cl = KubeClient(KubeConfig(api.url), native=True)
        try:
            await cl.create("nodes", make_node("n1"))
            s = make_scv("n1", update_time=time.time())
            s.update_interval_ms = 600_000
            await cl.create("scvs", s.to_json())
            cfg = parse_config(yoda_config())
            cfg.pod_initial_backoff_seconds = 0.01
            cfg.native_lane = "off"
            sched = Scheduler(cl, cfg)
            await sched.start()
            orig, calls = cl.native.bind_many, []

            def flaky(binds, cbs, timeout=0.0):
                calls.append(len(binds))
                if len(calls) == 1:
                    raise RuntimeError("transport refused the run")
                return orig(binds, cbs, timeout)
            cl.native.bind_many = flaky
            for i in range(12):
                await cl.create("pods", {"metadata": {"name": f"f{i}", "labels": {"scv/memory": "1000"}},
                                         "spec": {"schedulerName": "yoda-scheduler",
                                                  "tolerations": [{"key": "node.kubernetes.io/not-ready",
                                                                   "operator": "Exists", "effect": "NoExecute"}]}})
            t0 = time.time()
            while len(sched.queue._active_entries) < 12 and time.time() - t0 < 5:
                await asyncio.sleep(0.01)         # the burst is queued: the loop takes it as one run
            loop_t = asyncio.get_event_loop().create_task(sched.scheduling_loop())
            t0 = time.time()
            while sched.scheduled < 12 and time.time() - t0 < 15:
                sched.queue.flush_backoff_completed()
                await asyncio.sleep(0.02)
            out = sched.scheduled, sched.bind_errors, len(calls), sched.pending_binds
            await sched.shutdown()
            loop_t.cancel()
            return out
        finally:
            await cl.close()
            api.stop()
    scheduled, errors, calls, pending = run(go())
    assert scheduled == 12 and errors >= 1 and calls >= 2 and pending == 0, (scheduled, errors, calls, pending)


def test_native_apiserver_bench_burst_and_reset_run_in_slices(native_api):
    """The bench endpoints answer at once and create / delete in 64-pod slices between event
    loop turns, so other requests (a Binding here) are served while a burst is being created;
    a watch sees every pod ADDED, the bound one MODIFIED and every pod DELETED after the reset,
    and the status endpoint's latencies cover the bound pods."""
    import aiohttp

    from yoda_scheduler_amd.bench.workloads import pod_object

    async def go():
        cl = KubeClient(KubeConfig(native_api.url), native=True)
        http = aiohttp.ClientSession()
        try:
            await cl.create("nodes", make_node("n1"))
            _, rv = await cl.list("pods")
            n = 640
            async with http.post(native_api.url + "/debug/bench/load",
                                 json={"pods": [pod_object(i, {"scv/memory": "1"}, "x") for i in range(n)]}) as r:
                assert (await r.json())["n"] == n
            seen = {"ADDED": 0, "MODIFIED": 0, "DELETED": 0}

            async def watcher():
                async for typ, _obj in cl.watch("pods", rv):
                    seen[typ] += 1
                    if seen["DELETED"] == n:
                        return
            t = asyncio.get_event_loop().create_task(watcher())
            await asyncio.sleep(0.05)
            async with http.post(native_api.url + "/debug/bench/burst", json={"tag": "s"}) as r:
                assert (await r.json())["n"] == n
            for _ in range(500):                          # the first slice is there soon
                try:
                    p = await cl.get("pods", "s-0", "default")
                    break
                except ApiError:
                    await asyncio.sleep(0.002)
            await cl.bind("default", "s-0", p["metadata"]["uid"], "n1")
            for _ in range(500):
                async with http.get(native_api.url + "/debug/bench/status?full=1") as r:
                    st = await r.json()
                if st["created"] == n:
                    break
                await asyncio.sleep(0.005)
            assert st["created"] == n and st["bound"] == 1 and len(st["latencies"]) == 1
            async with http.post(native_api.url + "/debug/bench/reset") as r:
                assert (await r.json())["deleted"] == n
            await asyncio.wait_for(t, 10)
            assert seen == {"ADDED": n, "MODIFIED": 1, "DELETED": n}
            items, _ = await cl.list("pods")
            assert items == []
        finally:
            await http.close()
            await cl.close()
    run(go())


def test_labels_hash_agrees_across_scanner_and_projections():
    """The watch identity scanner's labels hash equals the full projections' (flat and DOM), so
    the lane's selector census can keep a bound pod's projected labels across light echo events
    until a label actually changes (then the hashes differ)."""
    import json
    from yoda_scheduler_amd._native import _yoda_kube as k
    base = {"metadata": {"name": "p", "namespace": "ns", "uid": "u1", "resourceVersion": "7",
                         "labels": {"app": "web", "tier": 'a"b'}},
            "spec": {"nodeName": "n1", "containers": [{"name": "c"}]}, "status": {"phase": "Running"}}
    hashes = []
    # escaped value (parser path), plain strings (hashed from the text), none, empty, raw UTF-8,
    # several members, an empty value, a non-string value (parser path), compact separators
    cases = [({"app": "web", "tier": 'a"b'}, True), ({"app": "web", "tier": "x"}, True), (None, True), ({}, True),
             ({"app": "wéb"}, False), ({"a": "1", "b": "", "c.d/e": "x-y_z"}, True), ({"n": 5}, True),
             ({"app": "web", "tier": "x"}, "compact")]
    for labels, ascii_ in cases:
        obj = json.loads(json.dumps(base))
        if labels is None:
            obj["metadata"].pop("labels")
        else:
            obj["metadata"]["labels"] = labels
        sep = (",", ":") if ascii_ == "compact" else None
        raw = json.dumps(obj, ensure_ascii=bool(ascii_), separators=sep)
        line = json.dumps({"type": "MODIFIED", "object": obj}, ensure_ascii=bool(ascii_), separators=sep)
        h_scan = k.scan_labels_hash(line)
        assert h_scan == k.project_flat(raw).labels_hash == k.project(raw).labels_hash != 0, labels
        hashes.append(h_scan)
    # the same labels hash alike whatever the whitespace; different labels differ
    assert hashes[1] == hashes[-1] and len(set(hashes)) == len(cases) - 1


@settings(max_examples=200, deadline=None)
@given(st.lists(st.one_of(
    st.builds(lambda c: {"name": "v", "persistentVolumeClaim": {"claimName": c}},
              st.one_of(st.text(min_size=0, max_size=6), st.integers(0, 3), st.none())),
    st.just({"name": "v", "persistentVolumeClaim": {}}),
    st.builds(lambda n: {"name": n, "ephemeral": {"volumeClaimTemplate": {}}}, st.text(min_size=0, max_size=6)),
    st.just({"ephemeral": {}}),
    st.just({"name": "t", "emptyDir": {}}),
    st.just({"name": "d", "gcePersistentDisk": {"pdName": "x"}})), max_size=4),
    st.text(min_size=1, max_size=5))
def test_projected_claims_equal_the_volume_plugins_claim_names(vols, pod_name):
    """The lane admits PVC pods by their claim names (``PodEvent.claims``): equal to
    plugins/volumes.py::_claim_names for string names; a non-string name becomes a sentinel no
    PersistentVolumeClaim key can equal."""
    from yoda_scheduler_amd.plugins.volumes import _claim_names
    obj = {"metadata": {"name": pod_name, "namespace": "default", "uid": "u"},
           "spec": {"schedulerName": "s", "containers": [{"name": "c", "image": "x"}], "volumes": vols}}
    ev = K.project_flat(json.dumps(obj))
    assert ev.ok
    want = _claim_names(PodInfo.from_obj(obj))
    assert len(ev.claims) == len(want)
    for got, w in zip(ev.claims, want):
        assert got == w if isinstance(w, str) else got == "\x01"


@settings(max_examples=150, deadline=None)
@given(_pod, st.sampled_from([{}, {"phase": "Pending"}]))
def test_lazy_hash_of_a_lane_decoded_pod_equals_the_eager_one(pod, status):
    """With a native lane attached the watch stream decodes ADDED pods without the spec /
    metadata hash (only Python's update check of a forwarded pod, or the lane's of a queued one,
    compares it); ``PodEvent.hash`` computes it from the raw object on first use — equal to the
    eager projection's, and every other field is the same."""
    pod = dict(pod, status=status)
    raw = json.dumps(pod)
    lazy, eager = K.project_flat_nohash(raw), K.project(raw)
    assert lazy.info_args() == eager.info_args() and lazy.flags == eager.flags
    assert lazy.hash == eager.hash and lazy.ident() == eager.ident()
