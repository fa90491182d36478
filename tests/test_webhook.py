"""Admission webhook for the scv label API: validation rules, the
scheduler-name mutation, and AdmissionReview round trips over HTTPS like the apiserver
makes them."""
import asyncio
import base64
import json
import shutil
import ssl
import subprocess

import pytest

from yoda_scheduler_amd.webhook.admission import AdmissionPolicy, apply_add_ops, review, validate_labels


def ar(labels, scheduler=None, op="CREATE", uid="u1"):
    spec = {"containers": [{"name": "c", "image": "x"}]}
    if scheduler is not None:
        spec["schedulerName"] = scheduler
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
            "request": {"uid": uid, "kind": {"group": "", "version": "v1", "kind": "Pod"}, "operation": op,
                        "name": "p", "namespace": "default",
                        "object": {"metadata": {"name": "p", "labels": labels}, "spec": spec}}}


def test_validation_rules():
    ok, warn = validate_labels({"scv/number": "2", "scv/memory": "1000", "scv/clock": "2400", "scv/priority": "-3",
                                "scv.amd.com/clock-min": "2100", "scv.amd.com/gang": "numa", "app": "x"})
    assert ok == [] and warn == []
    bad, _ = validate_labels({"scv/number": "abc"})           # reference: Atoi error → 0 → fits everywhere (Q5)
    assert "non-negative decimal integer" in bad[0]
    assert validate_labels({"scv/number": "-1"})[0]            # reference: wraps to 2^64-1
    assert validate_labels({"scv/number": "0"})[0]
    assert validate_labels({"scv/number": "65"})[0]
    assert validate_labels({"scv/memory": str(288 * 1024 + 1)})[0]
    assert validate_labels({"scv/memory": "+5"})[0]
    assert validate_labels({"scv/priority": "high"})[0]
    assert validate_labels({"scv.amd.com/gang": "ring"})[0]
    assert validate_labels({"scv/memory": "1000"}, AdmissionPolicy(max_memory_mb=500))[0]
    _, warn = validate_labels({"scv/memroy": "1000"})
    assert warn and "scv/memroy" in warn[0]


def test_review_validate_and_mutate():
    out = review(ar({"scv/number": "x"}), mutate=False)
    assert out["kind"] == "AdmissionReview" and out["response"]["uid"] == "u1"
    assert out["response"]["allowed"] is False and out["response"]["status"]["code"] == 422
    assert review(ar({"scv/memory": "1000"}), mutate=False)["response"]["allowed"] is True
    # mutate: scv pods left on the default scheduler go to the yoda profile
    m = review(ar({"scv/memory": "1000"}), mutate=True)["response"]
    assert m["allowed"] and m["patchType"] == "JSONPatch"
    ops = json.loads(base64.b64decode(m["patch"]))
    assert ops[0] == {"op": "add", "path": "/spec/schedulerName", "value": "yoda-scheduler"}
    assert [o["path"] for o in ops[1:]] == ["/spec/containers/0/env"]          # GPU pinning, below
    m = review(ar({"scv/memory": "1000"}, scheduler="default-scheduler"), mutate=True)["response"]
    assert json.loads(base64.b64decode(m["patch"]))[0]["op"] == "replace"
    # an explicit yoda profile keeps its name (only the GPU pinning is added); non-scv pods,
    # other schedulers and updates are left alone
    ops = json.loads(base64.b64decode(review(ar({"scv/memory": "1"}, scheduler="yoda-scheduler2"),
                                             mutate=True)["response"]["patch"]))
    assert [o["path"] for o in ops] == ["/spec/containers/0/env"]
    assert "patch" not in review(ar({"scv/memory": "1"}, scheduler="other"), mutate=True)["response"]
    assert "patch" not in review(ar({"app": "web"}), mutate=True)["response"]
    assert "patch" not in review(ar({"scv/memory": "1"}, op="UPDATE"), mutate=True)["response"]
    assert "patch" not in review(ar({"scv/memory": "1"}), mutate=True,
                                 policy=AdmissionPolicy(mutate_scheduler_name=False,
                                                        inject_visible_devices=False))["response"]


def test_visible_devices_injection():
    """Containers of yoda pods read the GPU assignment through the downward API; the
    Binding copies ``scv.amd.com/visible-devices`` (ROCr UUIDs) onto the pod before
    containers start. Only ROCR_VISIBLE_DEVICES is set: HIP_VISIBLE_DEVICES would index
    the already-filtered devices."""
    body = ar({"scv/number": "2"}, scheduler="yoda-scheduler")
    spec = body["request"]["object"]["spec"]
    spec["containers"].append({"name": "side", "image": "y", "env": [{"name": "A", "value": "1"}]})
    spec["containers"].append({"name": "own", "image": "z", "env": [{"name": "HIP_VISIBLE_DEVICES", "value": "3"}]})
    spec["initContainers"] = [{"name": "init", "image": "w"}]
    ops = json.loads(base64.b64decode(review(body, mutate=True)["response"]["patch"]))
    pod = apply_add_ops(body["request"]["object"], ops)
    ref = {"fieldRef": {"fieldPath": "metadata.annotations['scv.amd.com/visible-devices']"}}
    for c in (pod["spec"]["containers"][0], pod["spec"]["containers"][1], pod["spec"]["initContainers"][0]):
        env = {e["name"]: e.get("valueFrom") for e in c["env"]}
        assert env["ROCR_VISIBLE_DEVICES"] == ref and "HIP_VISIBLE_DEVICES" not in env
    assert pod["spec"]["containers"][1]["env"][0] == {"name": "A", "value": "1"}
    assert pod["spec"]["containers"][2]["env"] == [{"name": "HIP_VISIBLE_DEVICES", "value": "3"}]   # untouched
    # device-plugin pods and opted-out pods are left alone
    dp = ar({"scv/number": "1"}, scheduler="yoda-scheduler")
    dp["request"]["object"]["spec"]["containers"][0]["resources"] = {"limits": {"amd.com/gpu": "1"}}
    assert "patch" not in review(dp, mutate=True)["response"]
    out = ar({"scv/number": "1"}, scheduler="yoda-scheduler")
    out["request"]["object"]["metadata"]["annotations"] = {"scv.amd.com/inject-visible-devices": "false"}
    assert "patch" not in review(out, mutate=True)["response"]


def test_webhook_over_https(tmp_path):
    if not shutil.which("openssl"):
        pytest.skip("openssl not available")
    d = tmp_path
    sh = lambda *a: subprocess.run(a, check=True, capture_output=True)  # noqa: E731
    sh("openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "1", "-subj", "/CN=127.0.0.1",
       "-addext", "subjectAltName=IP:127.0.0.1", "-keyout", str(d / "tls.key"), "-out", str(d / "tls.crt"))
    from yoda_scheduler_amd.webhook.server import WebhookServer

    async def go():
        sctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        sctx.load_cert_chain(str(d / "tls.crt"), str(d / "tls.key"))
        srv = WebhookServer("127.0.0.1", 0, ssl_context=sctx)
        port = await srv.start()
        cctx = ssl.create_default_context(cafile=str(d / "tls.crt"))
        import aiohttp
        try:
            async with aiohttp.ClientSession() as s:
                async with s.post(f"https://127.0.0.1:{port}/validate", json=ar({"scv/number": "-1"}),
                                  ssl=cctx) as r:
                    rej = await r.json()
                async with s.post(f"https://127.0.0.1:{port}/mutate", json=ar({"scv/number": "2"}), ssl=cctx) as r:
                    mut = await r.json()
                async with s.get(f"https://127.0.0.1:{port}/healthz", ssl=cctx) as r:
                    health = await r.text()
        finally:
            await srv.stop()
        return rej, mut, health, srv.reviewed, srv.rejected
    rej, mut, health, reviewed, rejected = asyncio.run(go())
    assert rej["response"]["allowed"] is False and mut["response"]["allowed"] is True
    assert "patch" in mut["response"] and health == "ok" and (reviewed, rejected) == (2, 1)


def test_deploy_manifest_and_cli_entry():
    import os
    import yaml
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    docs = list(yaml.safe_load_all(open(os.path.join(root, "deploy", "yoda-webhook.yaml"))))
    kinds = [d["kind"] for d in docs]
    assert kinds == ["Deployment", "Service", "ValidatingWebhookConfiguration", "MutatingWebhookConfiguration"]
    paths = [w["clientConfig"]["service"]["path"] for d in docs[2:] for w in d["webhooks"]]
    assert paths == ["/validate", "/mutate"]
    from yoda_scheduler_amd.cmd.webhook import main
    with pytest.raises(SystemExit):
        main(["--help"])


def test_executor_resolves_downward_api_env():
    from yoda_scheduler_amd.sniffer.executor import resolve_env
    body = ar({"scv/number": "2"}, scheduler="yoda-scheduler")
    ops = json.loads(base64.b64decode(review(body, mutate=True)["response"]["patch"]))
    pod = apply_add_ops(body["request"]["object"], ops)
    pod["metadata"]["annotations"] = {"scv.amd.com/gpus": "3,5",                  # written by the Binding
                                      "scv.amd.com/visible-devices": "GPU-aa,GPU-bb"}
    pod["spec"]["containers"][0]["env"].append({"name": "NODE", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}})
    pod["spec"]["nodeName"] = "n7"
    env = resolve_env(pod, pod["spec"]["containers"][0])
    assert env == {"ROCR_VISIBLE_DEVICES": "GPU-aa,GPU-bb", "NODE": "n7"}
