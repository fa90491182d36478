"""Drop-in proof: the reference's own ConfigMap (``/root/reference/deploy/yoda-scheduler.yaml:1-31``,
copied verbatim to ``tests/fixtures/reference_scheduler_configmap.yaml``) drives the shipped
``yoda-scheduler`` binary unchanged: v1beta1, leader election on a Lease, PrioritySort
(the yoda QueueSort stays disabled), yoda at filter (weight 0) and score (weight 300)
only — no PostFilter — and no ``clientConnection`` (upstream QPS 50 / burst 100).

With two feasible GPU nodes the reference fails every Score (``"Max"`` is only written
in PostFilter); here the maxima come from PreScore, so pods bind."""
from __future__ import annotations

import asyncio
import os
import socket
import subprocess
import sys
import time

import yaml

from yoda_scheduler_amd.kube.client import KubeClient, KubeConfig
from yoda_scheduler_amd.models.device import make_node, make_scv
from yoda_scheduler_amd.testing import NativeApiServerProcess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "reference_scheduler_configmap.yaml")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_reference_configmap_verbatim_schedules_on_two_nodes(tmp_path):
    with open(FIXTURE) as f:
        cm = yaml.safe_load(f)
    assert cm["kind"] == "ConfigMap" and cm["metadata"]["name"] == "scheduler-config2"
    cfg_text = cm["data"]["scheduler-config.yaml"]
    cfg_path = tmp_path / "scheduler-config.yaml"
    cfg_path.write_text(cfg_text)                       # exactly the mounted file of the reference Deployment
    api = NativeApiServerProcess()
    kc = tmp_path / "kubeconfig"
    kc.write_text(yaml.safe_dump({
        "apiVersion": "v1", "kind": "Config", "current-context": "fake",
        "clusters": [{"name": "fake", "cluster": {"server": api.url}}],
        "contexts": [{"name": "fake", "context": {"cluster": "fake", "user": "u"}}],
        "users": [{"name": "u", "user": {}}]}))
    status_port = _free_port()
    proc = None

    async def go():
        nonlocal proc
        cl = KubeClient(KubeConfig(api.url))
        try:
            for n in ("gpu-a", "gpu-b"):
                await cl.create("nodes", make_node(n))
                s = make_scv(n, update_time=time.time())
                s.update_interval_ms = 600_000
                await cl.create("scvs", s.to_json())
            # the reference Deployment's args (deploy/yoda-scheduler.yaml:60-63) + a kubeconfig
            proc = subprocess.Popen([sys.executable, "-m", "yoda_scheduler_amd.cmd.scheduler",
                                     f"--config={cfg_path}", "--v=3", f"--kubeconfig={kc}",
                                     "--port", str(status_port), "--bind-address", "127.0.0.1"],
                                    env=dict(os.environ, PYTHONPATH=ROOT), stdout=subprocess.PIPE,
                                    stderr=subprocess.STDOUT, text=True)
            for i in range(6):
                await cl.create("pods", {"metadata": {"name": f"ref-{i}", "namespace": "default",
                                                      "labels": {"scv/memory": "1000", "scv/number": "1"}},
                                         "spec": {"schedulerName": "yoda-scheduler2",
                                                  "containers": [{"name": "c", "image": "rocm/pytorch"}]}})
            deadline = time.time() + 60
            nodes = {}
            while time.time() < deadline:
                items, _ = await cl.list("pods")
                nodes = {p["metadata"]["name"]: p["spec"].get("nodeName") for p in items}
                if all(nodes.values()):
                    break
                await asyncio.sleep(0.1)
            lease = await cl.get("leases", "yoda-scheduler", "kube-system")
            events, _ = await cl.list("events.k8s.io")
            return nodes, lease, events
        finally:
            await cl.close()

    try:
        nodes, lease, events = asyncio.run(go())
    finally:
        out = ""
        if proc is not None:
            proc.terminate()
            try:
                out, _ = proc.communicate(timeout=15)
            except subprocess.TimeoutExpired:
                proc.kill()
        api.stop()
    assert all(v in ("gpu-a", "gpu-b") for v in nodes.values()) and len(nodes) == 6, (nodes, out[-3000:])
    # the reference's leader-election settings took effect (Lease kube-system/yoda-scheduler)
    assert lease["spec"]["holderIdentity"], lease
    # both nodes were feasible and scored — the Q1 failure mode would show FailedScheduling
    reasons = [e.get("reason") for e in events]
    assert "Scheduled" in reasons and "FailedScheduling" not in reasons, reasons
