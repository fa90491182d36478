"""GPU: SURVEY §7.2 minimum end-to-end slice on a real MI355X.

C++ amd-smi sniffer → Scv published → scheduler (native engine) binds a ``scv/memory``
pod with a GPU assignment annotation → executor starts a ROCm process pinned with
HIP_VISIBLE_DEVICES that allocates the pod's HBM → the next amd-smi sample shows the drop,
and the new Scv makes the scheduler see it (ledger pending → sampled)."""
import asyncio
import base64
import json
import time

import pytest

pytestmark = pytest.mark.gpu


def test_minimum_end_to_end_slice(require_gpu):
    from yoda_scheduler_amd.fakeapi.client import InProcessClient
    from yoda_scheduler_amd.fakeapi.server import FakeApiServer
    from yoda_scheduler_amd.framework.config import parse_config
    from yoda_scheduler_amd.framework.scheduler import Scheduler
    from yoda_scheduler_amd.models.device import make_node
    from yoda_scheduler_amd.models.scv import Scv
    from yoda_scheduler_amd.sniffer.collector import AmdSmiBackend
    from yoda_scheduler_amd.sniffer.executor import PodExecutor
    from yoda_scheduler_amd.sniffer.publisher import SnifferAgent
    from yoda_scheduler_amd.testing import yoda_config
    from yoda_scheduler_amd.webhook.admission import apply_add_ops, review

    MB = 4096

    async def go():
        srv = FakeApiServer()
        cl = InProcessClient(srv)
        srv.create("nodes", make_node("mi355x-0"))
        agent = SnifferAgent(cl, "mi355x-0", AmdSmiBackend(), interval=60.0)
        await agent.publish_once()
        before = Scv.from_json(srv.get("scvs", "mi355x-0"))
        sched = Scheduler(cl, parse_config(yoda_config(yoda_args={"sampleSettleSeconds": 0.0})))
        await sched.start()
        loop_t = asyncio.get_event_loop().create_task(sched.scheduling_loop())
        # admission first: the webhook points the pod at the yoda profile and pins its
        # containers to the assignment through the downward API
        obj = {"metadata": {"name": "slice", "namespace": "default", "labels": {"scv/memory": str(MB)}},
               "spec": {"containers": [{"name": "main", "image": "rocm/pytorch"}]}}
        resp = review({"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                       "request": {"uid": "u", "kind": {"kind": "Pod"}, "operation": "CREATE", "object": obj}},
                      mutate=True)["response"]
        obj = apply_add_ops(obj, json.loads(base64.b64decode(resp["patch"])))
        srv.create("pods", obj)
        for _ in range(2000):
            if srv.bind_log:
                break
            await asyncio.sleep(0.005)
        pod = srv.get("pods", "slice", "default")
        ex = PodExecutor(cl, "mi355x-0", hold_seconds=120)
        r = ex.launch(pod)
        ok = await ex.wait_allocated(r)
        try:
            await asyncio.sleep(0.5)
            await agent.publish_once()
            after = Scv.from_json(srv.get("scvs", "mi355x-0"))
            await asyncio.sleep(0.05)
            gpu_state = sched.cache.node_gpu_state("mi355x-0")
        finally:
            ex.stop_all()
            await sched.shutdown()
            loop_t.cancel()
        return pod, ok, r.log, before, after, gpu_state, ex.env_log["default/slice"]

    pod, ok, log, before, after, gpu_state, env = asyncio.run(go())
    gpus = [int(x) for x in pod["metadata"]["annotations"]["scv.amd.com/gpus"].split(",")]
    assert len(gpus) == 1
    assert pod["spec"]["schedulerName"] == "yoda-scheduler"
    # pinned by ROCr UUID through the downward API, and the workload really ran on the
    # GPU whose amd-smi BDF the scheduler reserved (the identity contract end to end)
    vis = pod["metadata"]["annotations"]["scv.amd.com/visible-devices"]
    assert env["ROCR_VISIBLE_DEVICES"] == vis and env.get("HIP_VISIBLE_DEVICES") is None
    assert ok, log
    bus = next(line for line in log if line.startswith("allocated")).split("pci_bus_ids=")[1].split(",")[0]
    assert int(bus) == int(before.status.card_list[gpus[0]].bdf.split(":")[1], 16), (bus, log)
    g = gpus[0]
    drop = before.status.card_list[g].free_memory - after.status.card_list[g].free_memory
    assert drop >= MB, (drop, log)                        # the sniffer saw the pod's HBM
    assert gpu_state[g]["reserved"] == MB and gpu_state[g]["pending"] == 0   # sample now reflects it
