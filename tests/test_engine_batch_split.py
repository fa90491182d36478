"""Engine::schedule_batch splits a batch into k_batch dispatches around pods the device cannot
carry (VERDICT r5 next #3a), instead of sending the whole batch to per-pod cycles.

``native/core/fake_dev.cpp`` stands in for libyoda_hip.so: it records the size of every
``yoda_dev_schedule_batch`` call and refuses it, so the engine's CPU path still places every pod
(the placements are checked against a device-less engine with the same seed).
"""
import ctypes
import os
import subprocess

import pytest

from yoda_scheduler_amd.framework.cache import SchedulerCache
from yoda_scheduler_amd.models.device import make_node
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.ops.native import core, pod_req

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "native")
C = core()


@pytest.fixture(scope="module")
def fake_lib(tmp_path_factory):
    out = tmp_path_factory.mktemp("fakedev") / "libfake_dev.so"
    subprocess.run(["g++", "-std=c++17", "-O1", "-shared", "-fPIC", f"-I{NATIVE}/hip",
                    f"{NATIVE}/core/fake_dev.cpp", "-o", str(out)], check=True, timeout=120)
    return str(out)


def _cluster(n_nodes):
    from yoda_scheduler_amd.models.device import make_scv
    eng = C.Engine(False, 1)
    eng.seed(7)
    cache = SchedulerCache(eng)
    for i in range(n_nodes):
        cache.add_node(make_node(f"n{i}", labels={"pool": "a" if i % 2 else "b"}))
        cache.set_scv(make_scv(f"n{i}"))
    return eng, cache


def _pods():
    kinds = ["e", "e", "e", "x", "e", "e", "s", "e"]
    out = []
    for j, k in enumerate(kinds):
        spec = {"containers": [{"name": "c", "resources": {"requests": {"cpu": "1"}}}]}
        if k == "x":     # a node selector: the device needs a per-node candidate mask (per-pod cycle)
            spec["nodeSelector"] = {"pool": "a"}
        if k == "s":     # preferred node affinity with a NodeAffinity score weight: not on the device
            spec["affinity"] = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 5, "preference": {"matchExpressions": [
                    {"key": "pool", "operator": "In", "values": ["a"]}]}}]}}
        out.append(PodInfo.from_obj({"metadata": {"name": f"p{j}", "namespace": "default", "uid": f"bs-{j}",
                                                  "labels": {"scv/memory": "1000"}}, "spec": spec}))
    return out


def test_batch_runs_around_ineligible_pods_go_to_k_batch(fake_lib):
    lib = ctypes.CDLL(fake_lib)
    lib.yoda_fake_reset()
    eng, cache = _cluster(6)
    ok, err = eng.enable_device(fake_lib, 0, 1024, 2)
    assert ok, err
    pods = _pods()
    reqs = [pod_req(eng, p) for p in pods]
    res = eng.schedule_batch([p.num_id for p in pods], reqs)
    buf = (ctypes.c_int * 16)()
    n = lib.yoda_fake_batches(buf, 16)
    # runs [p0 p1 p2] and [p4 p5]; p3 (node selector), p6 (preferred affinity) and the lone p7
    # take per-pod cycles
    assert list(buf[:n]) == [3, 2]
    # the refused runs fell back to CPU cycles: every pod placed as by a device-less engine
    ref, ref_cache = _cluster(6)
    want = ref.schedule_batch([p.num_id for p in pods], [pod_req(ref, p) for p in pods])
    assert [r[0] for r in res] == [r[0] for r in want]
    assert all(r[0] >= 0 for r in res)
    assert eng.ledger_size == len(pods)
