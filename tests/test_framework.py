"""Config loading / default-plugin merging, the scheduling queue and the framework runtime."""
import asyncio
import os

import pytest

from yoda_scheduler_amd.framework.config import (DEFAULT_PLUGINS, load_config, merge_plugins, parse_config,
                                                 parse_duration)
from yoda_scheduler_amd.framework.queue import SchedulingQueue
from yoda_scheduler_amd.models.pod import PodInfo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_duration():
    assert parse_duration("15s") == 15 and parse_duration("1m30s") == 90 and parse_duration("100ms") == 0.1
    assert parse_duration(2) == 2.0
    with pytest.raises(ValueError):
        parse_duration("15 seconds")


def test_reference_manifest_loads_with_defaults():
    """deploy/yoda-scheduler.yaml (same object names as the reference) parses as the
    reference's v1beta1 profile: yoda at filter + score(300) on top of the defaults."""
    cfg = load_config(os.path.join(ROOT, "deploy", "yoda-scheduler.yaml"))
    assert cfg.api_version.endswith("v1beta1")
    le = cfg.leader_election
    assert (le.leader_elect, le.lease_duration, le.renew_deadline, le.retry_period) == (True, 15, 10, 2)
    assert (le.resource_name, le.resource_namespace, le.resource_lock) == ("yoda-scheduler", "kube-system", "leases")
    assert cfg.pod_initial_backoff_seconds == 1 and cfg.pod_max_backoff_seconds == 10
    names = [p.scheduler_name for p in cfg.profiles]
    assert "yoda-scheduler2" in names and "yoda-scheduler" in names    # Q6: serve both names
    p = cfg.profile("yoda-scheduler2")
    score = {r.name: r.weight for r in p.plugins["score"]}
    assert score["yoda"] == 300 and score["NodeResourcesLeastAllocated"] == 1
    assert [r.name for r in p.plugins["filter"]][-1] == "yoda"
    assert len(p.plugins["filter"]) == len(DEFAULT_PLUGINS["filter"]) + 1


def test_merge_disable_all_and_override_weight():
    m = merge_plugins({"score": {"enabled": [{"name": "NodeAffinity", "weight": 7}, {"name": "yoda", "weight": 300}],
                                 "disabled": [{"name": "ImageLocality"}]},
                       "queueSort": {"enabled": [{"name": "yoda"}], "disabled": [{"name": "*"}]}})
    s = [(r.name, r.weight) for r in m["score"]]
    assert ("NodeAffinity", 7) in s and ("yoda", 300) in s and all(n != "ImageLocality" for n, _ in s)
    assert [r.name for r in m["queueSort"]] == ["yoda"]


def test_config_validation():
    base = {"apiVersion": "kubescheduler.config.k8s.io/v1beta1", "kind": "KubeSchedulerConfiguration"}
    with pytest.raises(ValueError):
        parse_config({**base, "apiVersion": "v0"})
    with pytest.raises(ValueError):
        parse_config({**base, "percentageOfNodesToScore": 101})
    with pytest.raises(ValueError):
        parse_config({**base, "profiles": [{"schedulerName": "a"}, {"schedulerName": "a"}]})
    with pytest.raises(ValueError):
        parse_config({**base, "profiles": [{"schedulerName": "a"},
                                           {"schedulerName": "b", "plugins": {"queueSort": {
                                               "enabled": [{"name": "yoda"}], "disabled": [{"name": "*"}]}}}]})
    cfg = parse_config({**base, "apiVersion": "kubescheduler.config.k8s.io/v1"})
    assert cfg.profiles[0].scheduler_name == "default-scheduler"


def _pi(name, prio=0):
    return PodInfo.from_obj({"metadata": {"name": name, "uid": name, "labels": {"scv/priority": str(prio)}},
                             "spec": {}})


class FakeClock:
    def __init__(self):
        self.t = 100.0

    def __call__(self):
        return self.t


def test_queue_priority_then_fifo():
    q = SchedulingQueue(lambda p: (-p.gpu.priority,))
    for n, pr in [("a", 0), ("b", 5), ("c", 0), ("d", 5)]:
        q.add(_pi(n, pr))
    assert [q.pop_nowait().name for _ in range(4)] == ["b", "d", "a", "c"]
    assert q.pop_nowait() is None


def test_queue_backoff_and_unschedulable_moves():
    clk = FakeClock()
    q = SchedulingQueue(lambda p: (0,), initial_backoff=1, max_backoff=10, unschedulable_flush=60, clock=clk)
    q.add(_pi("x"))
    p = q.pop_nowait()
    cycle = q.scheduling_cycle
    q.add_unschedulable(p, cycle, unschedulable=True)
    assert q.pending()["unschedulable"] == 1
    assert q.pop_nowait() is None
    q.move_all_to_active_or_backoff("NodeAdd")        # still inside its 1 s backoff → backoffQ
    assert q.pending()["backoff"] == 1
    clk.t += 1.01
    q.flush_backoff_completed()
    p = q.pop_nowait()
    assert p.name == "x" and p.attempts == 2
    assert q.backoff_duration(p) == 2                  # 1 × 2^(2-1)
    p.attempts = 10
    assert q.backoff_duration(p) == 10                 # capped at podMaxBackoffSeconds


def test_queue_move_request_during_cycle_goes_to_backoff():
    clk = FakeClock()
    q = SchedulingQueue(lambda p: (0,), clock=clk)
    q.add(_pi("y"))
    p = q.pop_nowait()
    cycle = q.scheduling_cycle
    q.move_all_to_active_or_backoff("ScvUpdate")       # event while the pod was being scheduled
    q.add_unschedulable(p, cycle)
    assert q.pending()["backoff"] == 1 and q.pending()["unschedulable"] == 0


def test_queue_delete_and_update():
    q = SchedulingQueue(lambda p: (-p.gpu.priority,))
    q.add(_pi("a", 1))
    q.add(_pi("b", 2))
    q.delete("b")
    assert q.pop_nowait().name == "a" and q.pop_nowait() is None
    q.add(_pi("c"))
    q.update(_pi("c", 3))
    assert q.pop_nowait().gpu.priority == 3


def test_queue_update_resorts_active_pod():
    """A priority edit on a pod waiting in activeQ re-sorts it (upstream activeQ.Update);
    among equal priorities the original FIFO order is kept."""
    q = SchedulingQueue(lambda p: (-p.gpu.priority,))
    for n in ("a", "b", "c"):
        q.add(_pi(n, 1))
    q.update(_pi("c", 9))
    q.update(_pi("a", 1))                     # unchanged key: stays first among the 1s
    assert [q.pop_nowait().name for _ in range(3)] == ["c", "a", "b"]
    assert q.pop_nowait() is None and len(q) == 0


def test_queue_async_pop_wakes():
    async def run():
        q = SchedulingQueue(lambda p: (0,))
        t = asyncio.get_event_loop().create_task(q.pop())
        await asyncio.sleep(0.01)
        q.add(_pi("z"))
        return await asyncio.wait_for(t, 1)
    assert asyncio.run(run()).name == "z"


def test_unknown_plugin_and_wrong_point_rejected():
    from yoda_scheduler_amd.framework.runtime import Framework
    from yoda_scheduler_amd.framework.registry import default_registry
    cfg = parse_config({"apiVersion": "kubescheduler.config.k8s.io/v1beta1", "kind": "KubeSchedulerConfiguration",
                        "profiles": [{"schedulerName": "x", "plugins": {"filter": {"enabled": [{"name": "nope"}]}}}]})
    with pytest.raises(ValueError):
        Framework(cfg.profiles[0], default_registry(), None)
    cfg = parse_config({"apiVersion": "kubescheduler.config.k8s.io/v1beta1", "kind": "KubeSchedulerConfiguration",
                        "profiles": [{"schedulerName": "x", "plugins": {"score": {"enabled": [
                            {"name": "DefaultBinder"}]}}}]})
    with pytest.raises(ValueError):
        Framework(cfg.profiles[0], default_registry(), None)


def test_registry_with_plugin_out_of_tree():
    from yoda_scheduler_amd.framework.registry import default_registry
    from yoda_scheduler_amd.framework.interfaces import FilterPlugin, Status
    calls = []

    class OnlyNode1(FilterPlugin):
        name = "OnlyNode1"

        def filter(self, state, pod, node_name):
            calls.append(node_name)
            return Status.ok() if node_name == "n1" else Status.unschedulable("not n1")

    r = default_registry().with_plugin("OnlyNode1", lambda a, h: OnlyNode1(a, h))
    assert "OnlyNode1" in r.names()
    with pytest.raises(ValueError):
        r.register("OnlyNode1", lambda a, h: None)


def test_least_allocated_resource_weights():
    """NodeResourcesLeastAllocated ``resources`` weights (upstream resourceAllocationScorer):
    Σ score_r·w_r / Σ w_r, untracked resources only in the divisor."""
    from yoda_scheduler_amd.ops.native import core, pod_req
    from yoda_scheduler_amd.models.pod import PodInfo
    eng = core().Engine(False, 1)
    eng.filters = core().F_NODE_RESOURCES_FIT
    for i in range(6):
        eng.set_score_weight(i, 0)
    eng.set_score_weight(core().S_LEAST_ALLOCATED, 1)
    a = eng.upsert_node("a")
    b = eng.upsert_node("b")
    # a: cpu mostly free, memory mostly used; b: the opposite
    eng.set_node_meta(a, False, [], [], 100_000, 100 << 30, 110)
    eng.set_node_meta(b, False, [], [], 100_000, 100 << 30, 110)

    def load(idx, uid, cpu, mem):
        p = PodInfo.from_obj({"metadata": {"name": uid, "uid": uid}, "spec": {"containers": [
            {"name": "c", "resources": {"requests": {"cpu": cpu, "memory": mem}}}]}})
        assert eng.reserve(p.num_id, pod_req(eng, p), idx, [])
    load(a, "load-a", "10", "90Gi")
    load(b, "load-b", "90", "10Gi")
    pi = PodInfo.from_obj({"metadata": {"name": "p", "uid": "u-lw"},
                           "spec": {"containers": [{"name": "c", "resources": {"requests": {"cpu": "1", "memory": "1Gi"}}}]}})
    req = pod_req(eng, pi)
    default = eng.score_nodes(req, [a, b])
    eng.set_alloc_weights(False, 3, 1, 0)          # cpu counts 3×
    cpu_heavy = eng.score_nodes(req, [a, b])
    eng.set_alloc_weights(False, 1, 1, 2)          # two untracked resources in the divisor
    diluted = eng.score_nodes(req, [a, b])
    # a: cpu (100-11)% free = 89, memory (100-91)% = 9; b mirrored
    assert default == [49, 49]                      # (89 + 9) / 2
    assert cpu_heavy == [69, 29]                    # (89·3 + 9) / 4, (9·3 + 89) / 4
    assert diluted == [24, 24]                      # (89 + 9) / 4


def _granted(rules, group, resource, verb, name=None):
    for r in rules:
        if group not in r.get("apiGroups", []) or resource not in r.get("resources", []):
            continue
        if verb not in r.get("verbs", []) and "*" not in r.get("verbs", []):
            continue
        names = r.get("resourceNames")
        if names and (name is None or name not in names):
            continue
        return True
    return False


def test_deploy_rbac_covers_every_api_call():
    """The ClusterRole in deploy/yoda-scheduler.yaml grants each (group, resource, verb) the
    scheduler issues: informers, binding, status/condition patches, preemption deletes,
    events (both APIs), leader-election locks, the Scv CRD (C17, reference
    ``deploy/yoda-scheduler.yaml:71-216``)."""
    import os
    import yaml
    from yoda_scheduler_amd.kube.resources import RESOURCES
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    docs = [d for d in yaml.safe_load_all(open(os.path.join(root, "deploy", "yoda-scheduler.yaml"))) if d]
    role = [d for d in docs if d["kind"] == "ClusterRole"][0]
    assert role["metadata"]["name"] == "yoda-cr"
    rules = role["rules"]
    watched = ["pods", "nodes", "scvs", "poddisruptionbudgets", "services", "replicationcontrollers",
               "replicasets", "statefulsets", "persistentvolumeclaims", "persistentvolumes", "storageclasses",
               "csinodes"]
    need = [(RESOURCES[r].group, RESOURCES[r].name, v) for r in watched for v in ("list", "watch")]
    need += [("", "pods/binding", "create"), ("", "pods", "patch"), ("", "pods", "delete"),
             ("", "events", "create"), ("", "events", "update"),
             ("events.k8s.io", "events", "create"), ("events.k8s.io", "events", "patch"),
             ("coordination.k8s.io", "leases", "get"), ("coordination.k8s.io", "leases", "create"),
             ("coordination.k8s.io", "leases", "update"), ("core.run-linux.com", "scvs", "patch"),
             ("core.run-linux.com", "scvs/status", "update"), ("", "configmaps", "get")]
    missing = [n for n in need if not _granted(rules, *n)]
    assert missing == []
    for res in ("endpoints", "configmaps"):          # legacy / multi resourceLocks on the lock object
        assert _granted(rules, "", res, "create") and _granted(rules, "", res, "update", "yoda-scheduler")
