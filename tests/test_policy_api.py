"""Legacy scheduler Policy API (``--policy-config-file`` / ``--policy-configmap`` /
``algorithmSource.policy``) → plugin profile translation, and a Policy-configured
scheduler running end to end on the fake apiserver."""
import asyncio
import json

import pytest

from yoda_scheduler_amd.framework.config import apply_policy, parse_config, resolve_policy_configmap
from yoda_scheduler_amd.framework.policy import translate
from yoda_scheduler_amd.testing import FakeCluster, yoda_config


def names(plugins, point):
    return [r["name"] for r in plugins[point]["enabled"]]


def test_default_policy_when_lists_are_null():
    plugins, pc, ext = translate({"kind": "Policy", "apiVersion": "v1"})
    f = names(plugins, "filter")
    for n in ("NodeResourcesFit", "NodeName", "NodePorts", "NodeAffinity", "TaintToleration", "NodeUnschedulable",
              "VolumeBinding", "VolumeZone", "EBSLimits", "GCEPDLimits", "AzureDiskLimits", "NodeVolumeLimits",
              "VolumeRestrictions", "InterPodAffinity", "PodTopologySpread"):
        assert n in f, n
    scores = {r["name"]: r["weight"] for r in plugins["score"]["enabled"]}
    assert scores["NodePreferAvoidPods"] == 10000 and scores["PodTopologySpread"] == 2
    assert scores["SelectorSpread"] == 1 and scores["NodeResourcesLeastAllocated"] == 1
    assert names(plugins, "queueSort") == ["PrioritySort"] and names(plugins, "bind") == ["DefaultBinder"]
    assert names(plugins, "reserve") == ["VolumeBinding"] and names(plugins, "preBind") == ["VolumeBinding"]
    assert pc == [] and ext == []


def test_empty_lists_keep_only_mandatory_predicates():
    plugins, _, _ = translate({"predicates": [], "priorities": []})
    assert names(plugins, "filter") == ["TaintToleration", "NodeUnschedulable"]
    assert names(plugins, "score") == []


def test_custom_predicates_and_priorities_become_plugin_args():
    pol = {"predicates": [{"name": "PodFitsResources"},
                          {"name": "zone-present", "argument": {"labelsPresence": {"labels": ["zone"], "presence": True}}},
                          {"name": "no-spot", "argument": {"labelsPresence": {"labels": ["spot"], "presence": False}}},
                          {"name": "svc", "argument": {"serviceAffinity": {"labels": ["rack"]}}}],
           "priorities": [{"name": "MostRequestedPriority", "weight": 3},
                          {"name": "ssd", "weight": 2, "argument": {"labelPreference": {"label": "ssd", "presence": True}}},
                          {"name": "hdd", "weight": 1, "argument": {"labelPreference": {"label": "hdd", "presence": False}}},
                          {"name": "anti", "weight": 4, "argument": {"serviceAntiAffinity": {"label": "zone"}}},
                          {"name": "rtcr", "weight": 5, "argument": {"requestedToCapacityRatioArguments": {
                              "shape": [{"utilization": 0, "score": 0}, {"utilization": 100, "score": 10}],
                              "resources": [{"name": "amd.com/gpu", "weight": 1}]}}}],
           "hardPodAffinitySymmetricWeight": 7}
    plugins, pc, _ = translate(pol)
    args = {it["name"]: it["args"] for it in pc}
    assert args["NodeLabel"] == {"presentLabels": ["zone"], "absentLabels": ["spot"],
                                 "presentLabelsPreference": ["ssd"], "absentLabelsPreference": ["hdd"]}
    assert args["ServiceAffinity"] == {"affinityLabels": ["rack"], "antiAffinityLabelsPreference": ["zone"]}
    assert args["RequestedToCapacityRatio"]["resources"] == [{"name": "amd.com/gpu", "weight": 1}]
    assert args["InterPodAffinity"] == {"hardPodAffinityWeight": 7}
    scores = {r["name"]: r["weight"] for r in plugins["score"]["enabled"]}
    assert scores == {"NodeResourcesMostAllocated": 3, "NodeLabel": 3, "ServiceAffinity": 4,
                      "RequestedToCapacityRatio": 5}
    assert "ServiceAffinity" in names(plugins, "preFilter")


@pytest.mark.parametrize("bad", [
    {"predicates": [{"name": "NoSuchPredicate"}]},
    {"priorities": [{"name": "LeastRequestedPriority", "weight": 0}]},
    {"priorities": [{"name": "NoSuchPriority", "weight": 1}]},
    {"predicates": [{"name": "HostName"}, {"name": "HostName"}]},
    {"hardPodAffinitySymmetricWeight": 101},
])
def test_invalid_policies_rejected(bad):
    with pytest.raises(ValueError):
        translate(bad)


def test_policy_file_in_algorithm_source_keeps_yoda(tmp_path):
    p = tmp_path / "policy.json"
    p.write_text(json.dumps({"kind": "Policy", "apiVersion": "v1",
                             "predicates": [{"name": "GeneralPredicates"}],
                             "priorities": [{"name": "LeastRequestedPriority", "weight": 1}]}))
    doc = yoda_config()
    doc["algorithmSource"] = {"policy": {"file": {"path": str(p)}}}
    cfg = parse_config(doc)
    prof = cfg.profiles[0]
    f = [r.name for r in prof.plugins["filter"]]
    s = {r.name: r.weight for r in prof.plugins["score"]}
    assert "yoda" in f and "NodeResourcesFit" in f and "VolumeBinding" not in f
    assert s == {"NodeResourcesLeastAllocated": 1, "yoda": 300}
    assert [r.name for r in prof.plugins["queueSort"]] == ["yoda"]     # explicit out-of-tree order wins
    assert prof.plugin_config["yoda"] == {}


def test_policy_configmap_resolved_against_apiserver():
    async def go():
        c = FakeCluster()
        pol = {"kind": "Policy", "apiVersion": "v1", "predicates": [{"name": "PodFitsResources"}],
               "priorities": [{"name": "MostRequestedPriority", "weight": 2}]}
        c.server.create("configmaps", {"metadata": {"name": "sched-policy", "namespace": "kube-system"},
                                       "data": {"policy.cfg": json.dumps(pol)}})
        doc = yoda_config()
        doc["algorithmSource"] = {"policy": {"configMap": {"name": "sched-policy"}}}
        cfg = parse_config(doc)
        assert cfg.policy_configmap == ("kube-system", "sched-policy")
        cfg = await resolve_policy_configmap(cfg, c.client)
        prof = cfg.profiles[0]
        return {r.name: r.weight for r in prof.plugins["score"]}, cfg.policy_configmap
    scores, pending = asyncio.run(go())
    assert scores == {"NodeResourcesMostAllocated": 2, "yoda": 300} and pending is None


def test_policy_scheduler_end_to_end_node_label_presence():
    async def go():
        cfg = apply_policy(parse_config(yoda_config()), {
            "predicates": [{"name": "GeneralPredicates"},
                           {"name": "need-mi355x", "argument": {"labelsPresence": {"labels": ["amd.com/mi355x"],
                                                                                   "presence": True}}}],
            "priorities": [{"name": "LeastRequestedPriority", "weight": 1}]})
        c = FakeCluster()
        c.config = cfg
        c.add_node("other")
        c.add_node("mi", labels={"amd.com/mi355x": "true"})
        await c.start()
        for i in range(3):
            c.add_pod(f"p{i}", {"scv/memory": "1000"})
        assert await c.wait_bound(3)
        out = {c.node_of(f"p{i}") for i in range(3)}
        await c.stop()
        return out
    assert asyncio.run(go()) == {"mi"}


def test_cli_policy_config_file_flag(tmp_path):
    from yoda_scheduler_amd.cmd.scheduler import new_scheduler_command
    p = tmp_path / "policy.yaml"
    p.write_text("kind: Policy\napiVersion: v1\npredicates:\n- name: HostName\npriorities:\n"
                 "- name: ImageLocalityPriority\n  weight: 4\n")
    out = tmp_path / "cfg.json"
    rc = new_scheduler_command()(["--policy-config-file", str(p), "--use-legacy-policy-config", "true",
                                  "--write-config-to", str(out)])
    assert rc == 0
    cfg = json.loads(out.read_text())
    prof = cfg["profiles"][0]
    assert [r["name"] for r in prof["plugins"]["filter"]] == ["NodeName", "TaintToleration", "NodeUnschedulable"]
    assert [(r["name"], r["weight"]) for r in prof["plugins"]["score"]] == [("ImageLocality", 4)]
