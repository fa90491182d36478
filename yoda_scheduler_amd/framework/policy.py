"""Legacy scheduler ``Policy`` (``kind: Policy, apiVersion: v1``) → plugin profile.

kube-scheduler v1.20 — the binary the reference extends (``pkg/register/register.go:9-13``,
``go.mod:12``) — still accepts the pre-framework Policy API through
``--policy-config-file`` / ``--policy-configmap`` or the v1beta1 key
``algorithmSource.policy.{file.path, configMap.{namespace,name}}``. Upstream translates
each named predicate / priority into framework plugins (``legacy_registry.go``); this
module does the same translation into the profile format :mod:`config` consumes, so a
Policy-configured deployment keeps scheduling the same way here.

Choices worth knowing:

* ``predicates: null`` → the v1.20 default predicate set; ``[]`` → only the mandatory
  ones (taint toleration, unschedulable). ``priorities`` likewise.
* custom predicates/priorities with ``argument.labelsPresence`` / ``labelPreference``
  become one ``NodeLabel`` plugin (labels merged, score weight = Σ weights);
  ``serviceAffinity`` / ``serviceAntiAffinity`` one ``ServiceAffinity`` plugin;
  ``requestedToCapacityRatioArguments`` the ``RequestedToCapacityRatio`` args.
* Out-of-tree plugins the profile enables explicitly (``yoda``) are kept on top of the
  Policy-derived set — upstream would drop them, which would make a Policy file and
  the yoda plugin mutually exclusive.
* Parity is unpinned against an upstream run (no upstream source in the reference
  tree); the mapping table is tested in ``tests/test_policy_api.py``.
"""
from __future__ import annotations

import json
from typing import Optional

import yaml

# predicate → [(extension points, plugin)]
_F = ("filter",)
_PF = ("preFilter", "filter")
PREDICATES: dict[str, list[tuple[tuple[str, ...], str]]] = {
    "GeneralPredicates": [(_PF, "NodeResourcesFit"), (_F, "NodeName"), (_PF, "NodePorts"), (_F, "NodeAffinity")],
    "PodFitsResources": [(_PF, "NodeResourcesFit")],
    "HostName": [(_F, "NodeName")],
    "PodFitsHostPorts": [(_PF, "NodePorts")],
    "PodFitsPorts": [(_PF, "NodePorts")],
    "MatchNodeSelector": [(_F, "NodeAffinity")],
    "PodToleratesNodeTaints": [(_F, "TaintToleration")],
    "CheckNodeUnschedulable": [(_F, "NodeUnschedulable")],
    "CheckVolumeBinding": [(("preFilter", "filter", "reserve", "preBind"), "VolumeBinding")],
    "NoDiskConflict": [(_F, "VolumeRestrictions")],
    "NoVolumeZoneConflict": [(_F, "VolumeZone")],
    "MaxCSIVolumeCountPred": [(_F, "NodeVolumeLimits")],
    "MaxEBSVolumeCount": [(_F, "EBSLimits")],
    "MaxGCEPDVolumeCount": [(_F, "GCEPDLimits")],
    "MaxAzureDiskVolumeCount": [(_F, "AzureDiskLimits")],
    "MaxCinderVolumeCount": [(_F, "CinderLimits")],
    "MatchInterPodAffinity": [(_PF, "InterPodAffinity")],
    "EvenPodsSpread": [(_PF, "PodTopologySpread")],
    "CheckNodeLabelPresence": [(_F, "NodeLabel")],
    "CheckServiceAffinity": [(_PF, "ServiceAffinity")],
}
DEFAULT_PREDICATES = ("NoVolumeZoneConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount",
                      "MaxCSIVolumeCountPred", "MatchInterPodAffinity", "NoDiskConflict", "GeneralPredicates",
                      "PodToleratesNodeTaints", "CheckVolumeBinding", "CheckNodeUnschedulable", "EvenPodsSpread")
MANDATORY_PREDICATES = ("PodToleratesNodeTaints", "CheckNodeUnschedulable")

# priority → [(extension points, plugin)]; the plugin's score weight is the priority's
_S = ("score",)
_PS = ("preScore", "score")
PRIORITIES: dict[str, list[tuple[tuple[str, ...], str]]] = {
    "EvenPodsSpreadPriority": [(_PS, "PodTopologySpread")],
    "SelectorSpreadPriority": [(_PS, "SelectorSpread")],
    "ServiceSpreadingPriority": [(_PS, "SelectorSpread")],
    "TaintTolerationPriority": [(_PS, "TaintToleration")],
    "NodeAffinityPriority": [(_S, "NodeAffinity")],
    "ImageLocalityPriority": [(_S, "ImageLocality")],
    "InterPodAffinityPriority": [(_PS, "InterPodAffinity")],
    "NodePreferAvoidPodsPriority": [(_S, "NodePreferAvoidPods")],
    "MostRequestedPriority": [(_S, "NodeResourcesMostAllocated")],
    "BalancedResourceAllocation": [(_S, "NodeResourcesBalancedAllocation")],
    "LeastRequestedPriority": [(_S, "NodeResourcesLeastAllocated")],
    "RequestedToCapacityRatioPriority": [(_S, "RequestedToCapacityRatio")],
    "NodeLabelPriority": [(_S, "NodeLabel")],
    "ServiceAntiAffinityPriority": [(_S, "ServiceAffinity")],
}
DEFAULT_PRIORITIES = {"SelectorSpreadPriority": 1, "InterPodAffinityPriority": 1, "LeastRequestedPriority": 1,
                      "BalancedResourceAllocation": 1, "NodePreferAvoidPodsPriority": 10000,
                      "NodeAffinityPriority": 1, "TaintTolerationPriority": 1, "ImageLocalityPriority": 1,
                      "EvenPodsSpreadPriority": 2}
MAX_TOTAL_PRIORITY = 1 << 62
POINTS = ("queueSort", "preFilter", "filter", "postFilter", "preScore", "score", "reserve", "permit", "preBind",
          "bind", "postBind")


def load_policy_text(text: str) -> dict:
    """A Policy document (JSON, or YAML — upstream accepts both)."""
    try:
        doc = json.loads(text)
    except ValueError:
        doc = yaml.safe_load(text)
    if not isinstance(doc, dict):
        raise ValueError("policy: not an object")
    kind = doc.get("kind", "Policy")
    if kind != "Policy":
        raise ValueError(f"policy: kind must be Policy, got {kind!r}")
    return doc


def load_policy_file(path: str) -> dict:
    with open(path) as f:
        return load_policy_text(f.read())


def policy_from_configmap(cm: dict) -> dict:
    """upstream reads key ``policy.cfg`` of the ConfigMap."""
    data = (cm.get("data") or {}).get("policy.cfg")
    if data is None:
        raise ValueError("policy ConfigMap has no 'policy.cfg' key")
    return load_policy_text(data)


class _Builder:
    def __init__(self) -> None:
        self.points: dict[str, list[dict]] = {p: [] for p in POINTS}
        self.args: dict[str, dict] = {}

    def add(self, points, name: str, weight: int = 0) -> None:
        for pt in points:
            lst = self.points[pt]
            for ref in lst:
                if ref["name"] == name:
                    if pt == "score":
                        ref["weight"] += weight
                    break
            else:
                lst.append({"name": name, "weight": weight} if pt == "score" else {"name": name})

    def arg_list(self, plugin: str, key: str, values) -> None:
        a = self.args.setdefault(plugin, {})
        cur = a.setdefault(key, [])
        for v in values:
            if v not in cur:
                cur.append(v)


def translate(policy: dict) -> tuple[dict, list[dict], list[dict]]:
    """Policy → (``plugins`` block with every point fully specified, ``pluginConfig``,
    ``extenders``)."""
    b = _Builder()
    b.add(("queueSort",), "PrioritySort")
    b.add(("postFilter",), "DefaultPreemption")
    b.add(("bind",), "DefaultBinder")

    preds = policy.get("predicates")
    names = [{"name": n} for n in DEFAULT_PREDICATES] if preds is None else list(preds)
    seen = set()
    for m in MANDATORY_PREDICATES:
        if all(p.get("name") != m for p in names):
            names.append({"name": m})
    for p in names:
        name = p.get("name", "")
        if name in seen:
            raise ValueError(f"policy: duplicate predicate {name!r}")
        seen.add(name)
        arg = p.get("argument") or {}
        if "labelsPresence" in arg:
            lp = arg["labelsPresence"] or {}
            key = "presentLabels" if lp.get("presence", False) else "absentLabels"
            b.arg_list("NodeLabel", key, lp.get("labels") or [])
            b.add(_F, "NodeLabel")
        elif "serviceAffinity" in arg:
            b.arg_list("ServiceAffinity", "affinityLabels", (arg["serviceAffinity"] or {}).get("labels") or [])
            b.add(_PF, "ServiceAffinity")
        elif name in PREDICATES:
            for pts, plugin in PREDICATES[name]:
                b.add(pts, plugin)
        else:
            raise ValueError(f"policy: unknown predicate {name!r}")

    prios = policy.get("priorities")
    items = [{"name": n, "weight": w} for n, w in DEFAULT_PRIORITIES.items()] if prios is None else list(prios)
    total = 0
    seen = set()
    for p in items:
        name = p.get("name", "")
        w = int(p.get("weight", 0) or 0)
        if w <= 0:
            raise ValueError(f"policy: priority {name!r} weight must be positive")
        total += w
        if total > MAX_TOTAL_PRIORITY:
            raise ValueError("policy: total priority weight overflows")
        if name in seen:
            raise ValueError(f"policy: duplicate priority {name!r}")
        seen.add(name)
        arg = p.get("argument") or {}
        if "labelPreference" in arg:
            lp = arg["labelPreference"] or {}
            key = "presentLabelsPreference" if lp.get("presence", False) else "absentLabelsPreference"
            b.arg_list("NodeLabel", key, [lp.get("label", "")])
            b.add(_S, "NodeLabel", w)
        elif "serviceAntiAffinity" in arg:
            b.arg_list("ServiceAffinity", "antiAffinityLabelsPreference",
                       [(arg["serviceAntiAffinity"] or {}).get("label", "")])
            b.add(_S, "ServiceAffinity", w)
        elif "requestedToCapacityRatioArguments" in arg:
            r = arg["requestedToCapacityRatioArguments"] or {}
            b.args["RequestedToCapacityRatio"] = {"shape": list(r.get("shape") or []),
                                                  "resources": list(r.get("resources") or [])}
            b.add(_S, "RequestedToCapacityRatio", w)
        elif name in PRIORITIES:
            if name == "RequestedToCapacityRatioPriority" and "RequestedToCapacityRatio" not in b.args:
                raise ValueError("policy: RequestedToCapacityRatioPriority needs requestedToCapacityRatioArguments")
            for pts, plugin in PRIORITIES[name]:
                b.add(pts, plugin, w)
        else:
            raise ValueError(f"policy: unknown priority {name!r}")

    if "hardPodAffinitySymmetricWeight" in policy:
        w = int(policy["hardPodAffinitySymmetricWeight"])
        if not 0 <= w <= 100:
            raise ValueError("policy: hardPodAffinitySymmetricWeight must be in [0, 100]")
        b.args.setdefault("InterPodAffinity", {})["hardPodAffinityWeight"] = w

    plugins = {pt: {"enabled": refs, "disabled": [{"name": "*"}]} for pt, refs in b.points.items()}
    plugin_config = [{"name": n, "args": a} for n, a in b.args.items()]
    return plugins, plugin_config, list(policy.get("extenders") or [])


def builtin_plugin_names() -> set:
    """Names of the in-tree (upstream) plugins — everything but out-of-tree ones like yoda."""
    from ..plugins.defaults import register_defaults
    from .registry import Registry
    r = Registry()
    register_defaults(r)
    return set(r.names())


def apply_to_document(doc: dict, policy: dict, builtin: Optional[set] = None) -> dict:
    """Rewrite a KubeSchedulerConfiguration document so its (single) profile runs the
    Policy. ``builtin`` = in-tree plugin names; plugins outside it that the profile
    enables explicitly (e.g. ``yoda``) are kept."""
    profiles = doc.get("profiles") or [{}]
    if len(profiles) != 1:
        raise ValueError("policy: multiple profiles are not supported with a Policy")
    prof = dict(profiles[0])
    plugins, pc, ext = translate(policy)
    if builtin is not None:
        for pt, block in (prof.get("plugins") or {}).items():
            if pt not in plugins:
                continue
            for ref in (block or {}).get("enabled") or []:
                if ref.get("name") in builtin:
                    continue
                if pt == "queueSort":                 # one queue order: the explicit one wins
                    plugins[pt]["enabled"] = [dict(ref)]
                elif all(r["name"] != ref["name"] for r in plugins[pt]["enabled"]):
                    plugins[pt]["enabled"].append(dict(ref))
    prof["plugins"] = plugins
    by_name = {it["name"]: it for it in prof.get("pluginConfig") or []}
    for it in pc:
        by_name[it["name"]] = it
    prof["pluginConfig"] = list(by_name.values())
    out = dict(doc)
    out["profiles"] = [prof]
    if ext:
        out["extenders"] = list(doc.get("extenders") or []) + ext
    out.pop("algorithmSource", None)
    return out
