"""``KubeSchedulerConfiguration`` loader (v1beta1 as shipped by the reference, plus
v1beta2/v1beta3/v1), with upstream default-plugin merging.

The reference ships a v1beta1 config enabling ``yoda`` at filter (weight 0) and score
(weight 300) under ``schedulerName: yoda-scheduler2``, with leader election on lease
``kube-system/yoda-scheduler`` 15s/10s/2s, ``percentageOfNodesToScore: 0`` and pod
backoff 1s→10s (``deploy/yoda-scheduler.yaml:8-31``). Profiles only list yoda, so the
upstream defaults stay enabled; ``merge_plugins`` reproduces that.
"""
from __future__ import annotations

import copy
import re
from dataclasses import dataclass, field
from typing import Any, Optional

import yaml

from .interfaces import EXTENSION_POINTS

SUPPORTED_API_VERSIONS = (
    "kubescheduler.config.k8s.io/v1beta1",
    "kubescheduler.config.k8s.io/v1beta2",
    "kubescheduler.config.k8s.io/v1beta3",
    "kubescheduler.config.k8s.io/v1",
)


@dataclass
class PluginRef:
    name: str
    weight: int = 0


# kube-scheduler v1.20 (v1beta1) default plugin set, in upstream order.
DEFAULT_PLUGINS: dict[str, list[PluginRef]] = {
    "queueSort": [PluginRef("PrioritySort")],
    "preFilter": [PluginRef("NodeResourcesFit"), PluginRef("NodePorts"), PluginRef("PodTopologySpread"),
                  PluginRef("InterPodAffinity"), PluginRef("VolumeBinding")],
    "filter": [PluginRef("NodeUnschedulable"), PluginRef("NodeResourcesFit"), PluginRef("NodeName"),
               PluginRef("NodePorts"), PluginRef("NodeAffinity"), PluginRef("VolumeRestrictions"),
               PluginRef("TaintToleration"), PluginRef("EBSLimits"), PluginRef("GCEPDLimits"),
               PluginRef("NodeVolumeLimits"), PluginRef("AzureDiskLimits"), PluginRef("VolumeBinding"),
               PluginRef("VolumeZone"), PluginRef("PodTopologySpread"), PluginRef("InterPodAffinity")],
    "postFilter": [PluginRef("DefaultPreemption")],
    "preScore": [PluginRef("InterPodAffinity"), PluginRef("PodTopologySpread"), PluginRef("TaintToleration")],
    "score": [PluginRef("NodeResourcesBalancedAllocation", 1), PluginRef("ImageLocality", 1),
              PluginRef("InterPodAffinity", 1), PluginRef("NodeResourcesLeastAllocated", 1),
              PluginRef("NodeAffinity", 1), PluginRef("NodePreferAvoidPods", 10000),
              PluginRef("PodTopologySpread", 2), PluginRef("TaintToleration", 1)],
    "reserve": [PluginRef("VolumeBinding")],
    "permit": [],
    "preBind": [PluginRef("VolumeBinding")],
    "bind": [PluginRef("DefaultBinder")],
    "postBind": [],
}


@dataclass
class LeaderElectionConfig:
    leader_elect: bool = True
    lease_duration: float = 15.0
    renew_deadline: float = 10.0
    retry_period: float = 2.0
    resource_lock: str = "leases"
    resource_name: str = "kube-scheduler"
    resource_namespace: str = "kube-system"


@dataclass
class ClientConnection:
    kubeconfig: str = ""
    qps: float = 50.0
    burst: int = 100
    content_type: str = "application/json"


@dataclass
class Profile:
    scheduler_name: str = "default-scheduler"
    plugins: dict[str, list[PluginRef]] = field(default_factory=dict)
    plugin_config: dict[str, dict] = field(default_factory=dict)


@dataclass
class ExtenderConfig:
    """``extenders[]`` of KubeSchedulerConfiguration (upstream HTTP scheduler extenders)."""
    url_prefix: str
    filter_verb: str = ""
    prioritize_verb: str = ""
    bind_verb: str = ""
    weight: int = 1
    http_timeout: float = 30.0
    node_cache_capable: bool = False
    managed_resources: list = field(default_factory=list)   # [(name, ignoredByScheduler)]
    ignorable: bool = False


@dataclass
class SchedulerConfig:
    api_version: str = SUPPORTED_API_VERSIONS[0]
    leader_election: LeaderElectionConfig = field(default_factory=LeaderElectionConfig)
    client_connection: ClientConnection = field(default_factory=ClientConnection)
    percentage_of_nodes_to_score: int = 0
    pod_initial_backoff_seconds: float = 1.0
    pod_max_backoff_seconds: float = 10.0
    parallelism: int = 16
    health_bind_address: str = "0.0.0.0:10251"
    metrics_bind_address: str = "0.0.0.0:10251"
    enable_profiling: bool = True
    profiles: list[Profile] = field(default_factory=list)
    # yoda-mi355x extensions (top-level key ``yodaRuntime``): binding pipeline + batching
    bind_concurrency: int = 256
    batch_size: int = 256
    unschedulable_flush_seconds: float = 60.0
    gc_threshold: tuple = (50_000, 50, 1000)
    # gfx950 device scorer (yodaRuntime.deviceScorer): auto = use it when a GPU is visible
    device_scorer: str = "auto"
    device_index: int = 0
    # CPU engine vs k_batch per pod on MI355X cross at ≈ 44 nodes (profiles/bench/r3/crossover/)
    device_min_nodes: int = 48
    device_capacity: int = 65536
    engine_threads: int = 1
    # run native batches on a worker thread (GIL released) so the event loop binds and
    # ingests the previous batch meanwhile; auto = when the gfx950 device scorer is active
    # (config 6 on MI355X: +45-50 % pods/s, profiles/bench/README.md)
    overlap_engine: str = "auto"
    # native runs in flight on the engine worker at once (overlapped mode): 2 = one placing
    # while the previous is applied; 3 keeps one more queued so the engine (GPU) never idles
    # while the event loop catches up with binds and watch events
    overlap_depth: int = 3
    # Scv updates requeue parked pods only when the new sample can add capacity (a card
    # healthy again, more effective free HBM, a changed clock, more cards, stale → fresh);
    # False: every Scv event moves the whole unschedulable queue (upstream's behaviour for
    # any cluster event)
    scv_queueing_hint: bool = True
    # native pod lane (yodaRuntime.nativeLane): pods of all-native profiles are queued,
    # placed, bound, confirmed and released in C++ (native/core/lane.hpp) with no Python call
    # per pod; auto = on whenever the native Kubernetes transport is in use
    native_lane: str = "auto"
    # yodaRuntime.laneMirrorSettleSeconds: the Python cache mirrors lane pods for Python
    # plugins that read other pods (affinity, spread, preemption); once no Python-path cycle
    # has read the mirror for this long it is dropped and the lane's change log turned off
    lane_mirror_settle_s: float = 5.0
    # event API (yodaRuntime.eventsAPI): upstream v1.20 records through events.k8s.io/v1
    events_api: str = "events.k8s.io/v1"
    trace: bool = False
    extenders: list = field(default_factory=list)     # [ExtenderConfig]
    # legacy Policy held in a ConfigMap (algorithmSource.policy.configMap / --policy-configmap):
    # resolved against the apiserver by ``resolve_policy_configmap`` before the scheduler starts
    policy_configmap: Optional[tuple] = None
    source_doc: Optional[dict] = None

    def profile(self, name: str) -> Optional[Profile]:
        for p in self.profiles:
            if p.scheduler_name == name:
                return p
        return None


_DUR = re.compile(r"(\d+(?:\.\d+)?)(ns|us|µs|ms|s|m|h)")
_UNIT = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


def parse_duration(v: Any) -> float:
    """Go ``time.Duration`` string ("15s", "1m30s", "100ms") or a number of seconds."""
    if v is None:
        return 0.0
    if isinstance(v, (int, float)):
        return float(v)
    s = str(v).strip()
    if not s:
        return 0.0
    total, pos = 0.0, 0
    for m in _DUR.finditer(s):
        if m.start() != pos:
            raise ValueError(f"invalid duration {v!r}")
        total += float(m.group(1)) * _UNIT[m.group(2)]
        pos = m.end()
    if pos != len(s):
        raise ValueError(f"invalid duration {v!r}")
    return total


def _plugin_set(d: Optional[dict]) -> tuple[list[PluginRef], list[str]]:
    d = d or {}
    enabled = [PluginRef(p["name"], int(p.get("weight", 0) or 0)) for p in d.get("enabled") or []]
    disabled = [p["name"] for p in d.get("disabled") or []]
    return enabled, disabled


def merge_plugins(custom: dict[str, Any] | None) -> dict[str, list[PluginRef]]:
    """Upstream ``mergePlugins``: defaults minus ``disabled`` (``*`` = all); enabled
    plugins that are also defaults override the default in place; the rest append."""
    custom = custom or {}
    out: dict[str, list[PluginRef]] = {}
    for point in EXTENSION_POINTS:
        enabled, disabled = _plugin_set(custom.get(point))
        dis = set(disabled)
        en = {p.name: p for p in enabled}
        merged: list[PluginRef] = []
        used = set()
        if "*" not in dis:
            for p in DEFAULT_PLUGINS[point]:
                if p.name in dis:
                    continue
                if p.name in en:
                    merged.append(copy.copy(en[p.name]))
                    used.add(p.name)
                else:
                    merged.append(copy.copy(p))
        for p in enabled:
            if p.name not in used:
                merged.append(copy.copy(p))
                used.add(p.name)
        if point == "score":
            for p in merged:
                if p.weight == 0:
                    p.weight = 1
        out[point] = merged
    # multiPoint (v1beta3+): enable at every point the plugin implements; resolved later
    mp_enabled, _ = _plugin_set(custom.get("multiPoint"))
    if mp_enabled:
        out["multiPoint"] = mp_enabled
    return out


def _f(d: dict, key: str, default):
    v = d.get(key)
    return default if v is None else v


def parse_config(doc: dict) -> SchedulerConfig:
    av = doc.get("apiVersion", SUPPORTED_API_VERSIONS[0])
    if av not in SUPPORTED_API_VERSIONS:
        raise ValueError(f"unsupported apiVersion {av!r}")
    if doc.get("kind", "KubeSchedulerConfiguration") != "KubeSchedulerConfiguration":
        raise ValueError("kind must be KubeSchedulerConfiguration")
    policy_cm = None
    pol = (doc.get("algorithmSource") or {}).get("policy")
    if pol:
        if av != SUPPORTED_API_VERSIONS[0]:
            raise ValueError("algorithmSource (legacy Policy) is only supported in v1beta1")
        from . import policy as _policy
        if (pol.get("file") or {}).get("path"):
            doc = _policy.apply_to_document(doc, _policy.load_policy_file(pol["file"]["path"]),
                                            _policy.builtin_plugin_names())
        elif pol.get("configMap"):
            cm = pol["configMap"]
            if not cm.get("name"):
                raise ValueError("algorithmSource.policy.configMap.name is required")
            policy_cm = (cm.get("namespace") or "kube-system", cm["name"])
        else:
            raise ValueError("algorithmSource.policy needs file.path or configMap")
    le = doc.get("leaderElection") or {}
    cc = doc.get("clientConnection") or {}
    cfg = SchedulerConfig(
        api_version=av,
        leader_election=LeaderElectionConfig(
            leader_elect=bool(_f(le, "leaderElect", True)),
            lease_duration=parse_duration(_f(le, "leaseDuration", "15s")),
            renew_deadline=parse_duration(_f(le, "renewDeadline", "10s")),
            retry_period=parse_duration(_f(le, "retryPeriod", "2s")),
            resource_lock=_f(le, "resourceLock", "leases"),
            resource_name=_f(le, "resourceName", "kube-scheduler"),
            resource_namespace=_f(le, "resourceNamespace", "kube-system"),
        ),
        client_connection=ClientConnection(
            kubeconfig=_f(cc, "kubeconfig", ""), qps=float(_f(cc, "qps", 50)), burst=int(_f(cc, "burst", 100)),
            content_type=_f(cc, "contentType", "application/json")),
        percentage_of_nodes_to_score=int(_f(doc, "percentageOfNodesToScore", 0)),
        pod_initial_backoff_seconds=float(_f(doc, "podInitialBackoffSeconds", 1)),
        pod_max_backoff_seconds=float(_f(doc, "podMaxBackoffSeconds", 10)),
        parallelism=int(_f(doc, "parallelism", 16)),
        health_bind_address=_f(doc, "healthzBindAddress", "0.0.0.0:10251"),
        metrics_bind_address=_f(doc, "metricsBindAddress", "0.0.0.0:10251"),
        enable_profiling=bool(_f(doc, "enableProfiling", True)),
    )
    rt = doc.get("yodaRuntime") or {}
    cfg.bind_concurrency = int(_f(rt, "bindConcurrency", cfg.bind_concurrency))
    cfg.batch_size = int(_f(rt, "batchSize", cfg.batch_size))
    cfg.unschedulable_flush_seconds = float(_f(rt, "unschedulableFlushSeconds", cfg.unschedulable_flush_seconds))
    cfg.gc_threshold = tuple(int(x) for x in _f(rt, "gcThreshold", cfg.gc_threshold))
    ds = rt.get("deviceScorer") or {}
    en = _f(ds, "enabled", "auto")
    cfg.device_scorer = {True: "on", False: "off"}.get(en, str(en).lower()) if isinstance(en, bool) else str(en).lower()
    if cfg.device_scorer not in ("auto", "on", "off"):
        raise ValueError("yodaRuntime.deviceScorer.enabled must be auto|on|off")
    cfg.device_index = int(_f(ds, "device", 0))
    cfg.device_min_nodes = int(_f(ds, "minNodes", 48))
    cfg.device_capacity = int(_f(ds, "capacity", 65536))
    # the engine's node fan-out threads: yodaRuntime.engineThreads, else upstream's
    # `parallelism` (v1beta2+) when the document sets it, else 1 (the benches' setting)
    cfg.engine_threads = int(_f(rt, "engineThreads", _f(doc, "parallelism", 1)))
    if cfg.engine_threads < 1 or cfg.parallelism < 1:
        raise ValueError("engineThreads and parallelism must be >= 1")
    cfg.events_api = str(_f(rt, "eventsAPI", cfg.events_api))
    if cfg.events_api not in ("events.k8s.io/v1", "v1"):
        raise ValueError("yodaRuntime.eventsAPI must be events.k8s.io/v1 or v1")
    ov = _f(rt, "overlapEngine", cfg.overlap_engine)
    cfg.overlap_engine = {True: "on", False: "off"}.get(ov, str(ov).lower()) if isinstance(ov, bool) else str(ov).lower()
    if cfg.overlap_engine not in ("auto", "on", "off"):
        raise ValueError("yodaRuntime.overlapEngine must be auto|on|off")
    cfg.overlap_depth = int(_f(rt, "overlapDepth", cfg.overlap_depth))
    cfg.scv_queueing_hint = bool(_f(rt, "scvQueueingHint", cfg.scv_queueing_hint))
    nl = _f(rt, "nativeLane", cfg.native_lane)
    cfg.native_lane = {True: "on", False: "off"}.get(nl, str(nl).lower()) if isinstance(nl, bool) else str(nl).lower()
    if cfg.native_lane not in ("auto", "on", "off"):
        raise ValueError("yodaRuntime.nativeLane must be auto|on|off")
    cfg.lane_mirror_settle_s = float(_f(rt, "laneMirrorSettleSeconds", cfg.lane_mirror_settle_s))
    if cfg.lane_mirror_settle_s < 0:
        raise ValueError("yodaRuntime.laneMirrorSettleSeconds must be >= 0")
    if not 2 <= cfg.overlap_depth <= 16:
        raise ValueError("yodaRuntime.overlapDepth must be in [2, 16]")
    cfg.trace = bool(_f(rt, "trace", False))
    for e in doc.get("extenders") or []:
        if not e.get("urlPrefix"):
            raise ValueError("extender urlPrefix is required")
        cfg.extenders.append(ExtenderConfig(
            url_prefix=str(e["urlPrefix"]).rstrip("/"), filter_verb=e.get("filterVerb", ""),
            prioritize_verb=e.get("prioritizeVerb", ""), bind_verb=e.get("bindVerb", ""),
            weight=int(e.get("weight", 1)), http_timeout=parse_duration(e.get("httpTimeout", "30s")) or 30.0,
            node_cache_capable=bool(e.get("nodeCacheCapable", False)),
            managed_resources=[(r.get("name", ""), bool(r.get("ignoredByScheduler", False)))
                               for r in e.get("managedResources") or []],
            ignorable=bool(e.get("ignorable", False))))
        if cfg.extenders[-1].prioritize_verb and cfg.extenders[-1].weight <= 0:
            raise ValueError("extender weight must be positive")
    if sum(1 for e in cfg.extenders if e.bind_verb) > 1:
        raise ValueError("only one extender can implement bind")
    if not 0 <= cfg.percentage_of_nodes_to_score <= 100:
        raise ValueError("percentageOfNodesToScore must be in [0, 100]")
    if cfg.pod_initial_backoff_seconds <= 0 or cfg.pod_max_backoff_seconds < cfg.pod_initial_backoff_seconds:
        raise ValueError("invalid pod backoff")
    profiles = doc.get("profiles") or [{}]
    names = set()
    for pd in profiles:
        name = pd.get("schedulerName") or "default-scheduler"
        if name in names:
            raise ValueError(f"duplicate profile {name!r}")
        names.add(name)
        pc = {}
        for item in pd.get("pluginConfig") or []:
            pc[item["name"]] = dict(item.get("args") or {})
        cfg.profiles.append(Profile(scheduler_name=name, plugins=merge_plugins(pd.get("plugins")), plugin_config=pc))
    qs = {tuple(p.name for p in pr.plugins["queueSort"]) for pr in cfg.profiles}
    if len(qs) > 1:
        raise ValueError("all profiles must use the same queueSort plugin")
    cfg.policy_configmap = policy_cm
    cfg.source_doc = doc
    return cfg


def apply_policy(cfg: SchedulerConfig, policy: dict) -> SchedulerConfig:
    """Re-parse ``cfg``'s document with a legacy Policy applied to its profile."""
    from . import policy as _policy
    doc = dict(cfg.source_doc or {"apiVersion": SUPPORTED_API_VERSIONS[0], "kind": "KubeSchedulerConfiguration"})
    doc.pop("algorithmSource", None)
    return parse_config(_policy.apply_to_document(doc, policy, _policy.builtin_plugin_names()))


async def resolve_policy_configmap(cfg: SchedulerConfig, client) -> SchedulerConfig:
    """Fetch a ConfigMap-held Policy (``policy.cfg`` key) and apply it."""
    if cfg.policy_configmap is None:
        return cfg
    from . import policy as _policy
    ns, name = cfg.policy_configmap
    cm = await client.get("configmaps", name, ns)
    return apply_policy(cfg, _policy.policy_from_configmap(cm))


def load_config(path: str) -> SchedulerConfig:
    with open(path) as f:
        docs = [d for d in yaml.safe_load_all(f) if d]
    for d in docs:
        if d.get("kind") == "KubeSchedulerConfiguration":
            return parse_config(d)
    # allow the ConfigMap manifest itself (deploy/yoda-scheduler.yaml)
    for d in docs:
        if d.get("kind") == "ConfigMap":
            for v in (d.get("data") or {}).values():
                inner = yaml.safe_load(v)
                if isinstance(inner, dict) and inner.get("kind") == "KubeSchedulerConfiguration":
                    return parse_config(inner)
    raise ValueError(f"{path}: no KubeSchedulerConfiguration found")


def default_config(scheduler_name: str = "default-scheduler") -> SchedulerConfig:
    return parse_config({"apiVersion": SUPPORTED_API_VERSIONS[0], "kind": "KubeSchedulerConfiguration",
                         "profiles": [{"schedulerName": scheduler_name}]})
