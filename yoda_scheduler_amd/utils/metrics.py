"""Prometheus metrics mirroring upstream kube-scheduler names plus
``yoda_gpu_*`` gauges. Each scheduler instance owns a private registry so several
instances (tests, shards) can coexist in one process.

Hot-path cost matters (a 1000-pod burst observes ~5 series per pod), so per-cycle
observations go through pre-bound label children.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

_BUCKETS = (0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30)


class SchedulerMetrics:
    def __init__(self, registry: CollectorRegistry | None = None) -> None:
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.e2e = Histogram("scheduler_e2e_scheduling_duration_seconds",
                             "E2e scheduling latency (algorithm + binding)", ["result", "profile"],
                             buckets=_BUCKETS, registry=r)
        self.algorithm = Histogram("scheduler_scheduling_algorithm_duration_seconds",
                                   "Scheduling algorithm latency", buckets=_BUCKETS, registry=r)
        self.binding = Histogram("scheduler_binding_duration_seconds", "Binding latency", buckets=_BUCKETS,
                                 registry=r)
        self.extension_point = Histogram("scheduler_framework_extension_point_duration_seconds",
                                         "Latency of running a framework extension point",
                                         ["extension_point", "status", "profile"], buckets=_BUCKETS, registry=r)
        self.attempts = Counter("scheduler_schedule_attempts_total", "Number of attempts to schedule pods",
                                ["result", "profile"], registry=r)
        self.pending = Gauge("scheduler_pending_pods", "Number of pending pods, by queue", ["queue"], registry=r)
        self.pod_scheduling = Histogram("scheduler_pod_scheduling_duration_seconds",
                                        "E2e latency for a pod being scheduled (first attempt to bound)",
                                        buckets=_BUCKETS, registry=r)
        self.pod_attempts = Histogram("scheduler_pod_scheduling_attempts", "Attempts to successfully schedule a pod",
                                      buckets=(1, 2, 4, 8, 16), registry=r)
        self.preemption_victims = Histogram("scheduler_preemption_victims", "Number of selected preemption victims",
                                            buckets=(1, 2, 4, 8, 16, 32, 64), registry=r)
        self.preemption_attempts = Counter("scheduler_preemption_attempts_total", "Total preemption attempts",
                                           registry=r)
        self.gpu_reserved = Gauge("yoda_gpu_reserved_mb", "HBM reserved by the scheduler per GPU", ["node", "gpu"],
                                  registry=r)
        self.gpu_free = Gauge("yoda_gpu_free_mb", "Sniffed free HBM per GPU", ["node", "gpu"], registry=r)
        self.scv_stale = Gauge("yoda_scv_stale", "1 if the node's Scv sample is stale", ["node"], registry=r)
        self.incoming = Counter("scheduler_queue_incoming_pods_total",
                                "Number of pods added to scheduling queues by event and queue type",
                                ["event", "queue"], registry=r)
        self.cache_size = Gauge("scheduler_scheduler_cache_size", "Number of nodes, pods, and assumed (bound) pods "
                                "in the scheduler cache", ["type"], registry=r)
        self.permit_wait = Histogram("scheduler_permit_wait_duration_seconds", "Duration of waiting on permit",
                                     ["result"], buckets=_BUCKETS, registry=r)
        self.batch_size = Histogram("yoda_native_batch_size", "Pods per native scheduling batch",
                                    buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512), registry=r)
        self._children: dict = {}

    def child(self, metric, *labels):
        key = (id(metric), labels)
        c = self._children.get(key)
        if c is None:
            c = self._children[key] = metric.labels(*labels)
        return c

    def render(self) -> bytes:
        return generate_latest(self.registry)


def _fmt_labels(d: dict) -> str:
    esc = lambda v: str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")   # noqa: E731
    return ",".join(f'{k}="{esc(v)}"' for k, v in sorted(d.items()))


def _res_value(res: str, qty) -> tuple[float, str]:
    from .quantity import bytes_of, cpu_millis, parse_quantity
    if res == "cpu":
        return cpu_millis(qty) / 1000.0, "cores"
    if res in ("memory", "ephemeral-storage") or res.startswith("hugepages-"):
        return float(bytes_of(qty)), "bytes"
    return float(parse_quantity(qty)), ""


def pod_resource_metrics(pods) -> bytes:
    """``/metrics/resources`` (upstream v1.20 ``kube_pod_resource_request`` /
    ``kube_pod_resource_limit``): the effective request/limit of every non-terminal pod —
    Σ containers, max with each init container, + overhead — labelled with namespace, pod,
    node (empty while pending), scheduler, priority, resource and unit."""
    out = ["# HELP kube_pod_resource_request Resources requested by workloads on the cluster, broken down by pod.",
           "# TYPE kube_pod_resource_request gauge",
           "# HELP kube_pod_resource_limit Resources limit for workloads on the cluster, broken down by pod.",
           "# TYPE kube_pod_resource_limit gauge"]
    for o in pods:
        spec, meta = o.get("spec") or {}, o.get("metadata") or {}
        if (o.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
            continue
        base = {"namespace": meta.get("namespace", "default"), "pod": meta.get("name", ""),
                "node": spec.get("nodeName") or "", "scheduler": spec.get("schedulerName") or "default-scheduler",
                "priority": str(spec["priority"]) if spec.get("priority") is not None else ""}
        for kind, metric in (("requests", "kube_pod_resource_request"), ("limits", "kube_pod_resource_limit")):
            tot: dict = {}
            for c in spec.get("containers") or ():
                for r, q in (((c.get("resources") or {}).get(kind)) or {}).items():
                    v, unit = _res_value(r, q)
                    tot[r] = (tot.get(r, (0.0, unit))[0] + v, unit)
            for c in spec.get("initContainers") or ():
                for r, q in (((c.get("resources") or {}).get(kind)) or {}).items():
                    v, unit = _res_value(r, q)
                    if v > tot.get(r, (0.0, unit))[0]:
                        tot[r] = (v, unit)
            if tot:
                for r, q in (spec.get("overhead") or {}).items():
                    if r in tot:
                        v, unit = _res_value(r, q)
                        tot[r] = (tot[r][0] + v, unit)
            for r in sorted(tot):
                v, unit = tot[r]
                txt = str(int(v)) if v == int(v) else repr(v)
                out.append(f"{metric}{{{_fmt_labels(dict(base, resource=r, unit=unit))}}} {txt}")
    return ("\n".join(out) + "\n").encode()


class NullMetrics:
    """Drop-in no-op for benches that want zero instrumentation overhead."""

    def __getattr__(self, name):
        setattr(self, name, _NULL)       # later lookups hit the instance dict
        return _NULL

    def child(self, metric, *labels):
        return _NULL

    def render(self) -> bytes:
        return b""


class _Null:
    def __getattr__(self, name):
        return self

    def __call__(self, *a, **k):
        return self

    # the per-pod calls, as plain methods (no __getattr__ round trip)
    def observe(self, *a, **k):
        return None

    def inc(self, *a, **k):
        return None

    def set(self, *a, **k):
        return None


_NULL = _Null()
