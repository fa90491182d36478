"""The scheduler: informers → queue → (native) scheduling cycle → assume → async bind.

Re-provides the upstream runtime the reference links against:
``scheduleOne`` semantics, 1-feasible-node shortcut, score × weight summation,
selectHost with random tie-break, assume-before-bind, bind failure → forget + requeue
with backoff, ``FailedScheduling`` diagnosis, leader election gating.

Performance design (SURVEY §7.3 hard part 2): the per-pod cycle for an all-native
profile is a single C++ call; when several pods are waiting, up to ``batchSize`` of
them are scheduled in one GIL-free ``schedule_batch`` call (each pod still sees the
reservations of the pods before it, so the outcome equals sequential cycles). Binds
run through a bounded worker pool behind the client QPS limiter.
"""
from __future__ import annotations

import asyncio
import collections
import functools
import gc
import logging
import time
from typing import Callable, Optional

from ..kube.informer import Informer, NativePodInformer
from ..models.pod import PodInfo, forget_num_id
from ..models.scv import LazyScv
from ..plugins.defaults import bind_annotations
from ..ops.native import core, pod_req
from ..utils import gctune, klog
from ..utils.metrics import SchedulerMetrics
from ..utils.ratelimit import TokenBucket
from ..utils.tracing import Tracer
from .cache import SchedulerCache
from .config import SchedulerConfig
from .events import EventRecorder
from .interfaces import CycleState, Status
from .queue import SchedulingQueue
from .registry import Registry, default_registry
from .runtime import Framework

log = logging.getLogger("yoda.scheduler")

_EMPTY_STATE = CycleState()      # shared read-only state for all-native cycles
_EMPTY_DICT: dict = {}


def _sched_cond(obj: dict) -> Optional[tuple]:
    """status.conditions' PodScheduled entry of a pod object, as ``PodEvent.sched_cond``."""
    for c in ((obj.get("status") or _EMPTY_DICT).get("conditions")) or ():
        if isinstance(c, dict) and c.get("type") == "PodScheduled":
            return (str(c.get("status") or ""), str(c.get("reason") or ""), str(c.get("message") or ""),
                    str(c.get("lastTransitionTime") or ""))
    return None
ENGINE_SWITCH_INTERVAL_S = 0.0002
POD_FIELD_SELECTOR = "status.phase!=Succeeded,status.phase!=Failed"   # upstream NewPodInformer
_VOLATILE_META = ("resourceVersion", "generation", "managedFields")


def _pod_updated(old: dict, new: dict) -> bool:
    """Upstream ``isPodUpdated``: ignore changes to status and volatile metadata, so the
    scheduler's own unschedulable-condition writes do not pull a parked pod back into
    activeQ (that would spin failing pods in a hot loop)."""
    if old.get("spec") != new.get("spec"):
        return True
    om = {k: v for k, v in (old.get("metadata") or {}).items() if k not in _VOLATILE_META}
    nm = {k: v for k, v in (new.get("metadata") or {}).items() if k not in _VOLATILE_META}
    return om != nm


def ext_text(ext) -> str:
    """FitError text of the native extended-resource fit (engine ``RS_EXT_RESOURCES``): the
    pod's requested resources beyond cpu/memory, as upstream's "Insufficient <resource>"."""
    return "Insufficient " + ("/".join(sorted(ext)) if ext else "extended resources")


SPREAD_SOURCES = ("services", "replicationcontrollers", "replicasets", "statefulsets")


def push_spread_source(engine, res: str, obj: dict, deleted: bool) -> None:
    """One DefaultSelector source object into the engine (``Engine.set_service`` /
    ``set_controller``): a Service's map selector (None = nil, matches nothing), an RC's map
    selector, a ReplicaSet's / StatefulSet's LabelSelector (plugins/optional.py::default_selector)."""
    from ..models.selectors import LabelSelector
    meta = obj.get("metadata") or {}
    ns, name = meta.get("namespace") or "default", meta.get("name", "")
    spec = obj.get("spec") or {}
    if res == "services":
        if deleted:
            engine.remove_service(ns, name)
        else:
            sel = spec.get("selector")
            engine.set_service(ns, name, None if sel is None else [(str(k), str(v)) for k, v in sel.items()])
        return
    if deleted:
        engine.remove_controller(res, ns, name)
        return
    sel = spec.get("selector")
    if res == "replicationcontrollers":
        engine.set_controller(res, ns, name, [(str(k), str(v)) for k, v in (sel or {}).items()])
    else:
        engine.set_controller(res, ns, name, None if sel is None else LabelSelector(sel).native())


class Handle:
    """``framework.Handle`` analogue handed to plugin factories."""

    def __init__(self, sched: "Scheduler") -> None:
        self._s = sched

    @property
    def client(self):
        return self._s.client

    @property
    def cache(self) -> SchedulerCache:
        return self._s.cache

    @property
    def engine(self):
        return self._s.engine

    @property
    def recorder(self) -> EventRecorder:
        return self._s.recorder

    def lister(self, res: str) -> dict:
        """Informer store (key → object) of a resource a plugin declared in ``watches``."""
        inf = self._s.informers.get(res)
        return inf.store if inf is not None else {}

    def generation(self, res: str) -> int:
        """Moves whenever an object of ``res`` (a resource some plugin ``watches``) is added,
        updated or deleted: plugins key what they derive from a whole lister on it."""
        return self._s.extra_generation[res]

    def get_waiting_pod(self, uid: str):
        for fw in self._s.frameworks.values():
            wp = fw.get_waiting_pod(uid)
            if wp is not None:
                return wp
        return None

    def iterate_waiting_pods(self):
        return [wp for fw in self._s.frameworks.values() for wp in fw.iterate_waiting_pods()]

    def preempt(self, pod: PodInfo, node: str, victims: list[PodInfo]) -> None:
        self._s._preempt(pod, node, victims)


class Scheduler:
    def __init__(self, client, config: SchedulerConfig, registry: Optional[Registry] = None, *,
                 engine_threads: int = 1, metrics=None, record_events: bool = True,
                 seed: Optional[int] = None, clock: Callable[[], float] = time.monotonic,
                 bind_limiter: Optional[TokenBucket] = None) -> None:
        self.client = client
        self.config = config
        self.registry = registry or default_registry()
        self.metrics = metrics if metrics is not None else SchedulerMetrics()
        from ..utils.metrics import NullMetrics
        self._metrics_on = not isinstance(self.metrics, NullMetrics)
        cc = config.client_connection
        # native transport: its C++ token bucket enforces clientConnection QPS/burst for
        # binds, status patches and deletes (one bucket, as client-go's limiter)
        self.native = getattr(client, "native", None) if bind_limiter is None else None
        if self.native is not None:
            client.set_rate(cc.qps, cc.burst)
            self.limiter = TokenBucket(0, 1)
        else:
            self.limiter = bind_limiter or TokenBucket(cc.qps, cc.burst)
        # where all-native runs submit their Bindings directly (no bind worker): the native
        # transport, or an in-process apiserver's synchronous binder (behind self.limiter)
        self._binds = self.native
        if self._binds is None and hasattr(client, "direct_binds"):
            self._binds = client.direct_binds()
        self.bind_timeout = float(getattr(client, "timeout", 30.0) or 30.0)
        self.recorder = EventRecorder(client, enabled=record_events, api=config.events_api)
        self.handle = Handle(self)
        # the engine must exist before plugins are created (they may query it)
        compat = any(((p.plugin_config.get("yoda") or {}).get("compat", False)) for p in config.profiles)
        stale_factor = float(next(((p.plugin_config.get("yoda") or {}).get("staleFactor", 3.0)
                                   for p in config.profiles if "yoda" in p.plugin_config), 3.0))
        self.engine = core().Engine(bool(compat), max(1, int(engine_threads), config.engine_threads))
        if seed is not None:
            self.engine.seed(seed)
        self.device_error = ""
        self._compat = bool(compat)
        self._device_checked = False
        self.engine.set_percentage_of_nodes_to_score(config.percentage_of_nodes_to_score)
        self.cache = SchedulerCache(self.engine, compat=bool(compat), stale_factor=stale_factor, clock=clock)
        self.frameworks: dict[str, Framework] = {p.scheduler_name: Framework(p, self.registry, self.handle)
                                                 for p in config.profiles}
        qs = next(iter(self.frameworks.values())).queue_sort
        self.queue = SchedulingQueue(qs.sort_key, config.pod_initial_backoff_seconds, config.pod_max_backoff_seconds,
                                     config.unschedulable_flush_seconds, clock=clock)
        self._active_fw: Optional[Framework] = None
        self._bind_dq: collections.deque = collections.deque()
        self._bind_idle: collections.deque = collections.deque()
        self._tasks: list[asyncio.Task] = []
        self._engine_exec = None          # worker thread of schedule_batch_overlapped
        self._batch_worker = None         # native engine worker (core.BatchWorker)
        self.engine_batch_errors = 0
        self._run_direct: Optional[tuple] = None   # (framework, direct_bind_mask) during _finish_run
        self._bind_buf: Optional[list] = None      # native Bindings of the run being finished
        self._bind_cbs: list = []
        self._names: dict = {}                     # engine node index → name (_node_name)
        self._dev_flush = False                    # device scorer on: idle-time row uploads
        self._dev_flush_pending = False
        self._names_gen = -1
        self._f_yoda = core().F_YODA
        self._batch_futs: dict = {}
        self.engine_spans: Optional[list] = None   # (t_start, t_end, pods) of native batches
        self._inflight: collections.deque = collections.deque()   # (fw, run, cycle, t0, future) on that worker
        self._ann_memo: dict = {}          # _bind_annotations memo, valid for one cache generation
        self._ann_gen = -1
        self.informers: dict[str, Informer] = {}
        self.extra_generation: collections.Counter = collections.Counter()   # Handle.generation
        self._scheduled = 0                # bound by the Python path (the lane counts its own)
        self.failed = 0
        self.scv_requeues = 0          # Scv updates that moved the parked pods back
        self.scv_requeue_skips = 0     # Scv updates the queueing hint kept from doing so
        self.bind_errors = 0
        self._conditions: dict = {}        # uid → the PodScheduled=False condition last written
        self._lane_attempts_seen: dict = {}   # profile → lane (scheduled, failed) already exported
        self.status_patches_skipped = 0
        self._stop = asyncio.Event()
        self.leading = asyncio.Event()
        self._pending_binds = 0
        self.lane = None                   # framework.lane.NativeLane (native transport only)
        self._lane_held = ""                      # "held": lane parked (+ mirror); "gated": lane gated
        self.batching = config.batch_size > 1
        self.tracer = Tracer() if config.trace else None
        from .extender import HTTPExtender
        self.extenders = [HTTPExtender(e) for e in config.extenders]
        # resources an extender manages with ignoredByScheduler are not fitted here (upstream)
        ignored = {n for e in config.extenders for n, ign in e.managed_resources if ign}
        for fw in self.frameworks.values():
            fit = fw.plugins.get("NodeResourcesFit")
            if ignored and fit is not None and hasattr(fit, "ignored"):
                fit.ignored |= ignored
        # optional raw samples of scheduler-internal e2e (cycle start → bind acknowledged,
        # queue wait excluded; BASELINE.md protocol item 4) without the Prometheus cost
        self.e2e_samples: Optional[list] = None
        # preemptors nominated to a node: their request is held there (over the victims
        # until those are gone) so lower-priority pods cannot take the freed capacity
        self.nominations: dict[str, tuple[str, int, float]] = {}   # uid → (node, num_id, since)
        from .debugger import CacheDebugger
        self.debugger = CacheDebugger(self)
        if isinstance(self.metrics, SchedulerMetrics):
            m = self.metrics
            self.queue.incoming_hook = lambda ev, q, n: m.child(m.incoming, ev, q).inc(n)

    # ------------------------------------------------------------------ counters (Python + lane)
    @property
    def scheduled(self) -> int:
        """Pods whose Binding the apiserver acknowledged, on either path."""
        return self._scheduled + (self.lane.lane.scheduled if self.lane is not None else 0)

    @property
    def pending_binds(self) -> int:
        """Pods placed (or queued on the native lane) whose Binding is not answered yet."""
        return self._pending_binds + (self.lane.pending() if self.lane is not None else 0)

    def take_lane_samples(self) -> None:
        """Move the lane's raw e2e samples (cycle start → Binding acknowledged) into
        ``e2e_samples`` when that list is being collected (benchmarks); drop them otherwise."""
        if self.lane is None:
            return
        xs = self.lane.lane.take_e2e()
        if self.e2e_samples is not None:
            self.e2e_samples.extend(xs)

    def lane_owned(self) -> int:
        """Pods the native lane owns (queued, in flight, binding or bound)."""
        return self.lane.owned() if self.lane is not None else 0

    def _lane_refresh(self) -> None:
        if self.lane is not None:
            self.lane.refresh()

    def _settle_lane_mirror(self) -> bool:
        """Drop the cache's mirror of lane pods (and the lane's change log with it) once no
        Python-path cycle has read it for ``laneMirrorSettleSeconds``: a burst with a few
        affinity pods must not make every later lane Binding feed a Python mirror."""
        c = self.cache
        if self.lane is None or self._lane_held:
            return False
        now, settle = c.clock(), self.config.lane_mirror_settle_s
        if c.lane_census_at is not None and now - c.lane_census_at >= settle:
            self.lane.lane.stop_census()        # the selector census, likewise
            c.lane_census_at = None
        if c.lane_synced_at is None or now - c.lane_synced_at < settle:
            return False
        c.drop_lane_mirror()
        c.lane_synced_at = None
        return True

    def _lane_cards(self, name: str) -> None:
        """The per-card device identities a lane Binding's annotations name (plugins.defaults
        .visible_device_ids), pushed whenever the node's Scv changes."""
        if self.lane is None:
            return
        scv = self.cache.scvs.get(name)
        if scv is None:
            self.lane.lane.remove_node_cards(name)
            return
        from ..models.scv import card_vis
        per = scv.card_vis() if isinstance(scv, LazyScv) else \
            card_vis([(c.id, c.uuid, c.hip_uuid, c.hip_id) for c in scv.status.card_list])
        self.lane.lane.set_node_cards(name, [(str(v), str(u or "")) for v, u in per])

    def _request_device_flush(self) -> None:
        """Released reservations dirty device rows; when nothing is being placed, upload
        them right away (coalesced per loop turn) so the next batch's launch does not carry
        them (a burst's deletions are ~1000 rows, ≈0.5 ms on the first batch of the next burst)."""
        if not self._dev_flush_pending:
            self._dev_flush_pending = True
            asyncio.get_event_loop().call_soon(self._device_flush_idle)

    def _device_flush_idle(self) -> None:
        self._dev_flush_pending = False
        if self._inflight or self.queue._active_entries:
            return                                # a batch is coming: it carries the rows
        self.engine.device_flush()

    def _maybe_enable_device(self) -> None:
        """Attach the gfx950 device scorer once the cluster is big enough for it to pay
        (``deviceScorer.minNodes``). ``auto`` uses it only when a GPU is visible and the
        library loads; ``on`` attaches at start-up and makes any failure fatal. Called after
        the informers synced and from housekeeping (clusters grow)."""
        mode = self.config.device_scorer
        if mode == "off" or self._compat or self._device_checked or self.engine.device_enabled:
            return
        nodes = self.engine.live_nodes
        if mode == "auto" and nodes < self.config.device_min_nodes:
            return
        self._device_checked = True
        try:
            from ..ops import device_scorer, hip
            if mode == "auto" and hip.device_count() <= 0:
                return
            cap = max(self.config.device_capacity, 4 * nodes)
            device_scorer.enable(self.engine, self.config.device_index, cap, self.config.device_min_nodes)
            self._dev_flush = True
            log.info("device scorer enabled on GPU %d (%d nodes, capacity %d)", self.config.device_index, nodes, cap)
        except Exception as e:  # noqa: BLE001
            self.device_error = str(e)
            if mode == "on":
                raise
            log.info("device scorer not used: %s", e)

    # ================================================================== informers
    def _responsible(self, obj: dict) -> bool:
        return ((obj.get("spec") or {}).get("schedulerName") or "default-scheduler") in self.frameworks

    @staticmethod
    def _assigned(obj: dict) -> bool:
        return bool((obj.get("spec") or {}).get("nodeName"))

    @staticmethod
    def _terminal(obj: dict) -> bool:
        return (obj.get("status") or {}).get("phase") in ("Succeeded", "Failed")

    def on_pod_add(self, obj: dict) -> None:
        spec = obj.get("spec") or _EMPTY_DICT
        if spec.get("nodeName"):
            if self.nominations:
                self._clear_nomination((obj.get("metadata") or {}).get("uid"))
            if not self._terminal(obj):
                self.cache.add_pod(obj)
        elif (spec.get("schedulerName") or "default-scheduler") in self.frameworks and not self._terminal(obj):
            self.queue.add(PodInfo.from_obj(obj))
            if self._metrics_on:
                self.metrics.child(self.metrics.incoming, "PodAdd", "active").inc()

    def on_pod_update(self, old: dict, new: dict) -> None:
        node = (new.get("spec") or _EMPTY_DICT).get("nodeName")
        if node:
            uid = new["metadata"].get("uid")
            if self._terminal(new):
                self.cache.remove_pod(uid)
                self.queue.move_all_to_active_or_backoff("AssignedPodCompleted")
                return
            if not (old.get("spec") or _EMPTY_DICT).get("nodeName"):
                # the Binding's echo (usually of our own assumed pod)
                if self._conditions:
                    self._conditions.pop(uid, None)
                self.queue.delete(uid)
                if uid in self.nominations:
                    self._clear_nomination(uid)
                ps = self.cache.pods.get(uid)
                if ps is not None and ps.assumed:
                    if self._metrics_on:
                        self.metrics.pod_scheduling.observe(max(0.0, time.monotonic() - ps.info.initial_attempt))
                        self.metrics.pod_attempts.observe(ps.info.attempts)
                    if ps.node == node:          # confirm in place (cache.add_pod's fast path)
                        ps.assumed, ps.deadline = False, None
                        ps.info.obj = new
                        return
                self.cache.add_pod(new)
            else:
                self.cache.update_pod(new)
        elif self._responsible(new) and not self._terminal(new):
            uid = new["metadata"].get("uid")
            if self.cache.is_assumed(uid):
                return   # upstream skipPodUpdate: assumed pods only get status noise
            if self._conditions and uid in self._conditions:
                self._sync_condition(uid, _sched_cond(new))
            if not _pod_updated(old, new):
                return   # status/resourceVersion-only change (e.g. our own PodScheduled=False)
            self.queue.update(PodInfo.from_obj(new))

    def on_pod_delete(self, obj: dict) -> None:
        uid = (obj.get("metadata") or {}).get("uid")
        self._conditions.pop(uid, None)
        if uid in self.nominations:
            self._clear_nomination(uid)
        if self._assigned(obj) or self.cache.is_assumed(uid):
            self.cache.remove_pod(uid)
            self.queue.move_all_to_active_or_backoff("AssignedPodDelete")
        else:
            self.queue.delete(uid)
        forget_num_id(uid)

    def on_pod_native(self, typ: str, ev, idt: tuple, old: Optional[tuple]) -> None:
        """Pod events from :class:`NativePodInformer` (C++-decoded ``PodEvent`` + its
        ident tuple): the same transitions as ``on_pod_add/update/delete`` without a dict."""
        _key, uid, node, sched, phase, h = idt
        terminal = phase == "Succeeded" or phase == "Failed"
        if self._conditions and (typ == "DELETED" or node):
            self._conditions.pop(uid, None)
        if typ == "DELETED":
            if uid in self.nominations:
                self._clear_nomination(uid)
            if node or self.cache.is_assumed(uid):
                self.cache.remove_pod(uid)
                self.queue.move_all_to_active_or_backoff("AssignedPodDelete")
                if self._dev_flush:
                    self._request_device_flush()
            else:
                self.queue.delete(uid)
            forget_num_id(uid)
            return
        if old is None:
            if node:
                if self.nominations:
                    self._clear_nomination(uid)
                if not terminal:
                    self.cache.add_pod_native(ev, uid, node)
            elif sched in self.frameworks and not terminal:
                self.queue.add(PodInfo.from_native(ev))
                if self._metrics_on:
                    self.metrics.child(self.metrics.incoming, "PodAdd", "active").inc()
            return
        oidt = old[1]
        if node:
            if terminal:
                self.cache.remove_pod(uid)
                self.queue.move_all_to_active_or_backoff("AssignedPodCompleted")
                return
            if not oidt[2]:
                # the Binding's echo (usually of our own assumed pod)
                self.queue.delete(uid)
                if uid in self.nominations:
                    self._clear_nomination(uid)
                ps = self.cache.pods.get(uid)
                if ps is not None and ps.assumed:
                    if self._metrics_on:
                        self.metrics.pod_scheduling.observe(max(0.0, time.monotonic() - ps.info.initial_attempt))
                        self.metrics.pod_attempts.observe(ps.info.attempts)
                    if ps.node == node:          # confirm in place (cache.add_pod_native's fast path)
                        ps.assumed, ps.deadline = False, None
                        ps.info.set_source(ev)
                        return
                self.cache.add_pod_native(ev, uid, node)
            else:
                self.cache.update_pod_native(ev, uid, node, oidt[5] == h)
        elif sched in self.frameworks and not terminal:
            if self.cache.is_assumed(uid):
                return   # upstream skipPodUpdate
            if self._conditions and uid in self._conditions:
                self._sync_condition(uid, ev.sched_cond)
            if oidt[5] == h:
                return   # status/resourceVersion-only change
            self.queue.update(PodInfo.from_native(ev))

    def on_node_add(self, obj: dict) -> None:
        self.cache.add_node(obj)
        if self.lane is not None:
            self.lane.node_event((obj.get("metadata") or {}).get("name", ""))
        self.queue.move_all_to_active_or_backoff("NodeAdd")
        self._lane_refresh()

    def on_node_update(self, old: dict, new: dict) -> None:
        self.cache.update_node(new)
        if self.lane is not None:
            self.lane.node_event((new.get("metadata") or {}).get("name", ""))
        self._lane_refresh()
        if old.get("spec") != new.get("spec") or (old.get("metadata") or {}).get("labels") != \
                (new.get("metadata") or {}).get("labels") or (old.get("status") or {}).get("allocatable") != \
                (new.get("status") or {}).get("allocatable"):
            self.queue.move_all_to_active_or_backoff("NodeUpdate")

    def on_node_delete(self, obj: dict) -> None:
        self.cache.remove_node(obj["metadata"]["name"])
        if self.lane is not None:
            self.lane.node_event(obj["metadata"]["name"])
        self._lane_refresh()

    def on_scv(self, obj: dict) -> None:
        self.cache.add_scv(obj)
        self._lane_cards((obj.get("metadata") or {}).get("name", ""))
        self.queue.move_all_to_active_or_backoff("ScvAdd")

    def _capacity(self, name: str) -> Optional[tuple]:
        """What the yoda filter can see of a node's GPUs — read from the engine's own filter
        inputs (``Engine::filter_view``, next to ``yoda_filter``), so the hint cannot drift
        from the filter: (unfit: no Scv or stale, CardNumber, per card (healthy, free,
        effective free, clock)); None for a node the engine does not know."""
        idx = self.engine.node_index(name)
        v = self.engine.filter_view(idx) if idx >= 0 else None
        if v is None:
            return None
        has_scv, stale, cn, cards = v
        return bool(stale or not has_scv), cn, tuple(tuple(c) for c in cards)

    @staticmethod
    def _capacity_grew(b: tuple, a: tuple) -> bool:
        """Can a pod that failed the yoda filter against ``b`` pass against ``a``? The
        filter is monotone in health, free / effective-free HBM, card count and freshness,
        and matches the clock exactly, so: anything up, or any clock different."""
        if (b[0] and not a[0]) or a[1] > b[1] or len(a[2]) > len(b[2]):
            return True
        for (hb, fb, eb, cb), (ha, fa, ea, ca) in zip(b[2], a[2]):
            if (ha and not hb) or fa > fb or ea > eb or ca != cb:
                return True
        return False

    def on_scv_update(self, old: dict, new: dict) -> None:
        """Queueing hint for Scv updates (upstream v1.22+ QueueingHint, applied to the
        telemetry CRD): the update is applied to the cache, and parked pods are moved back
        only when the node's filter-visible capacity grew. A steady stream of telemetry that
        only records load then costs one cache update per event, not a retry of every
        parked pod (``scv_requeues`` / ``scv_requeue_skips`` count both outcomes)."""
        if not self.config.scv_queueing_hint:
            self.cache.add_scv(new)
            self._lane_cards((new.get("metadata") or {}).get("name", ""))
            self.queue.move_all_to_active_or_backoff("ScvUpdate")
            self.scv_requeues += 1
            return
        name = (new.get("metadata") or {}).get("name", "")
        before = self._capacity(name)
        self.cache.add_scv(new)
        self._lane_cards(name)
        after = self._capacity(name)
        if before is None or after is None:
            self.queue.move_all_to_active_or_backoff("ScvUpdate")
            self.scv_requeues += 1
        elif self._capacity_grew(before, after):
            if self.lane is not None:
                self.lane.move_node(self.engine.node_index(name))
            # per pod (upstream QueueingHint): only pods whose GPU request the node's new
            # capacity satisfies can now pass the yoda filter there; other filters do not
            # read Scv, so a pod they rejected on this node stays rejected
            compat = self.cache.compat
            self.queue.move_matching_to_active_or_backoff(lambda pi: self._gpu_fits(pi, after, compat), "ScvUpdate")
            self.scv_requeues += 1
        else:
            self.scv_requeue_skips += 1

    @staticmethod
    def _gpu_fits(pi: PodInfo, cap: tuple, compat: bool) -> bool:
        """Would ``pi`` pass the yoda filter (filter.go PodFitsNumber / PodFitsMemory /
        PodFitsClock, plus the MI355X freshness and clock-floor rules) on a node with
        capacity ``cap`` (see ``_capacity``)?"""
        stale, card_number, cards = cap
        g = pi.gpu
        if stale and not compat:
            return False
        if g.has_number:
            if g.number > card_number:
                return False
        elif card_number <= 0:
            return False
        fit = 0
        for h, free, eff, clock in cards:
            if h and (free if compat else eff) >= g.memory and (not g.has_clock or clock == g.clock) \
                    and clock >= g.clock_min:
                fit += 1
        return fit >= g.number

    def on_scv_delete(self, obj: dict) -> None:
        self.cache.remove_scv(obj["metadata"]["name"])
        self._lane_cards(obj["metadata"]["name"])

    def make_informers(self) -> dict[str, Informer]:
        self.informers = {
            "nodes": Informer(self.client, "nodes", self.on_node_add, self.on_node_update, self.on_node_delete),
            "scvs": Informer(self.client, "scvs", self.on_scv, self.on_scv_update, self.on_scv_delete),
            # upstream v1.20 scheduler pod informer: terminal pods are filtered by the apiserver
            "pods": (NativePodInformer(self.client, self.on_pod_native, field_selector=POD_FIELD_SELECTOR,
                                       lane=self._make_lane())
                     if self.native is not None else
                     Informer(self.client, "pods", self.on_pod_add, self.on_pod_update, self.on_pod_delete,
                              field_selector=POD_FIELD_SELECTOR)),
        }
        # objects only some plugins need (PVCs, PVs, StorageClasses, CSINodes): watched when
        # an enabled plugin declares them; any change may make a parked pod schedulable
        extra = sorted({r for fw in self.frameworks.values() for p in fw.plugins.values()
                        if not getattr(p, "inert", False) for r in getattr(p, "watches", ())})
        for res in extra:
            ev = f"{res}Change"
            if res in SPREAD_SOURCES:
                # DefaultSelector sources: the engine keeps them (native PodTopologySpread)
                self.informers[res] = Informer(
                    self.client, res,
                    lambda o, ev=ev, res=res: self._spread_source(res, o, False, ev),
                    lambda a, b, ev=ev, res=res: self._spread_source(res, b, False, ev),
                    lambda o, ev=ev, res=res: self._spread_source(res, o, True, None))
                continue
            self.informers[res] = Informer(self.client, res,
                                           lambda o, ev=ev, res=res: self._extra_event(ev, res, o),
                                           lambda a, b, ev=ev, res=res: self._extra_event(ev, res, b),
                                           lambda o, res=res: self._extra_event(None, res, o))
        return self.informers

    def _extra_event(self, ev: Optional[str], res: str = "", obj: Optional[dict] = None) -> None:
        if res:
            self.extra_generation[res] += 1
            if obj is not None and self.lane is not None:
                self.lane.claims_event(res, obj)
        if ev is not None:
            self.queue.move_all_to_active_or_backoff(ev)
        self._lane_refresh()

    def _spread_source(self, res: str, obj: dict, deleted: bool, ev: Optional[str]) -> None:
        """A Service / RC / ReplicaSet / StatefulSet changed: the engine's DefaultSelector
        sources follow (upstream helper.DefaultSelector reads them through listers)."""
        push_spread_source(self.engine, res, obj, deleted)
        if ev is not None:
            self._extra_event(ev)
        else:
            self._lane_refresh()

    def _make_lane(self):
        """The native pod lane when the transport is native and ``yodaRuntime.nativeLane``
        allows it; returns the ``core.Lane`` for the pod informer (or None)."""
        if self.native is None or self.config.native_lane == "off" or self.lane is not None:
            return self.lane.lane if self.lane is not None else None
        from .lane import NativeLane
        self.lane = NativeLane(self, self.native)
        self.cache.lane = self.lane.lane
        self.cache.on_anti_change = self.lane.anti_changed
        return self.lane.lane

    # ================================================================== cycle
    def _activate(self, fw: Framework) -> None:
        if self._active_fw is not fw:
            fw.apply(self.engine)
            self._active_fw = fw

    def _pod_gone(self, pi: PodInfo) -> bool:
        inf = self.informers.get("pods")
        if inf is None:
            return False
        if self.native is not None:
            e = inf.entries.get(pi.key)
            return e is None or e[1][1] != pi.uid or bool(e[1][2])
        cur = inf.store.get(pi.key)
        return cur is None or cur["metadata"].get("uid") != pi.uid or self._assigned(cur)

    def schedule_one(self, pi: PodInfo) -> None:
        fw = self.frameworks.get(pi.scheduler_name)
        memo = pi.applies_memo
        if fw is None or self._pod_gone(pi):
            if memo is not None and memo.get("_adopt"):
                pi.applies_memo = None
            return
        if memo is None or memo.get("_adopt"):
            # (a memo _batch_runs started for this pod, with nothing run in between, is adopted)
            with fw.memo_cycle(pi):
                return self.schedule_one(pi)
        if self.lane is not None and not fw.native_for(pi) and not self._lane_held:
            # Python plugins read other pods, lane pods included. Either the lane is gated — it
            # takes no pod the cycle's plugins are sensitive to (a pod matching this pod's
            # anti-affinity terms or spread selectors) and keeps placing the others — or, when a
            # plugin cannot declare that, parked (and mirrored) for the whole cycle, as upstream's
            # serial scheduleOne: either way no lane pod this pod's filters would have rejected
            # can be placed between their view of the cluster and this pod's assume
            mirror = fw.needs_lane_mirror(pi, self.cache.lane_never_flags)
            terms = None if mirror else fw.own_gate_terms(pi)
            self._lane_held = "held" if terms is None else "gated"
            try:
                with (self.lane.held(sync=mirror) if terms is None else self.lane.gated(terms)):
                    return self.schedule_one(pi)
            finally:
                self._lane_held = ""
        self._clear_nominations_for((pi,))       # the preemptor competes with its own hold gone
        self._activate(fw)
        cycle = self.queue.scheduling_cycle
        t0 = time.perf_counter()
        state = CycleState()
        if fw.native_for(pi):
            res = self.engine.schedule(pi.num_id, pod_req(self.engine, pi), True)
        else:
            res = self._hybrid_cycle(fw, state, pi)
            if res is None:
                return
        self._finish_cycle(fw, state, pi, res, cycle, t0)
        if self.tracer is not None:
            tr = self.tracer
            tr.span("cycle", tr.now_us() - (time.perf_counter() - t0) * 1e6, pod=pi.key, node=res[0],
                    feasible=res[1], native=fw.native_for(pi))

    def _hybrid_cycle(self, fw: Framework, state: CycleState, pi: PodInfo):
        pre = self._hybrid_filter(fw, state, pi)
        if pre is None:
            return None
        return self._hybrid_finish(fw, state, pi, *pre)

    async def schedule_one_async(self, pi: PodInfo) -> None:
        """The cycle with HTTP extenders: framework filters, then every interested
        extender's filter (in config order), then Python + extender priorities on top of
        the native scores."""
        from .extender import ExtenderError, run_extenders
        fw = self.frameworks.get(pi.scheduler_name)
        if fw is None or self._pod_gone(pi):
            return
        if self.lane is not None:
            self.cache.sync_lane()
        self._clear_nominations_for((pi,))
        self._activate(fw)
        cycle = self.queue.scheduling_cycle
        t0 = time.perf_counter()
        state = CycleState()
        pre = self._hybrid_filter(fw, state, pi)
        if pre is None:
            return
        req, feas_idx, reasons, failed = pre
        names = [self.engine.node_name(i) for i in feas_idx]
        node_objs = {n: self.cache.nodes[n].obj for n in names if n in self.cache.nodes}
        try:
            keep, ext_failed, ext_scores = await run_extenders(self.extenders, pi, names, node_objs)
        except ExtenderError as e:
            self._fail(fw, state, pi, cycle, f"extender: {e}", t0, unschedulable=False)
            return
        self._activate(fw)               # other cycles may have run while awaiting
        for n, why in ext_failed.items():
            failed[n] = Status.unschedulable(why or "node(s) rejected by an extender")
        keep_set = set(keep)
        feas_idx = [i for i, n in zip(feas_idx, names) if n in keep_set]
        res = self._hybrid_finish(fw, state, pi, req, feas_idx, reasons, failed, ext_scores)
        if res is not None:
            self._finish_cycle(fw, state, pi, res, cycle, t0)

    def _hybrid_filter(self, fw: Framework, state: CycleState, pi: PodInfo):
        st = fw.run_pre_filter(state, pi)
        if not st.is_success():
            self._fail(fw, state, pi, self.queue.scheduling_cycle, f"0/{self.engine.live_nodes} nodes are available: "
                       f"{st.message()}", time.perf_counter())
            return None
        req = pod_req(self.engine, pi)
        eng = self.engine
        if fw.has_active_filter_py(pi):
            # percentageOfNodesToScore must sample nodes that pass ALL filters (upstream runs
            # every filter plugin inside the same search): take every native-feasible node,
            # let the Python filters stop at numFeasibleNodesToFind
            feas_idx, reasons = eng.feasible_nodes(req, [], True)
            limit = eng.num_feasible_to_find(eng.live_nodes)
        else:
            feas_idx, reasons = eng.feasible_nodes(req, [])
            limit = None
        names = [eng.node_name(i) for i in feas_idx]
        names2, failed = fw.run_filter_py(state, pi, names, limit)
        if len(names2) != len(names):
            keep = set(names2)
            feas_idx = [i for i, n in zip(feas_idx, names) if n in keep]
        return req, feas_idx, reasons, failed

    def _hybrid_finish(self, fw: Framework, state: CycleState, pi: PodInfo, req, feas_idx, reasons, failed,
                       ext_scores: Optional[dict] = None):
        if not feas_idx:
            # the engine's cycle tuple (node, feasible, evaluated, cards, score, reasons,
            # gang quality, node gen, stale) + the Python filters' statuses
            return (-1, 0, self.engine.live_nodes, [], 0, list(reasons), 0, 0, False, failed, len(failed))
        names = [self.engine.node_name(i) for i in feas_idx]
        extra = fw.run_score_py(state, pi, names) if (len(names) > 1 and fw.score_py) else []
        if ext_scores:
            extra = [(extra[k] if extra else 0) + ext_scores.get(n, 0) for k, n in enumerate(names)]
        return self.engine.schedule(pi.num_id, req, True, feas_idx, extra)

    def _finish_cycle(self, fw: Framework, state: CycleState, pi: PodInfo, res, cycle: int, t0: float) -> None:
        node_idx = res[0]
        m = self.metrics
        if node_idx < 0:
            if res[8] is True:
                # the device placed the pod on a node deleted meanwhile: retry, not unschedulable
                self._fail(fw, state, pi, cycle, "the selected node was removed during the cycle", t0,
                           unschedulable=False)
                return
            msg = self._fit_error(res, pi)
            self._fail(fw, state, pi, cycle, msg, t0)
            return
        node, gen = self._node_name(node_idx)
        if gen != res[7]:
            # the slot's node was removed (its reservations with it) or replaced by another
            # node between the engine cycle and now: binding there would skip every filter
            self.engine.release(pi.num_id)
            self._fail(fw, state, pi, cycle, "the selected node was removed before the binding", t0,
                       unschedulable=False)
            return
        cards = res[3]
        self.cache.assumed(pi, node, cards)
        pi.assigned_cards = cards if (fw.filter_mask & self._f_yoda) else None
        if fw.reserve and state is not None and (fw.reserve_static or not fw.native_for(pi)):
            st = fw.run_reserve(state, pi, node)
            if not st.is_success():
                self.cache.forget(pi)
                self._fail(fw, state, pi, cycle, st.message(), t0, unschedulable=False)
                return
        waiting = False
        if fw.permit and state is not None:
            st, _wait = fw.run_permit(state, pi, node)
            waiting = st.code.name == "WAIT"
            if not st.is_success() and not waiting:
                fw.run_unreserve(state, pi, node)
                self.cache.forget(pi)
                self._fail(fw, state, pi, cycle, st.message(), t0, unschedulable=st.is_unschedulable())
                return
        if self._metrics_on:
            m.algorithm.observe(time.perf_counter() - t0)
            m.child(m.attempts, "scheduled", fw.name).inc()
        if klog.V(3):
            log.info("pod %s → node %s gpus=%s score=%d feasible=%d", pi.key, node, cards, res[4], res[1])
        self._pending_binds += 1
        if waiting:       # held at Permit: its own task waits, then hands it to the binders
            asyncio.get_event_loop().create_task(self._permit_then_bind((fw, state, pi, node, cycle, t0)))
        else:
            self._enqueue_bind((fw, state, pi, node, cycle, t0))

    def _node_name(self, idx: int) -> tuple:
        """Engine node index → (name, slot generation), memoised until a node is added or
        removed. A cycle result whose generation differs names a slot that was freed (and
        maybe reused by another node) after the engine placed the pod."""
        if self._names_gen != self.cache.node_generation:
            self._names.clear()
            self._names_gen = self.cache.node_generation
        ng = self._names.get(idx)
        if ng is None:
            ng = self._names[idx] = (self.engine.node_name(idx), self.engine.node_gen(idx))
        return ng

    async def _permit_then_bind(self, item: tuple) -> None:
        fw, state, pi, node, cycle, t0 = item
        tw = time.perf_counter()
        st = await fw.wait_on_permit(pi)
        self.metrics.child(self.metrics.permit_wait, "Success" if st.is_success() else "Unschedulable").observe(
            time.perf_counter() - tw)
        if st.is_success():
            self._enqueue_bind(item)
            return
        self._pending_binds -= 1
        fw.run_unreserve(state, pi, node)
        self.cache.forget(pi)
        self.failed += 1
        self.recorder.pod_event(pi, "Warning", "FailedScheduling", st.message())
        self.queue.add_unschedulable(pi, cycle, unschedulable=True)

    def _fit_error(self, res, pi: Optional[PodInfo] = None) -> str:
        reasons = res[5]
        names = core().REASONS
        text = {"NodeUnschedulable": "node(s) were unschedulable", "NodeName": "node(s) didn't match the requested node name",
                "TaintToleration": "node(s) had taints that the pod didn't tolerate",
                "NodeAffinity": "node(s) didn't match node selector", "NodeResourcesFit": "Insufficient cpu/memory/pods",
                "NoScv": "node(s) have no Scv telemetry", "ScvStale": "node(s) have stale Scv telemetry",
                "GpuNumber": "node(s) have too few GPUs", "GpuMemory": "node(s) have too few GPUs with enough free HBM",
                "GpuClock": "node(s) have too few GPUs with the requested clock",
                "GpuFit": "node(s) have too few healthy GPUs matching scv/memory+scv/clock",
                "NodeResourcesFitExtended": ext_text(pi.ext if pi is not None else None),
                "PodTopologySpread": "node(s) didn't match pod topology spread constraints",
                "PodTopologySpreadLabel": "node(s) didn't match pod topology spread constraints (missing required label)",
                "InterPodAffinityExisting": "node(s) didn't satisfy existing pods anti-affinity rules",
                "InterPodAffinity": "node(s) didn't match pod affinity rules",
                "InterPodAntiAffinity": "node(s) didn't match pod anti-affinity rules",
                "NodePorts": "node(s) didn't have free ports for the requested pod ports",
                "VolumeBinding": "node(s) had volume node affinity conflict",
                "VolumeZone": "node(s) had no available volume zone"}
        parts = [f"{c} {text.get(names[i], names[i])}" for i, c in enumerate(reasons) if c and i]
        if len(res) > 10 and res[10]:
            by_msg: dict[str, int] = {}
            for st in res[9].values():
                by_msg[st.message() or "node(s) rejected by out-of-tree filters"] = \
                    by_msg.get(st.message() or "node(s) rejected by out-of-tree filters", 0) + 1
            parts.extend(f"{c} {m}" for m, c in by_msg.items())
        return f"0/{res[2]} nodes are available: " + ", ".join(sorted(parts)) + "."

    def _fail(self, fw: Framework, state: CycleState, pi: PodInfo, cycle: int, msg: str, t0: float,
              unschedulable: bool = True) -> None:
        m = self.metrics
        self.failed += 1
        nominated = ""
        if state is None:
            state = CycleState()
        if unschedulable and fw.post_filter:
            if self.lane is not None and self._lane_held != "held" and pi.priority > self.lane.preempt_above(fw):
                prev = self._lane_held
                self._lane_held = "held"
                # park the lane for the ledger what-ifs; mirror lane pods only for a Python
                # what-if (the native search reads the ledger, which holds them)
                sync = any(getattr(p, "needs_mirror", lambda _pod: True)(pi) for p in fw.post_filter)
                try:
                    with self.lane.held(sync=sync):
                        return self._fail(fw, state, pi, cycle, msg, t0, unschedulable)
                finally:
                    self._lane_held = prev
            for p in fw.post_filter:
                try:
                    r, st = p.post_filter(state, pi, {})
                except Exception as e:  # noqa: BLE001
                    log.warning("postFilter %s failed: %r", getattr(p, "name", p), e)
                    continue
                if st.is_success() and r is not None and r.nominated_node:
                    nominated = r.nominated_node
                    self._nominate(pi, nominated, r.cards or [])
                    break
        m.child(m.attempts, "unschedulable" if unschedulable else "error", fw.name).inc()
        m.algorithm.observe(time.perf_counter() - t0)
        self.recorder.pod_event(pi, "Warning", "FailedScheduling", msg)
        if klog.V(2):
            log.info("unable to schedule %s: %s", pi.key, msg)
        self.queue.add_unschedulable(pi, cycle, unschedulable)
        asyncio.get_event_loop().create_task(self._update_condition(pi, msg, nominated))

    def _sync_condition(self, uid: str, cond: Optional[tuple]) -> None:
        """A pending pod's PodScheduled condition as its latest update shows it ((status, reason,
        message, lastTransitionTime) or None): what ``_condition_patch`` compares with next, as
        upstream compares with the informer's pod. None (not echoed yet) keeps what was written."""
        if cond is None:
            return
        prev = self._conditions.get(uid)
        if cond[0] == "False":
            self._conditions[uid] = (cond[1], cond[2], cond[3], prev[3] if prev else "")
        else:                       # another status: the next write is a transition
            self._conditions.pop(uid, None)

    def _condition_patch(self, pi: PodInfo, msg: str, nominated: str) -> Optional[dict]:
        """upstream v1.20 ``updatePod`` + ``podutil.UpdatePodCondition``: the PodScheduled=False
        condition as a strategic merge patch of pods/status, or None when the pod already says
        the same (same status, reason and message, no new nominated node) — then nothing is
        written. lastTransitionTime is set when the condition first appears and kept while its
        status stays False. What the pod "already says" is its condition as its latest update
        showed it (``_sync_condition``), else what this scheduler last wrote for it (until the
        write's echo arrives), or the condition on the pod object when that is already decoded
        (a condition a previous scheduler instance wrote)."""
        prev = self._conditions.get(pi.uid)
        if prev is None and pi._obj is not None:
            for c in ((pi._obj.get("status") or {}).get("conditions")) or ():
                if isinstance(c, dict) and c.get("type") == "PodScheduled" and c.get("status") == "False":
                    prev = (c.get("reason"), c.get("message"), c.get("lastTransitionTime"),
                            (pi._obj.get("status") or {}).get("nominatedNodeName") or "")
        if prev is not None and prev[0] == "Unschedulable" and prev[1] == msg and (not nominated or prev[3] == nominated):
            self.status_patches_skipped += 1
            return None
        ltt = prev[2] if prev is not None and prev[2] else time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        self._conditions[pi.uid] = ("Unschedulable", msg, ltt, nominated or (prev[3] if prev else ""))
        patch = {"status": {"conditions": [{"type": "PodScheduled", "status": "False", "lastProbeTime": None,
                                            "lastTransitionTime": ltt, "reason": "Unschedulable", "message": msg}]}}
        if nominated:
            patch["status"]["nominatedNodeName"] = nominated
        return patch

    async def _update_condition(self, pi: PodInfo, msg: str, nominated: str) -> None:
        patch = self._condition_patch(pi, msg, nominated)
        if patch is None:
            return
        try:
            if self.native is not None:
                await self.client.patch("pods", pi.name, patch, pi.namespace, limited=True, strategic=True)
            else:
                await self.limiter.acquire()
                await self.client.patch("pods", pi.name, patch, pi.namespace, strategic=True)
        except Exception as e:  # noqa: BLE001 - best effort like upstream
            log.debug("condition update for %s failed: %r", pi.key, e)

    def _nominate(self, pi: PodInfo, node: str, cards: list) -> None:
        self._clear_nomination(pi.uid)
        idx = self.engine.node_index(node)
        if idx >= 0 and self.engine.reserve(pi.num_id, pod_req(self.engine, pi), idx, list(cards)):
            self.nominations[pi.uid] = (node, pi.num_id, time.monotonic())

    def _clear_nomination(self, uid: str) -> None:
        nom = self.nominations.pop(uid, None)
        if nom is not None:
            self.engine.release(nom[1])
            # pods parked while the hold stood may fit now: the preemptor need not retake the
            # same cards (or any, on that node), and no other cluster event reports the release
            self.queue.move_all_to_active_or_backoff("NominatedPodRelease")

    def _clear_nominations_for(self, pods) -> None:
        if self.nominations:
            for p in pods:
                if p.uid in self.nominations:
                    self._clear_nomination(p.uid)

    def _preempt(self, pod: PodInfo, node: str, victims: list[PodInfo]) -> None:
        self.metrics.preemption_attempts.inc()
        self.metrics.preemption_victims.observe(len(victims))
        for v in victims:
            self.recorder.pod_event(v, "Normal", "Preempted", f"Preempted by {pod.key} on node {node}", related=pod)
            asyncio.get_event_loop().create_task(self._delete_victim(v))

    async def _delete_victim(self, v: PodInfo) -> None:
        try:
            if self.native is not None:
                await self.client.delete("pods", v.name, v.namespace, limited=True)
            else:
                await self.limiter.acquire()
                await self.client.delete("pods", v.name, v.namespace)
        except Exception as e:  # noqa: BLE001
            log.warning("preemption: deleting %s failed: %r", v.key, e)

    # ================================================================== batch cycle
    def _batch_runs(self, pods: list[PodInfo], adopt: bool = False):
        """Split popped pods into single Python cycles (``(None, pod)``) and runs of
        consecutive pods of an all-native profile (``(fw, [pods])``). ``adopt``: the consumer
        runs each single cycle right after it is yielded (no await in between), so the plugin
        applicability computed here for a flagged pod is handed to its cycle's memo."""
        i = 0
        masks: dict = {}           # framework → native_mask(), once per batch
        while i < len(pods):
            p = pods[i]
            fw = self.frameworks.get(p.scheduler_name)
            if fw is not None and fw not in masks:
                masks[fw] = fw.native_mask()
            m = masks.get(fw)
            masked = m is not None and not (p.flags & m)
            if adopt and fw is not None and not masked and p.applies_memo is None:
                p.applies_memo = {"_adopt": True}
            # the mask settles the common case; flagged pods still get the per-plugin check
            if fw is None or not (masked or fw.native_for(p)):
                yield None, p
                i += 1
                continue
            if p.applies_memo is not None and p.applies_memo.get("_adopt"):
                p.applies_memo = None
            j = i
            run = []
            while j < len(pods) and pods[j].scheduler_name == fw.name and \
                    ((m is not None and not (pods[j].flags & m)) or fw.native_for(pods[j])):
                if not self._pod_gone(pods[j]):
                    run.append(pods[j])
                j += 1
            i = j
            if run:
                yield fw, run

    def _prepare_run(self, fw: Framework, run: list[PodInfo]):
        self._activate(fw)
        self._clear_nominations_for(run)
        eng = self.engine
        return self.queue.scheduling_cycle, time.perf_counter(), [p.num_id for p in run], \
            [pod_req(eng, p) for p in run]

    def _finish_run(self, fw: Framework, run: list[PodInfo], results, cycle: int, t0: float) -> None:
        self.metrics.batch_size.observe(len(run))
        if self.tracer is not None:
            tr = self.tracer
            tr.span("native_batch", tr.now_us() - (time.perf_counter() - t0) * 1e6, pods=len(run),
                    device_cycles=self.engine.device_cycles)
        # the direct-bind decision's plugin checks, once for the run (see _native_direct)
        binder = fw.bind_plugins[0] if len(fw.bind_plugins) == 1 else None
        if not self.extenders and binder is not None and getattr(binder, "native_bind", False):
            self._run_direct = (fw, fw.direct_bind_mask())
        # the run's native Bindings go to the transport in one hand-off at the end
        buf = self._bind_buf = [] if self._binds is not None else None
        try:
            for p, res in zip(run, results):
                self._finish_cycle(fw, None, p, res, cycle, t0)   # all-native: no Python state
        finally:
            self._run_direct = None
            if buf is not None:
                self._bind_buf = None
                cbs, self._bind_cbs = self._bind_cbs, []
                if buf:
                    try:
                        self._binds.bind_many(buf, cbs, self.bind_timeout)
                    except Exception as e:  # noqa: BLE001 - the run's pods must not stay assumed
                        log.error("handing %d Bindings to the transport failed: %r", len(buf), e)
                        msg = repr(e).encode()
                        for cb in cbs:              # each goes through the bind-failure path
                            cb(-1, msg)

    def schedule_batch(self, pods: list[PodInfo]) -> None:
        """Schedule a run of popped pods; consecutive pods of an all-native profile go
        through one GIL-free engine call."""
        for fw, item in self._batch_runs(pods, adopt=True):
            if fw is None:
                self.schedule_one(item)
                continue
            cycle, t0, ids, reqs = self._prepare_run(fw, item)
            try:
                results = self.engine.schedule_batch(ids, reqs)
            except Exception as e:  # noqa: BLE001 - as _finish_inflight_run
                self._engine_batch_failed(item, cycle, e)
                continue
            self._finish_run(fw, item, results, cycle, t0)

    def _overlap(self) -> bool:
        mode = self.config.overlap_engine
        return mode == "on" or (mode == "auto" and self.engine.device_enabled and
                                self.engine.live_nodes >= self.config.device_min_nodes)

    async def schedule_batch_overlapped(self, pods: list[PodInfo]) -> None:
        """``schedule_batch`` as a pipeline: each native run goes to the engine worker
        thread, and older runs are finished (assumed into the cache, binds enqueued) while
        the engine — with the device scorer, the GPU — places the newer ones. Up to
        ``yodaRuntime.overlapDepth`` runs are in flight, so the engine keeps a run queued
        while the event loop catches up with binds and watch events. The event loop
        meanwhile keeps binding and ingesting informer events. The engine already reserved
        every returned placement in its own ledger, so a run can be placed before Python has
        applied the previous runs' results; those are applied in order. The engine's
        process-wide lock (native/core/bindings.cpp) serialises any engine call the loop
        makes meanwhile. Runs left in flight are finished when the queue runs dry
        (``finish_inflight``)."""
        loop = asyncio.get_event_loop()
        depth = self.config.overlap_depth
        for fw, item in self._batch_runs(pods):
            if fw is None:
                await self.finish_inflight()
                self.schedule_one(item)
                continue
            cycle, t0, ids, reqs = self._prepare_run(fw, item)
            fut = self._submit_engine_batch(loop, ids, reqs)
            self._inflight.append((fw, item, cycle, t0, fut, reqs))
            while len(self._inflight) >= depth:
                await self._finish_inflight_run(self._inflight.popleft())

    def _submit_engine_batch(self, loop, ids: list, reqs: list) -> asyncio.Future:
        """Hand a batch to the engine's native worker thread (``BatchWorker``: no GIL on that
        thread, results converted here when collected); an engine that is not the native
        class (test doubles) goes to a Python executor thread instead."""
        Engine = core().Engine
        if isinstance(self.engine, Engine):
            if self._batch_worker is None:
                self._batch_worker = core().BatchWorker(self.engine)
                loop.add_reader(self._batch_worker.fileno(), self._collect_engine_batches)
            fut = loop.create_future()
            self._batch_futs[self._batch_worker.submit(ids, reqs)] = fut
            return fut
        if self._engine_exec is None:
            import concurrent.futures
            import sys
            self._engine_exec = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix="yoda-engine")
            # the worker re-takes the GIL to hand back each batch's results; with the
            # default 5 ms switch interval it waits that long behind the busy event loop
            # (measured: +7 µs per pod on MI355X config 6), so ask for 0.2 ms
            sys.setswitchinterval(min(sys.getswitchinterval(), ENGINE_SWITCH_INTERVAL_S))
        return loop.run_in_executor(self._engine_exec, self.engine.schedule_batch, ids, reqs)

    def _collect_engine_batches(self) -> None:
        for jid, res, err, ts, te in self._batch_worker.collect():
            fut = self._batch_futs.pop(jid, None)
            if self.engine_spans is not None:
                self.engine_spans.append((ts, te, len(res) if res is not None else 0))
            if fut is None or fut.done():
                continue
            if err is not None:
                fut.set_exception(RuntimeError(f"engine batch failed: {err}"))
            else:
                fut.set_result(res)

    async def _finish_inflight_run(self, run: tuple) -> None:
        fw, item, cycle, t0, fut = run[:5]
        try:
            results = await fut
        except asyncio.CancelledError:
            raise
        except Exception as e:  # noqa: BLE001 - a failed engine batch must not stop the loop
            self._engine_batch_failed(item, cycle, e)
            return
        self._finish_run(fw, item, results, cycle, t0)

    def _engine_batch_failed(self, item: list, cycle: int, e: Exception) -> None:
        """Drop whatever the engine may have reserved for the run and retry its pods from
        backoff (an error, not "unschedulable")."""
        self.engine_batch_errors += 1
        log.error("engine batch of %d pods failed: %r; pods go back to the queue", len(item), e)
        for p in item:
            self.engine.release(p.num_id)
            self.queue.add_unschedulable(p, cycle, unschedulable=False)

    async def _await_pods_or_result(self) -> None:
        """Wait until the oldest in-flight run's result lands (then apply it) or a pod reaches
        the active queue, whichever is first."""
        fut = self._inflight[0][4]
        if not fut.done():
            q = self.queue
            wake = asyncio.get_event_loop().create_future()

            def on_result(_f, wake=wake) -> None:
                if not wake.done():
                    wake.set_result(None)
            q.wake = wake
            fut.add_done_callback(on_result)
            try:
                await wake
            finally:
                q.wake = None
                fut.remove_done_callback(on_result)
            if not fut.done():
                return                            # pods first: the loop pops them
        await self._finish_inflight_run(self._inflight.popleft())

    async def finish_inflight(self) -> None:
        """Apply the results of every run still on the engine worker, oldest first."""
        while self._inflight:
            await self._finish_inflight_run(self._inflight.popleft())

    # ================================================================== binding
    def _native_direct(self, fw: Framework, pi: PodInfo) -> bool:
        """This pod's bind can go straight to the native transport: DefaultBinder is the
        only bind plugin, no PreBind plugin applies to the pod, no extenders."""
        if self.extenders:
            return False
        rd = self._run_direct
        if rd is not None and rd[0] is fw and rd[1] is not None and not (pi.flags & rd[1]):
            return True                          # the run's mask: no PreBind plugin applies
        b = fw.direct_binder_for(pi)
        return b is not None and getattr(b, "native_bind", False)

    def _enqueue_bind(self, item: tuple) -> None:
        fw = item[0]
        if (self._binds is not None and self._native_direct(fw, item[2])
                and (self.native is not None or self.limiter.try_acquire())):
            pi, node = item[2], item[3]
            cb = functools.partial(self._native_bind_done, item, time.perf_counter())
            buf = self._bind_buf
            if buf is not None:                  # inside _finish_run: submitted with the run
                buf.append((pi.namespace, pi.name, pi.uid, node, self._bind_annotations(pi, node)))
                self._bind_cbs.append(cb)
                return
            self._binds.bind(pi.namespace, pi.name, pi.uid, node, self._bind_annotations(pi, node), cb,
                             self.bind_timeout)
            return
        self._bind_dq.append(item)
        idle = self._bind_idle
        while idle:                       # wake exactly one parked worker
            fut = idle.popleft()
            if not fut.done():
                fut.set_result(None)
                break

    def _bind_annotations(self, pi: PodInfo, node: str) -> list:
        """The Binding's GPU annotations (plugins.defaults.bind_annotations), memoised per
        (node, GPU set, HBM request) until the cache's node/Scv generation moves: a burst
        repeats a handful of placements per node."""
        cards = pi.assigned_cards
        if cards is None:
            return []
        scv = self.cache.scvs.get(node)
        if isinstance(scv, LazyScv):
            # per Scv version: survives other nodes' telemetry updates (the generation memo
            # below is flushed by every one of them)
            memo = scv.ann_memo
            key = (tuple(cards), pi.gpu.memory if pi.gpu.has_memory else -1)
            ann = memo.get(key)
            if ann is None:
                if len(memo) >= 1024:
                    memo.clear()
                ann = memo[key] = bind_annotations(pi, self.cache.scvs, node)
            return ann
        gen = self.cache.generation
        if self._ann_gen != gen:
            self._ann_memo.clear()
            self._ann_gen = gen
        key = (node, tuple(cards), pi.gpu.memory if pi.gpu.has_memory else -1)
        ann = self._ann_memo.get(key)
        if ann is None:
            if len(self._ann_memo) > 65536:
                self._ann_memo.clear()
            ann = self._ann_memo[key] = bind_annotations(pi, self.cache.scvs, node)
        return ann

    def _native_bind_done(self, item: tuple, tb: float, status: int, body: bytes) -> None:
        """Completion of a native binding POST (runs from the transport's eventfd callback)."""
        fw, state, pi, node, cycle, t0 = item
        self._pending_binds -= 1
        if 200 <= status < 300:
            if self.tracer is None and fw.post_bind_noop:
                # the common case inlined (_after_bind's success branch, no tracer / PostBind)
                now = time.perf_counter()
                self.cache.finish_binding(pi)
                self._scheduled += 1
                if self.lane is not None:
                    self.lane.python_bound()
                if self.e2e_samples is not None:
                    self.e2e_samples.append(now - t0)
                if self._metrics_on:
                    m = self.metrics
                    m.binding.observe(now - tb)
                    m.child(m.e2e, "scheduled", fw.name).observe(now - t0)
                self.recorder.pod_scheduled(pi, node)
                return
            st = Status.ok()
        else:
            from ..kube.native import api_error
            if status == 401 and self.native is not None:
                self.client._refresh_token(force=True)
            st = Status.error(f"binding rejected: {api_error(status, body)}", plugin="DefaultBinder")
        self._after_bind(fw, state if state is not None else _EMPTY_STATE, pi, node, cycle, t0, tb, st)

    def _after_bind(self, fw: Framework, state: CycleState, pi: PodInfo, node: str, cycle: int, t0: float,
                    tb: float, st: Status) -> None:
        m = self.metrics
        m.binding.observe(time.perf_counter() - tb)
        if self.tracer is not None:
            self.tracer.span("bind", self.tracer.now_us() - (time.perf_counter() - tb) * 1e6, cat="bind",
                             pod=pi.key, node=node, ok=st.is_success())
        if st.is_success():
            self.cache.finish_binding(pi)
            fw.run_post_bind(state, pi, node)
            self._scheduled += 1
            if self.lane is not None:
                self.lane.python_bound()
            if self.e2e_samples is not None:
                self.e2e_samples.append(time.perf_counter() - t0)
            m.child(m.e2e, "scheduled", fw.name).observe(time.perf_counter() - t0)
            self.recorder.pod_scheduled(pi, node)
        else:
            self.bind_errors += 1
            ps = self.cache.pods.get(pi.uid)
            if ps is not None and not ps.assumed and ps.node == node:
                # the Binding was applied — its watch echo already confirmed the pod — and
                # only the answer was lost (connection closed under pipelined requests,
                # client timeout): the pod is bound, so neither forget it (its reservation
                # is real) nor retry it (upstream ForgetPod refuses pods no longer assumed)
                self._scheduled += 1
                if self.lane is not None:
                    self.lane.python_bound()
                log.info("bind %s → %s answered %s after its echo confirmed it; kept as bound",
                         pi.key, node, st.message())
                return
            fw.run_unreserve(state, pi, node)
            self.cache.forget(pi)
            m.child(m.e2e, "error", fw.name).observe(time.perf_counter() - t0)
            self.recorder.pod_event(pi, "Warning", "FailedScheduling", f"Binding rejected: {st.message()}")
            log.info("bind %s → %s failed: %s", pi.key, node, st.message())
            self.queue.add_unschedulable(pi, cycle, unschedulable=False)

    async def _bind_worker(self) -> None:
        """Bind workers drain a shared deque and park (one future each) only when it is
        empty; an enqueue wakes at most one parked worker. A burst therefore costs a
        handful of task switches instead of one (or, with a broadcast event, one per
        worker) per pod, and ``bindConcurrency`` workers keep that many binds in flight
        against a remote apiserver."""
        dq, m = self._bind_dq, self.metrics
        loop = asyncio.get_event_loop()
        while True:
            if not dq:
                fut = loop.create_future()
                self._bind_idle.append(fut)
                await fut
                continue
            fw, state, pi, node, cycle, t0 = dq.popleft()
            if state is None:
                state = _EMPTY_STATE
            try:
                if not self.limiter.try_acquire():
                    await self.limiter.acquire()
                tb = time.perf_counter()
                try:
                    direct = fw.direct_binder() if not self.extenders else None
                    if direct is not None:
                        st = await direct.bind(state, pi, node)
                        if st.code.name == "SKIP":
                            st = Status.error("no bind plugin bound the pod")
                    else:
                        st = await fw.run_bind(state, pi, node, self._extender_binder(pi))
                except Exception as e:  # noqa: BLE001
                    st = Status.error(repr(e))
                self._after_bind(fw, state, pi, node, cycle, t0, tb, st)
            finally:
                self._pending_binds -= 1

    def _extender_binder(self, pi: PodInfo):
        for e in self.extenders:
            if e.cfg.bind_verb and e.is_interested(pi):
                return e
        return None

    # ================================================================== loops
    def _export_gpu_metrics(self, max_nodes: int = 2048) -> None:
        """yoda_gpu_* gauges (per-GPU reserved / sniffed free HBM, Scv staleness)."""
        m = self.metrics
        for k, name in enumerate(self.cache.nodes):
            if k >= max_nodes:
                break
            for i, g in enumerate(self.cache.node_gpu_state(name)):
                m.child(m.gpu_reserved, name, str(i)).set(g["reserved"])
                m.child(m.gpu_free, name, str(i)).set(g["free"])
            m.child(m.scv_stale, name).set(1 if self.cache._stale.get(name) else 0)

    async def _housekeeping(self, period: float = 0.5) -> None:
        m = self.metrics
        tick = 0
        while True:
            await asyncio.sleep(period)
            self.queue.flush_backoff_completed()
            self.queue.flush_unschedulable_leftover()
            self.cache.cleanup_expired()
            if self.nominations:                 # a nomination never outlives a minute
                now = time.monotonic()
                for uid in [u for u, (_n, _i, t) in self.nominations.items() if now - t > 60.0]:
                    self._clear_nomination(uid)
            self._maybe_enable_device()
            self._lane_refresh()                 # cluster gates (services, images, anti-affinity)
            self._settle_lane_mirror()
            refresh = getattr(self.client, "_refresh_token", None)
            if refresh is not None:
                refresh()                        # rotated service-account tokens
            tick += 1
            if tick % 4 == 0 and isinstance(m, SchedulerMetrics):
                self._export_gpu_metrics()
            flipped = self.cache.refresh_staleness()
            if flipped:
                self.queue.move_all_to_active_or_backoff("ScvStale")
            pend = self.queue.pending()
            if self.lane is not None:
                self._lane_metrics(m, pend)
            for q, n in pend.items():
                m.child(m.pending, q).set(n)
            counts = self.cache.snapshot_counts()
            m.child(m.cache_size, "nodes").set(counts["nodes"])
            m.child(m.cache_size, "pods").set(counts["pods"])
            m.child(m.cache_size, "assumed_pods").set(counts["assumed"])

    def _lane_metrics(self, m, pend: dict) -> None:
        """The lane's pods in the scheduler's metrics: its queued / in-flight pods are
        pending in activeQ, its unschedulableQ and podBackoffQ add to those gauges, and its
        scheduling attempts — Bindings acknowledged and unschedulable attempts it kept native —
        feed scheduler_schedule_attempts_total per profile."""
        st = self.lane.lane.stats()
        pend["active"] = pend.get("active", 0) + st["queued"] + st["inflight"]
        pend["backoff"] = pend.get("backoff", 0) + st["backoff"]
        pend["unschedulable"] = pend.get("unschedulable", 0) + st["parked"]
        seen = self._lane_attempts_seen
        for prof, (sched, failed) in st["by_profile"].items():
            ps, pf = seen.get(prof, (0, 0))
            if sched > ps:
                m.child(m.attempts, "scheduled", prof).inc(sched - ps)
            if failed > pf:
                m.child(m.attempts, "unschedulable", prof).inc(failed - pf)
            seen[prof] = (sched, failed)

    async def scheduling_loop(self) -> None:
        q = self.queue
        bs = max(1, self.config.batch_size)
        if self.lane is not None:
            self.lane.refresh()
            self.lane.set_active(True)           # the lane schedules while this loop does
        while not self._stop.is_set():
            if self._inflight and not q._active_entries:
                # nothing to pop: apply the oldest run when it lands, unless pods arrive first
                # (then they go to the engine behind it, which keeps the GPU busy while a burst
                # is still being ingested)
                await self._await_pods_or_result()
                continue
            pi = await q.pop()
            if pi is None:
                if q.closed:
                    await self.finish_inflight()
                    return
                continue
            if self.extenders:
                await self.finish_inflight()
                await self.schedule_one_async(pi)
            elif self.batching and q._active_entries:
                batch = [pi] + q.pop_batch(bs - 1)
                if self._overlap():
                    await self.schedule_batch_overlapped(batch)
                    # no yield here: the next batch's engine call starts first, and the
                    # binds / informer events of this one run during its await
                    continue
                else:
                    await self.finish_inflight()
                    self.schedule_batch(batch)
            else:
                await self.finish_inflight()
                self.schedule_one(pi)
            # let informers / binders run between cycles
            await asyncio.sleep(0)

    async def start(self, wait_sync: bool = True) -> None:
        """Start informers, binders, recorder and housekeeping (not the scheduling loop)."""
        loop = asyncio.get_event_loop()
        if not self.informers:
            self.make_informers()
        if self.lane is not None:
            self.lane.attach()                   # before the pod watch starts
        for inf in self.informers.values():
            self._tasks.append(loop.create_task(inf.run()))
        n_workers = max(1, self.config.bind_concurrency)
        for _ in range(n_workers):
            self._tasks.append(loop.create_task(self._bind_worker()))
        self._tasks.append(loop.create_task(self.recorder.run()))
        self._tasks.append(loop.create_task(self._housekeeping()))
        if wait_sync:
            await self.wait_synced()
        self._maybe_enable_device()
        self._lane_refresh()
        gctune.tune(self.config.gc_threshold)

    async def wait_synced(self) -> None:
        for inf in self.informers.values():
            await inf.synced.wait()

    async def run(self, elector=None) -> None:
        await self.start()
        if elector is not None:
            await elector.acquire()
            self.leading.set()
            self._tasks.append(asyncio.get_event_loop().create_task(self._watch_leadership(elector)))
        else:
            self.leading.set()
        await self.scheduling_loop()

    async def _watch_leadership(self, elector) -> None:
        await elector.lost.wait()
        log.error("leader election lost; stopping scheduling")
        self.stop()

    def stop(self) -> None:
        self._stop.set()
        self.queue.close()
        if self.lane is not None:
            self.lane.set_active(False)
        for inf in self.informers.values():
            inf.stop()

    async def shutdown(self) -> None:
        self.stop()
        for t in self._tasks:
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)
        self._tasks.clear()
        for e in self.extenders:
            await e.close()
        if self.lane is not None:
            self.lane.close()
        if self._engine_exec is not None:
            self._engine_exec.shutdown(wait=True)
            self._engine_exec = None
        if self._batch_worker is not None:
            w, self._batch_worker = self._batch_worker, None
            try:
                asyncio.get_event_loop().remove_reader(w.fileno())
            except (ValueError, OSError):
                pass
            w.close()
            for fut in self._batch_futs.values():
                if not fut.done():
                    fut.cancel()
            self._batch_futs.clear()

    async def drain_binds(self) -> None:
        while self.pending_binds:
            await asyncio.sleep(0)
