"""Python side of the native pod lane (``native/core/lane.hpp``).

The reference plugin only supplies Filter/Score; upstream kube-scheduler runs the per-pod
lifecycle around it in compiled Go — informer → activeQ → ``scheduleOne`` → assume → bind
goroutine → confirm / forget (``/root/reference/pkg/yoda/scheduler.go:76-130``). Here that
lifecycle runs in C++ for every pod an all-native profile can take: the transport hands the
lane every pod watch event, the lane thread queues, places (``Engine::schedule_batch``),
assumes and POSTs the Binding, and handles the answer, the watch echo and the deletion.

This module is everything Python still does, none of it per lane pod:

* decides per profile whether the lane may take its pods (the same conditions under which
  the Python runner would take the fully native path and bind directly) and with which
  pod-flag mask; re-decided when a cluster-wide plugin gate flips;
* applies what the lane forwards — events of pods it does not own (dispatched to the
  scheduler's ``on_pod_native`` exactly as the Python informer would), pods handed over
  after an unschedulable cycle or a failed Binding (FailedScheduling event, backoff queue,
  PostFilter/preemption), and a count of releases (the queue's move request);
* mirrors reserved lane pods into the cache on demand (``SchedulerCache.sync_lane``) for
  the Python plugins that read other pods, and parks the lane around ledger what-ifs.
"""
from __future__ import annotations

import asyncio
import os
import contextlib
import logging
from typing import Optional

from ..models.pod import PF_CLAIMS, PodInfo
from ..ops.native import core

log = logging.getLogger("yoda.lane")


class NativeLane:
    def __init__(self, sched, transport) -> None:
        from .events import API_EVENTS_V1
        self.s = sched
        self.transport = transport            # kube.native.NativeTransport
        rec = sched.recorder
        qs = next(iter(sched.frameworks.values())).queue_sort
        qname = getattr(qs, "name", "")
        self.sort_kind = {"yoda": 0, "PrioritySort": 1}.get(qname, -1)
        self.lane = core().Lane(sched.engine, batch=max(1, sched.config.batch_size), bind_timeout=sched.bind_timeout,
                                sort_kind=max(self.sort_kind, 0), events=rec.enabled,
                                events_v1=rec.api == API_EVENTS_V1, event_qps=float(rec.limiter.qps),
                                event_burst=int(rec.limiter.burst), event_buffer=rec.max_buffer, host=rec.host,
                                name_prefix=rec._name_prefix,
                                # runs on an engine worker while the lane serves its inbox: with a
                                # device scorer (1, default), never (0), always (2: tests)
                                async_mode=int(os.environ.get("YODA_LANE_ASYNC", "1")),
                                engine_delay_us=int(os.environ.get("YODA_LANE_ENGINE_DELAY_US", "0")),
                                # busy-wait (µs) of the lane thread / engine worker around device runs
                                spin_us=int(os.environ.get("YODA_LANE_SPIN_US", "0")),
                                # the lane's own unschedulableQ / podBackoffQ (native unschedulable path)
                                initial_backoff=float(sched.config.pod_initial_backoff_seconds),
                                max_backoff=float(sched.config.pod_max_backoff_seconds),
                                unschedulable_flush=float(sched.config.unschedulable_flush_seconds))
        self.lane.set_port(transport.t.port_ptr())
        self._profiles: dict[str, tuple] = {}
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self.handoffs = 0
        self.forwarded = 0
        self._waiters: list = []           # (target scheduled count, future)
        self._unowned_waiters: list = []   # futures resolved once the lane owns no pod
        self._draining = False             # applying the lane's own move request (not echoed back)
        self._temp_terms: tuple = ()        # gates of a Python cycle running beside the lane (gated)
        self._in_gated = False             # inside gated(): anti-affinity changes wait for its exit
        self._gates_pending = False        # a coalesced gate update (holder removals) is scheduled
        self._sticky_never = (1 << 62) - 1  # AND of the masks of profiles eligible since the lane last owned nothing
        self._inert = None                 # plugins/volumes.py::LaneClaims, made on first use
        self._claims = frozenset()         # the claims the lane may admit (the table's keys)
        self._limits_dirty: Optional[set] = None   # nodes whose CSI attach limits to push (None: all)
        self._limits: dict = {}            # node → the CSI limits pushed to the engine
        sched.queue.on_move_all = self._move_all

    # ------------------------------------------------------------------ lifecycle
    def attach(self) -> None:
        """Route the transport's pod watch events into the lane and wake the loop on its
        output. Must precede the pod informer's first watch."""
        self.transport.t.set_pod_sink(self.lane.sink_ptr())
        loop = asyncio.get_event_loop()
        if self._loop is not loop:
            loop.add_reader(self.lane.fileno(), self._drain)
            self._loop = loop

    def set_active(self, on: bool) -> None:
        self.lane.set_active(bool(on))

    def close(self) -> None:
        if self._loop is not None and not self._loop.is_closed():
            with contextlib.suppress(Exception):
                self._loop.remove_reader(self.lane.fileno())
        self._loop = None
        self.transport.t.set_pod_sink(0)
        self.lane.close()

    # ------------------------------------------------------------------ profiles
    def eligible_mask(self, fw) -> Optional[int]:
        """Pod-flag mask for which the lane may run ``fw``'s pods end to end, or None: the
        profile's cycle must be fully native for such pods (Framework.native_mask, which is
        None while a cluster gate is active) and their binding a direct DefaultBinder POST
        with no PreBind/Reserve/Permit/PostBind plugin applying (Framework.direct_bind_mask)."""
        s = self.s
        if s.extenders or self.sort_kind < 0 or not fw.fully_native_static or not fw.post_bind_noop:
            return None
        m = fw.native_mask(lane=True)
        if m is None or fw.lane_flags is None:
            return None
        m |= fw.lane_flags
        if len(fw.bind_plugins) != 1 or not getattr(fw.bind_plugins[0], "native_bind", False):
            return None
        bm = fw.direct_bind_mask()
        if bm is None:
            return None
        return m | bm

    INT64_MIN, INT64_MAX = -(1 << 63), (1 << 63) - 1

    def preempt_above(self, fw) -> int:
        """Unschedulable pods of ``fw`` with ``spec.priority`` above this go to Python, where a
        PostFilter may act on them; the lane fails the others natively (FailedScheduling,
        PodScheduled=False, its own unschedulableQ / backoffQ). The yoda PostFilter is a no-op
        (maxima are computed in PreScore), and DefaultPreemption preempts only for pods with a
        positive priority unless ``preemptZeroPriority`` is set; any other PostFilter plugin may
        act on any pod."""
        above = self.INT64_MAX
        for p in fw.post_filter:
            name = getattr(p, "name", "")
            if name == "yoda":
                continue
            if name == "DefaultPreemption" and not (getattr(p, "args", None) or {}).get("preemptZeroPriority", False):
                above = min(above, 0)
                continue
            return self.INT64_MIN
        return above

    def _move_all(self) -> None:
        """A Python move request (node/Scv add or update, a Python pod's deletion, staleness, ...)
        moves the lane's parked pods too (upstream has one queue for both)."""
        if not self._draining:
            self.lane.move(-1)

    def move_node(self, idx: int) -> None:
        """Queueing hint: ``idx``'s filter-visible capacity grew; parked lane pods that now pass
        every filter there move (re-filtered in C++ against the node)."""
        self.lane.move(idx)

    def refresh(self) -> None:
        """(Re)declare every profile to the lane when its eligibility changed. A profile the
        lane may no longer run gets its queued pods back through the Python queue."""
        s = self.s
        f_yoda = core().F_YODA
        never = (1 << 62) - 1                  # pod flags no lane pod carries (AND of the masks)
        # sticky across eligibility flips: a profile that turned ineligible still has
        # its reserved pods in the lane, so its mask keeps counting until the lane owns nothing
        if self._sticky_never != never and self.owned() == 0:
            self._sticky_never = never
        claims = self._refresh_claims()
        for name, fw in s.frameworks.items():
            m = self.eligible_mask(fw)
            c_ok = m is not None and fw.claims_ok()
            if m is not None:
                # lane pods may carry PF_CLAIMS (claim-table claims only) once the table is non-empty
                lm = m & ~PF_CLAIMS if c_ok and claims else m
                never &= lm
                self._sticky_never &= lm
            filters = {p.name for p in fw.filter_py}
            want = (m is not None, m or 0, bool(fw.filter_mask & f_yoda), self.preempt_above(fw),
                    fw.gate_terms() + self._temp_terms if m is not None else (), c_ok,
                    "VolumeBinding" in filters, "VolumeZone" in filters, "NodeVolumeLimits" in filters)
            if self._profiles.get(name) == want:
                continue
            s._activate(fw)                    # the lane snapshots the engine config now applied
            self.lane.set_profile(s.engine, name, want[0], want[1], want[2], want[3], list(want[4]), want[5],
                                  want[6], want[7], want[8])
            self._profiles[name] = want
            log.info("native lane: profile %s %s (flag mask %#x)", name, "on" if want[0] else "off", want[1])
        s.cache.lane_never_flags = never & self._sticky_never

    def claims_event(self, res: str, obj: dict) -> None:
        """A PVC / PV / StorageClass / CSINode changed: what it affects is re-evaluated on the next
        refresh (O(change); a StorageClass re-evaluates every claim)."""
        if res == "csinodes":
            self.node_event((obj.get("metadata") or {}).get("name", ""))
            return
        if self._inert is None:
            return
        if res == "persistentvolumeclaims":
            self._inert.pvc_event(obj)
        elif res == "persistentvolumes":
            self._inert.pv_event(obj)
        elif res == "storageclasses":
            self._inert.sc_event(obj)

    def node_event(self, name: str) -> None:
        """A node (or its CSINode) changed: its CSI attach limits are pushed on the next refresh."""
        if self._limits_dirty is not None:
            self._limits_dirty.add(name)

    def _push_limits(self) -> None:
        """The nodes' CSI attach limits (plugins/volumes.py::node_csi_limits) to the engine, which
        counts lane pods' PVC volumes against them (NodeVolumeLimits)."""
        from ..plugins.volumes import node_csi_limits
        s = self.s
        dirty, self._limits_dirty = self._limits_dirty, set()
        names = set(s.cache.nodes) | set(self._limits) if dirty is None else dirty
        csinodes = s.handle.lister("csinodes")
        for name in names:
            info = s.cache.nodes.get(name)
            idx = s.engine.node_index(name) if info is not None else -1
            if idx < 0:
                self._limits.pop(name, None)
                continue
            lim = node_csi_limits(info.obj, csinodes.get(name)) or {}
            if self._limits.get(name, {}) != lim or dirty is None:
                s.engine.set_node_vol_limits(idx, sorted(lim.items()))
                self._limits[name] = lim

    def _refresh_claims(self) -> set:
        """Keep the lane's claim table (plugins/volumes.py::LaneClaims) current: the claims a pod
        may mount and still take the native cycle, with the node constraints of their PVs. Only
        profiles whose volume plugins all allow it (``claims_ok``) use it; changes go to the
        lane as deltas."""
        s = self.s
        if not any(fw.claims_ok() for fw in s.frameworks.values()):
            return self._claims
        if self._inert is None:
            from ..plugins.volumes import LaneClaims
            self._inert = LaneClaims(s.handle)
        if self._limits_dirty is None or self._limits_dirty:
            self._push_limits()
        full, changed, removed, vfull, vchanged, vremoved = self._inert.refresh()
        if vchanged or vremoved:                 # before the table: a pod admitted next counts them
            s.engine.set_claim_volumes([(k, d, h) for k, (d, h) in sorted(vchanged.items())], sorted(vremoved))
        if full is not None:
            self.lane.update_claims(s.engine, True, [_claim_item(k, v) for k, v in sorted(full.items())], [])
        elif changed or removed:
            self.lane.update_claims(s.engine, False, [_claim_item(k, v) for k, v in sorted(changed.items())],
                                    sorted(removed))
        self._claims = self._inert.keys
        return self._claims

    def anti_changed(self, grew: bool = True) -> None:
        """The bound/assumed pods with required anti-affinity changed. A new holder's terms reach
        the lane now (it must not place a pod they reject); removals — a burst's deletions come
        one event at a time — are coalesced into one update at the end of the loop turn (until
        then the lane only holds back pods it could have taken: safe)."""
        loop = self._loop
        if grew or loop is None or loop.is_closed():
            self.refresh_gates()
            return
        if not self._gates_pending:
            self._gates_pending = True
            loop.call_soon(self._refresh_pending_gates)

    def _refresh_pending_gates(self) -> None:
        self._gates_pending = False
        self.refresh_gates()

    def refresh_gates(self) -> None:
        """Only the selector gates changed (a pod with required anti-affinity was assumed or
        left): re-send the terms of the profiles the lane runs — eligibility itself does not
        depend on them (``Framework.native_mask(lane=True)``)."""
        if self._in_gated:
            return                             # gated() re-sends the gates when the cycle ends
        s = self.s
        for name, fw in s.frameworks.items():
            want = self._profiles.get(name)
            if want is None or not want[0]:
                continue
            terms = fw.gate_terms() + self._temp_terms
            if terms == want[4]:
                continue
            self.lane.set_gates(name, list(terms))
            self._profiles[name] = want[:4] + (terms,) + want[5:]

    # ------------------------------------------------------------------ lane output
    async def wait_scheduled(self, target: int, timeout: float) -> bool:
        """Until ``target`` Bindings are acknowledged on either path (``Scheduler.scheduled``:
        the lane's count plus the Python path's), or ``timeout``. The lane wakes the loop when
        its own count crosses ``target`` minus the Python path's (no polling); a Python-path
        bind re-checks and moves that watermark (``python_bound``)."""
        if self.s.scheduled >= target:
            return True
        fut = asyncio.get_event_loop().create_future()
        self._waiters.append((target, fut))
        self._set_watermark()
        try:
            await asyncio.wait_for(asyncio.shield(fut), timeout)
            return True
        except asyncio.TimeoutError:
            return self.s.scheduled >= target
        finally:
            self._waiters = [(t, f) for t, f in self._waiters if f is not fut]
            self._set_watermark()

    def _set_watermark(self) -> None:
        # the lane signals when its own count reaches the nearest total target less the
        # Python path's binds so far
        if self._waiters:
            self.lane.set_watermark(max(0, min(t for t, _ in self._waiters) - self.s._scheduled))
        else:
            self.lane.set_watermark((1 << 64) - 1)

    def python_bound(self) -> None:
        """A Python-path Binding was acknowledged: wake waiters it satisfies, lower the lane's
        watermark for the rest."""
        if self._waiters:
            self._wake_waiters()
            self._set_watermark()

    async def wait_unowned(self, timeout: float) -> bool:
        """Until the lane owns no pod (e.g. every pod of a burst deleted and released), or
        ``timeout``. Woken by the lane's own signal (a release is a move request), re-checked
        every 2 ms in case the last change signalled nothing."""
        loop = asyncio.get_event_loop()
        end = loop.time() + timeout
        while self.owned():
            left = end - loop.time()
            if left <= 0:
                return False
            fut = loop.create_future()
            self._unowned_waiters.append(fut)
            try:
                await asyncio.wait_for(asyncio.shield(fut), min(left, 0.002))
            except asyncio.TimeoutError:
                pass
            finally:
                self._unowned_waiters = [f for f in self._unowned_waiters if f is not fut]
        return True

    def _wake_waiters(self) -> None:
        n = self.s.scheduled
        for t, f in self._waiters:
            if n >= t and not f.done():
                f.set_result(None)

    def _drain(self) -> None:
        fwd, hand, moves = self.lane.drain()
        if self._waiters:
            self._wake_waiters()
        if self._unowned_waiters and not self.owned():
            for f in self._unowned_waiters:
                if not f.done():
                    f.set_result(None)
        s = self.s
        if fwd:
            self.forwarded += len(fwd)
            handler = s.on_pod_native
            for typ, ev, old in fwd:
                try:
                    handler(typ, ev, ev.ident(), (old, old.ident()) if old is not None else None)
                except Exception:  # noqa: BLE001 - isolate handlers, like the informer
                    log.exception("native lane: pod event handler failed")
        if moves:
            self._draining = True              # the lane already moved its own parked pods
            try:
                s.queue.move_all_to_active_or_backoff("AssignedPodDelete")
            finally:
                self._draining = False
            if s._dev_flush:
                s._request_device_flush()
        for h in hand:
            try:
                self._handoff(h)
            except Exception:  # noqa: BLE001
                log.exception("native lane: handoff failed")

    def _handoff(self, h: tuple) -> None:
        """A pod the lane gave up: from here on it is an ordinary Python-path pod."""
        kind, ev, prof, res, status, msg, t_enq, t_cycle, attempts = h
        s = self.s
        self.handoffs += 1
        fw = s.frameworks.get(prof) or next(iter(s.frameworks.values()))
        pi = PodInfo.from_native(ev)
        pi.attempts = max(1, attempts)
        pi.initial_attempt = pi.enqueued = t_enq
        if kind == 2:
            # a waiting lane pod its profile's lane may no longer run: Python's podBackoffQ, its
            # attempts (and so its backoff) carried over, no second FailedScheduling
            pi.initial_attempt = t_enq
            s.queue.add_unschedulable(pi, -1, unschedulable=False)
            return
        if kind == 0:
            # cycle -1: a move request may have arrived since the lane's cycle, so the pod
            # retries from backoff rather than parking in unschedulableQ (never lose a wake-up)
            if fw.post_filter:
                with self.held():             # preemption reads other pods and what-ifs the ledger
                    s._fail(fw, None, pi, -1, s._fit_error(res, pi), t_cycle)
            else:
                s._fail(fw, None, pi, -1, s._fit_error(res, pi), t_cycle)
            return
        from ..kube.native import api_error
        if status == 401:
            s.client._refresh_token(force=True)
        s.bind_errors += 1
        err = api_error(status, msg)
        s.recorder.pod_event(pi, "Warning", "FailedScheduling", f"Binding rejected: {err}")
        log.info("bind %s failed: %s", pi.key, err)
        s.queue.add_unschedulable(pi, -1, unschedulable=False)

    # ------------------------------------------------------------------ cache view
    @contextlib.contextmanager
    def held(self, sync: bool = True):
        """The lane thread is parked (and, with ``sync``, the cache mirrors its reserved pods):
        Python plugins may read other pods — natively counted or mirrored — and run ledger
        what-ifs (preemption) with no lane placement in between. The lane is parked first and
        mirrored second: a pod it placed in between would otherwise be missing from the mirror."""
        self.lane.pause(True)
        try:
            if sync:
                self.s.cache.sync_lane()
            yield
        finally:
            self.lane.pause(False)

    @contextlib.contextmanager
    def gated(self, queries):
        """A Python cycle runs while the lane keeps placing pods, except pods matching
        ``queries`` (the native terms the cycle's plugins are sensitive to; a conjunctive query
        gates each of its terms: a superset). The gates are sent, then the lane is parked for
        a moment — it applies them, finishes any run, and evicts queued matching pods to
        Python — and released: from then on every lane pod the cycle could care about is
        reserved (the census shows it) or handed to the Python queue."""
        terms = tuple(t for q in queries for t in q)
        if not terms:
            yield
            return
        self._temp_terms = terms
        try:
            self.refresh_gates()
            self.lane.pause(True)
            self.lane.pause(False)
            # the cycle's own assume may add gate terms (its required anti-affinity): they are
            # sent once, with the temporary terms dropped, when the cycle ends
            self._in_gated = True
            yield
        finally:
            self._in_gated = False
            self._temp_terms = ()
            self.refresh_gates()

    # ------------------------------------------------------------------ counters
    def pending(self) -> int:
        st = self.lane.stats()
        return st["queued"] + st["inflight"] + st["binding"]

    def waiting(self) -> int:
        """Lane pods in its unschedulableQ or podBackoffQ."""
        st = self.lane.stats()
        return st["parked"] + st["backoff"]

    def owned(self) -> int:
        return self.lane.stats()["owned"]


def _claim_item(key: str, v) -> tuple:
    """A claim-table entry for ``Lane.update_claims``: (key, node terms | None, zone terms | None),
    terms as [[(key, op, [values])]] (plugins/volumes.py::claim_lane)."""
    if v is None:
        return key, None, None
    node, zone = v
    conv = (lambda terms: None if terms is None else [[(k, op, list(vals)) for k, op, vals in t] for t in terms])
    return key, conv(node), conv(zone)


class LaneEntries:
    """``key → (PodEvent, ident)`` view of the lane's pod store for the pod informer (the
    informer keeps no per-pod state of its own when the lane owns the stream)."""

    def __init__(self, lane) -> None:
        self._l = lane

    def get(self, key, default=None):
        r = self._l.lookup(key)
        if r is None:
            return default
        ev = r[0]
        return ev, ev.ident()

    def __getitem__(self, key):
        v = self.get(key)
        if v is None:
            raise KeyError(key)
        return v

    def __contains__(self, key) -> bool:
        return self._l.lookup(key) is not None

    def __iter__(self):
        return iter(self._l.keys())

    def __len__(self) -> int:
        return len(self._l)

    # the lane is the store's only writer: informer-side writes are no-ops
    def __setitem__(self, key, value) -> None:
        return None

    def pop(self, key, default=None):
        return self.get(key, default)
