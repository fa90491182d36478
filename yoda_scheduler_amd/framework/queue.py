"""Scheduling queue: activeQ heap + podBackoffQ + unschedulableQ.

* activeQ is ordered by the profile's QueueSort plugin. The reference's ``Less`` has no
  tie-break (``pkg/yoda/sort/sort.go:8-10``, quirk Q7); here every key ends with a
  monotonically increasing enqueue sequence number, so equal priorities are FIFO.
* Failed pods go to backoffQ with ``initial × 2^(attempts−1)`` capped at ``max``
  (``podInitialBackoffSeconds``/``podMaxBackoffSeconds``, ``deploy:19-20``), or to the
  unschedulableQ when the failure was "unschedulable"; cluster events move them back,
  and a periodic flush re-activates pods parked longer than the flush interval.
"""
from __future__ import annotations

import asyncio
import collections
import heapq
import itertools
import time
from typing import Callable, Optional

from ..models.pod import PodInfo


class SchedulingQueue:
    def __init__(self, sort_key: Callable[[PodInfo], tuple], initial_backoff: float = 1.0,
                 max_backoff: float = 10.0, unschedulable_flush: float = 60.0,
                 clock: Callable[[], float] = time.monotonic) -> None:
        self._sort_key = sort_key
        self._seq = itertools.count()
        self._active: list[tuple] = []           # (key..., seq, uid)
        self._active_entries: dict[str, tuple] = {}
        self._backoff: list[tuple[float, int, str]] = []
        self._backoff_pods: dict[str, PodInfo] = {}
        self._unsched: dict[str, tuple[PodInfo, float]] = {}
        self._pods: dict[str, PodInfo] = {}       # uid → info for everything queued
        self.initial_backoff = initial_backoff
        self.max_backoff = max_backoff
        self.unschedulable_flush = unschedulable_flush
        self.clock = clock
        self._cond: Optional[asyncio.Event] = None
        self.scheduling_cycle = 0
        self._move_request_cycle = -1
        # hinted moves (cycle, predicate), newest last: a pod that fails a cycle started
        # before one of them retries from backoff only if that predicate accepts it
        # (upstream's in-flight events + QueueingHint); older entries are dropped
        self._hint_moves: collections.deque = collections.deque()
        self._hint_dropped_cycle = -1
        self.closed = False
        # one-shot future resolved by the next push to the active queue (the scheduling loop
        # waits on it together with an engine result: one event-loop hop to wake, where an
        # asyncio.Event behind asyncio.wait takes three — each behind a chunk of watch events)
        self.wake: Optional[asyncio.Future] = None
        # (event, queue, n) → scheduler_queue_incoming_pods_total; None = not counted
        self.incoming_hook: Optional[Callable[[str, str, int], None]] = None
        # every move-all request is forwarded here too (the native lane's own parked pods)
        self.on_move_all: Optional[Callable[[], None]] = None

    # ------------------------------------------------------------------ helpers
    def _event(self) -> asyncio.Event:
        if self._cond is None:
            self._cond = asyncio.Event()
        return self._cond

    def _push_active(self, pi: PodInfo) -> None:
        pi.enqueued = self.clock()
        if not pi.initial_attempt:
            pi.initial_attempt = pi.enqueued
        entry = (*self._sort_key(pi), next(self._seq), pi.uid)
        self._active_entries[pi.uid] = entry
        self._pods[pi.uid] = pi
        heapq.heappush(self._active, entry)
        if self._cond is not None:
            self._cond.set()
        w = self.wake
        if w is not None:
            self.wake = None
            if not w.done():
                w.set_result(None)

    def backoff_duration(self, pi: PodInfo) -> float:
        d = self.initial_backoff * (2 ** max(pi.attempts - 1, 0))
        return min(d, self.max_backoff)

    # ------------------------------------------------------------------ API
    def __len__(self) -> int:
        return len(self._active_entries) + len(self._backoff_pods) + len(self._unsched)

    def pending(self) -> dict[str, int]:
        return {"active": len(self._active_entries), "backoff": len(self._backoff_pods),
                "unschedulable": len(self._unsched)}

    def contains(self, uid: str) -> bool:
        return uid in self._pods

    def add(self, pi: PodInfo) -> None:
        """New pending pod (informer add)."""
        if pi.uid in self._pods:
            self.update(pi)
            return
        self._push_active(pi)

    def update(self, pi: PodInfo) -> None:
        old = self._pods.get(pi.uid)
        if old is None:
            self._push_active(pi)
            return
        pi.attempts, pi.initial_attempt = old.attempts, old.initial_attempt
        entry = self._active_entries.get(pi.uid)
        if entry is not None:
            self._pods[pi.uid] = pi      # the info is refreshed
            key = self._sort_key(pi)
            if tuple(entry[:len(key)]) != tuple(key):
                # order changed (e.g. scv/priority edited): re-sort like upstream's
                # activeQ.Update, keeping the original FIFO sequence number
                new = (*key, entry[-2], pi.uid)
                self._active_entries[pi.uid] = new
                heapq.heappush(self._active, new)
            return
        # an update may make an unschedulable pod schedulable: retry now
        self._remove_parked(pi.uid)
        self._push_active(pi)

    def _remove_parked(self, uid: str) -> None:
        self._backoff_pods.pop(uid, None)
        self._unsched.pop(uid, None)

    def delete(self, uid: str) -> None:
        self._pods.pop(uid, None)
        self._active_entries.pop(uid, None)   # lazy heap deletion
        self._remove_parked(uid)

    def pop_nowait(self) -> Optional[PodInfo]:
        while self._active:
            entry = heapq.heappop(self._active)
            uid = entry[-1]
            if self._active_entries.get(uid) is not entry:
                continue
            del self._active_entries[uid]
            pi = self._pods.pop(uid)
            pi.attempts += 1
            self.scheduling_cycle += 1
            return pi
        return None

    def pop_batch(self, n: int) -> list[PodInfo]:
        out = []
        while len(out) < n:
            pi = self.pop_nowait()
            if pi is None:
                break
            out.append(pi)
        return out

    async def pop(self, timeout: Optional[float] = None) -> Optional[PodInfo]:
        while True:
            self.flush_backoff_completed()
            pi = self.pop_nowait()
            if pi is not None or self.closed:
                return pi
            ev = self._event()
            ev.clear()
            wait = self._next_backoff_wait()
            if timeout is not None:
                wait = timeout if wait is None else min(wait, timeout)
            try:
                if wait is None:
                    await ev.wait()
                else:
                    await asyncio.wait_for(ev.wait(), wait)
            except asyncio.TimeoutError:
                if timeout is not None and self._next_backoff_wait() is None and not self._active_entries:
                    return None

    def _next_backoff_wait(self) -> Optional[float]:
        while self._backoff and self._backoff[0][2] not in self._backoff_pods:
            heapq.heappop(self._backoff)
        if not self._backoff:
            return None
        return max(0.0, self._backoff[0][0] - self.clock())

    def add_unschedulable(self, pi: PodInfo, cycle: int, unschedulable: bool = True) -> None:
        """Re-queue a pod whose cycle failed. If a move request happened since the pod
        was popped, go straight to backoff (upstream ``moveRequestCycle`` rule)."""
        if pi.uid in self._pods:
            return
        self._pods[pi.uid] = pi
        pi.enqueued = self.clock()          # backoff counts from the failed attempt
        if not unschedulable or self._move_request_cycle >= cycle or self._hinted_since(pi, cycle):
            self._to_backoff(pi)
            where = "backoff"
        else:
            self._unsched[pi.uid] = (pi, self.clock())
            where = "unschedulable"
        if self.incoming_hook is not None:
            self.incoming_hook("ScheduleAttemptFailure", where, 1)

    def _to_backoff(self, pi: PodInfo) -> None:
        t = self.clock() + self.backoff_duration(pi)
        self._backoff_pods[pi.uid] = pi
        heapq.heappush(self._backoff, (t, next(self._seq), pi.uid))
        if self._cond is not None:
            self._cond.set()

    def flush_backoff_completed(self) -> int:
        now, n = self.clock(), 0
        while self._backoff and self._backoff[0][0] <= now:
            _, _, uid = heapq.heappop(self._backoff)
            pi = self._backoff_pods.pop(uid, None)
            if pi is not None:
                self._pods.pop(uid, None)
                self._push_active(pi)
                n += 1
        return n

    def flush_unschedulable_leftover(self) -> int:
        now = self.clock()
        old = [pi for pi, t in self._unsched.values() if now - t > self.unschedulable_flush]
        for pi in old:
            del self._unsched[pi.uid]
            self._pods.pop(pi.uid, None)
            self._route(pi)
        return len(old)

    def _route(self, pi: PodInfo) -> bool:
        """Backoff if the pod's backoff has not expired yet, else active; True = active."""
        if self.clock() - pi.enqueued < self.backoff_duration(pi):
            self._to_backoff(pi)
            return False
        self._push_active(pi)
        return True

    def move_all_to_active_or_backoff(self, event: str = "") -> int:
        """A cluster event (node add, Scv update, pod delete...) may make parked pods
        schedulable."""
        if self.on_move_all is not None:
            self.on_move_all()
        if not self._unsched:                  # the common case (every pod deletion): only
            self._move_request_cycle = self.scheduling_cycle   # record the move request
            return 0
        pods = [pi for pi, _ in self._unsched.values()]
        self._unsched.clear()
        return self._move(pods, event)

    def move_matching_to_active_or_backoff(self, pred, event: str = "") -> int:
        """Queueing hint: move only the parked pods for which ``pred(pod)`` says the event
        could make them schedulable. The move request is recorded either way, so a pod in
        flight when the event arrived retries from backoff instead of parking."""
        pods = [pi for pi, _ in self._unsched.values() if pred(pi)]
        for pi in pods:
            del self._unsched[pi.uid]
        if self._hint_moves and self._hint_moves[-1][0] == self.scheduling_cycle:
            c, prev = self._hint_moves.pop()          # same cycle: one entry accepting either
            self._hint_moves.append((c, lambda pi, a=prev, b=pred: a(pi) or b(pi)))
        else:
            self._hint_moves.append((self.scheduling_cycle, pred))
        while len(self._hint_moves) > self.HINT_HISTORY:
            self._hint_dropped_cycle = self._hint_moves.popleft()[0]
        return self._move(pods, event, record=False)

    HINT_HISTORY = 256

    def _hinted_since(self, pi: PodInfo, cycle: int) -> bool:
        """Did a hinted move accept ``pi`` at or after ``cycle`` (its scheduling attempt)?
        Conservatively yes when entries that old were already dropped."""
        if self._hint_dropped_cycle >= cycle:
            return True
        for c, pred in reversed(self._hint_moves):
            if c < cycle:
                break
            if pred(pi):
                return True
        return False

    def _move(self, pods: list, event: str, record: bool = True) -> int:
        active = 0
        for pi in pods:
            self._pods.pop(pi.uid, None)
            active += self._route(pi)
        if record:
            self._move_request_cycle = self.scheduling_cycle
        if pods and self.incoming_hook is not None:
            if active:
                self.incoming_hook(event, "active", active)
            if len(pods) > active:
                self.incoming_hook(event, "backoff", len(pods) - active)
        return len(pods)

    def close(self) -> None:
        self.closed = True
        if self._cond is not None:
            self._cond.set()
