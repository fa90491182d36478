"""Who are this process's unnamed threads, and what are they doing?

The native threads of the scheduler are named (``yoda-io``, ``yoda-lane``, ``yoda-lane-eng``,
``yoda-engine``); threads started by libraries (the HIP/ROCr runtime, torch's pools) keep the
process name. ``bench.py`` reports their CPU as ``unnamed``. This module attributes them:

* **birth**: the tid sets at named points of start-up (``mark``) tell which step created a
  thread (e.g. ``import torch`` vs enabling the device scorer);
* **activity**: a sampler thread reads ``/proc/self/task/<tid>/syscall`` every ``period``
  seconds — the syscall a thread is blocked in (futex, poll, ioctl, …) or ``running``, and
  the user-space program counter, mapped to the library that owns it through
  ``/proc/self/maps`` — and the per-thread CPU ticks.

Linux only; everything degrades to empty results where ``/proc`` is not readable.
"""
from __future__ import annotations

import bisect
import collections
import os
import threading
import time
from typing import Optional

SYSCALLS = {0: "read", 1: "write", 7: "poll", 16: "ioctl", 23: "select", 35: "nanosleep", 202: "futex",
            228: "clock_gettime", 230: "clock_nanosleep", 232: "epoll_wait", 270: "pselect6", 271: "ppoll",
            281: "epoll_pwait", 24: "sched_yield", 47: "recvmsg", 45: "recvfrom", 441: "epoll_pwait2"}


def _tids() -> dict:
    out = {}
    try:
        for tid in os.listdir("/proc/self/task"):
            try:
                with open(f"/proc/self/task/{tid}/comm") as f:
                    out[int(tid)] = f.read().strip()
            except OSError:
                continue
    except OSError:
        pass
    return out


def _cpu_ticks(tid: int) -> int:
    try:
        with open(f"/proc/self/task/{tid}/stat") as f:
            fl = f.read().rsplit(")", 1)[1].split()
        return int(fl[11]) + int(fl[12])
    except (OSError, IndexError, ValueError):
        return 0


class _Maps:
    """Address → mapped file of this process (re-read when an address is not covered)."""

    def __init__(self) -> None:
        self.starts: list = []
        self.rows: list = []
        self.reload()

    def reload(self) -> None:
        rows = []
        try:
            with open("/proc/self/maps") as f:
                for ln in f:
                    parts = ln.split()
                    lo, hi = (int(x, 16) for x in parts[0].split("-"))
                    rows.append((lo, hi, os.path.basename(parts[5]) if len(parts) > 5 else "[anon]"))
        except OSError:
            pass
        rows.sort()
        self.rows, self.starts = rows, [r[0] for r in rows]

    def lib(self, addr: int) -> str:
        for attempt in (0, 1):
            k = bisect.bisect_right(self.starts, addr) - 1
            if k >= 0 and self.rows[k][0] <= addr < self.rows[k][1]:
                return self.rows[k][2]
            if attempt == 0:
                self.reload()
        return "?"


class ThreadScope:
    def __init__(self) -> None:
        self.births: dict[int, str] = {t: "start" for t in _tids()}
        self.names = _tids()
        self._maps: Optional[_Maps] = None
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None
        self.samples: dict[int, collections.Counter] = collections.defaultdict(collections.Counter)
        self.cpu0: dict[int, int] = {}
        self.cpu1: dict[int, int] = {}
        self.nsamples = 0

    def mark(self, label: str) -> None:
        """Threads first seen now were created by the step just before ``label``."""
        for t, nm in _tids().items():
            self.names.setdefault(t, nm)
            if t not in self.births:
                self.births[t] = label

    def _sample_one(self, tid: int) -> str:
        try:
            with open(f"/proc/self/task/{tid}/syscall") as f:
                s = f.read().split()
        except OSError:
            return "unreadable"
        if not s:
            return "?"
        if s[0] == "running":
            return "running"
        try:
            nr = int(s[0])
            pc = int(s[-1], 16)
        except ValueError:
            return s[0]
        return f"{SYSCALLS.get(nr, 'sys' + str(nr))}@{self._maps.lib(pc) if self._maps else '?'}"

    def _run(self, period: float, me: int) -> None:
        while not self._stop.wait(period):
            self.nsamples += 1
            for tid in list(_tids()):
                if tid != me:
                    self.samples[tid][self._sample_one(tid)] += 1

    def start(self, period: float = 0.002) -> None:
        self.mark("before-sampling")
        self._maps = _Maps()
        self.cpu0 = {t: _cpu_ticks(t) for t in _tids()}
        self._stop.clear()
        box: list = []

        def body() -> None:
            box.append(threading.get_native_id())
            self.me = box[0]
            self._run(period, box[0])
        self._th = threading.Thread(target=body, name="threadscope", daemon=True)
        self._th.start()

    def stop(self) -> None:
        self._stop.set()
        if self._th is not None:
            self._th.join(2.0)
        self.cpu1 = {t: _cpu_ticks(t) for t in _tids()}

    def report(self, only_unnamed: bool = True, top: int = 16) -> list:
        """Per thread (busiest first): tid, name, birth step, CPU ticks over the sampled window
        and its most frequent sampled states (syscall@library or running)."""
        proc = self.names.get(os.getpid(), "")
        out = []
        for tid, c1 in self.cpu1.items():
            nm = self.names.get(tid, _tids().get(tid, ""))
            if tid == getattr(self, "me", None) or (only_unnamed and (tid == os.getpid() or nm != proc)):
                continue
            d = c1 - self.cpu0.get(tid, 0)
            st = self.samples.get(tid, collections.Counter())
            out.append({"tid": tid, "name": nm, "born": self.births.get(tid, "?"), "cpu_ticks": d,
                        "states": st.most_common(4)})
        out.sort(key=lambda r: -r["cpu_ticks"])
        return out[:top]
