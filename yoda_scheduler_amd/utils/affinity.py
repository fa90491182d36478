"""CPU placement for the scheduler process: one last-level-cache domain.

A scheduled pod crosses three threads and a process — the transport's I/O thread decodes its
watch events, the native lane thread queues, places and binds it, the apiserver answers — so
watch events, queue entries and answers move between cores for every pod. On multi-CCD EPYC
hosts, threads spread over several L3 domains pay cross-die cache-line transfers for all of
it: on one MI355X box the same config-3 burst ran at 51-68 k pods/s unpinned and 99-108 k
pinned to one domain (profiles/bench/r3/pin_ab/). ``pin_l3`` restricts the calling thread —
and every thread and child process created afterwards — to one domain; call it before the
scheduler starts its threads.
"""
from __future__ import annotations

import os
from typing import Optional


def l3_cpu_sets() -> list[list[int]]:
    """The CPUs this process may use, grouped by shared last-level cache, in CPU order; []
    when the topology is not readable."""
    groups: dict[str, list[int]] = {}
    try:
        for c in sorted(os.sched_getaffinity(0)):
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                groups.setdefault(f.read().strip(), []).append(c)
    except (OSError, AttributeError):
        return []
    return sorted(groups.values(), key=lambda g: g[0])


def _busy_fractions(cpus: list[int], window_s: float = 0.05) -> dict[int, float]:
    """Per-CPU busy fraction over a short window (/proc/stat); {} when unreadable."""
    import time

    def snap() -> dict[int, tuple[int, int]]:
        out = {}
        with open("/proc/stat") as f:
            for ln in f:
                if ln.startswith("cpu") and ln[3:4].isdigit():
                    parts = ln.split()
                    vals = [int(x) for x in parts[1:]]
                    idle = vals[3] + (vals[4] if len(vals) > 4 else 0)
                    out[int(parts[0][3:])] = (sum(vals), idle)
        return out
    try:
        a = snap()
        time.sleep(window_s)
        b = snap()
    except (OSError, ValueError, IndexError):
        return {}
    res = {}
    for c in cpus:
        if c in a and c in b:
            tot = b[c][0] - a[c][0]
            res[c] = 1.0 - (b[c][1] - a[c][1]) / tot if tot > 0 else 0.0
    return res


def pin_l3(index: int = 0, least_busy: bool = False) -> Optional[list[int]]:
    """Restrict this thread (and what it creates later) to the ``index``-th cache domain
    (modulo their number), or — ``least_busy`` — to the domain whose CPUs were the most idle
    over the last 50 ms (a shared host's other tenants). Returns the CPUs, or None when there
    is a single domain."""
    sets = l3_cpu_sets()
    if len(sets) < 2:
        return None
    cpus = sets[index % len(sets)]
    if least_busy:
        busy = _busy_fractions([c for g in sets for c in g])
        if busy:
            cpus = min(sets, key=lambda g: sum(busy.get(c, 1.0) for c in g) / len(g))
    os.sched_setaffinity(0, cpus)
    return cpus


def ranked_l3_sets() -> list[list[int]]:
    """The cache domains this process may use, most idle first over the last 50 ms (ties keep
    CPU order); [] when the topology is not readable."""
    sets = l3_cpu_sets()
    busy = _busy_fractions([c for g in sets for c in g]) if len(sets) > 1 else {}
    if not busy:
        return sets
    return sorted(sets, key=lambda g: (round(sum(busy.get(c, 1.0) for c in g) / len(g), 2), g[0]))


def pin_cpus(cpus: Optional[list[int]]) -> Optional[list[int]]:
    """Restrict this thread (and what it creates later) to ``cpus``; None leaves it alone."""
    if cpus:
        os.sched_setaffinity(0, cpus)
    return cpus


def apply(spec: str) -> Optional[list[int]]:
    """``none`` | ``l3`` (the least busy domain) | ``l3:<index>`` (the CLI's --cpu-affinity)."""
    if not spec or spec == "none":
        return None
    if spec == "l3":
        return pin_l3(0, least_busy=True)
    if spec.startswith("l3:"):
        return pin_l3(int(spec[3:]))
    raise ValueError(f"--cpu-affinity: expected none, l3 or l3:<index>, got {spec!r}")
