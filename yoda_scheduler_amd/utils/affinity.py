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


def pin_l3(index: int = 0) -> Optional[list[int]]:
    """Restrict this thread (and what it creates later) to the ``index``-th cache domain
    (modulo their number). Returns the CPUs, or None when there is a single domain."""
    sets = l3_cpu_sets()
    if len(sets) < 2:
        return None
    cpus = sets[index % len(sets)]
    os.sched_setaffinity(0, cpus)
    return cpus


def apply(spec: str) -> Optional[list[int]]:
    """``none`` | ``l3`` | ``l3:<index>`` (the CLI's --cpu-affinity)."""
    if not spec or spec == "none":
        return None
    if spec == "l3":
        return pin_l3(0)
    if spec.startswith("l3:"):
        return pin_l3(int(spec[3:]))
    raise ValueError(f"--cpu-affinity: expected none, l3 or l3:<index>, got {spec!r}")
