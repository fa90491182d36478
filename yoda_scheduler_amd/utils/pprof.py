"""``/debug/pprof`` for a Python control plane (SURVEY §5 tracing row: upstream serves Go
pprof on the secure port when ``enableProfiling`` is on).

* ``profile?seconds=N[&sort=cumulative|tottime][&limit=K]`` — a deterministic profile of the
  event-loop thread (where every scheduling cycle, informer handler and bind runs) over the
  next N seconds, as pstats text; native engine time shows up under the pybind11 calls.
* ``goroutine`` — stacks of every thread and every pending asyncio task.
* ``heap`` — GC generation counts/thresholds and the most numerous live object types.
"""
from __future__ import annotations

import asyncio
import cProfile
import gc
import io
import pstats
import sys
import threading
import traceback
from collections import Counter

_busy = False


async def profile_text(seconds: float, sort: str = "cumulative", limit: int = 60) -> str:
    global _busy
    seconds = max(0.05, min(float(seconds), 300.0))
    if _busy:
        return "another profile is running\n"
    _busy = True
    prof = cProfile.Profile()
    prof.enable()
    try:
        await asyncio.sleep(seconds)
    finally:
        prof.disable()
        _busy = False
    out = io.StringIO()
    st = pstats.Stats(prof, stream=out)
    st.sort_stats(sort if sort in ("cumulative", "tottime", "calls", "ncalls") else "cumulative")
    st.print_stats(max(1, int(limit)))
    return out.getvalue()


def goroutine_text() -> str:
    out = io.StringIO()
    names = {t.ident: t.name for t in threading.enumerate()}
    for ident, frame in sys._current_frames().items():
        out.write(f"thread {names.get(ident, ident)}:\n")
        out.write("".join(traceback.format_stack(frame)))
        out.write("\n")
    try:
        tasks = asyncio.all_tasks()
    except RuntimeError:
        tasks = set()
    out.write(f"{len(tasks)} asyncio task(s)\n")
    for t in tasks:
        out.write(f"task {t.get_name()} {t.get_coro()!r}:\n")
        for fr in t.get_stack(limit=12):
            out.write("".join(traceback.format_stack(fr, limit=1)))
        out.write("\n")
    return out.getvalue()


def heap_summary(top: int = 30) -> dict:
    counts = Counter(type(o).__name__ for o in gc.get_objects())
    return {"gc_count": gc.get_count(), "gc_threshold": gc.get_threshold(), "gc_frozen": gc.get_freeze_count(),
            "objects": sum(counts.values()), "top_types": counts.most_common(top)}
