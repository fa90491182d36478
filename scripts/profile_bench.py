#!/usr/bin/env python3
"""cProfile of the scheduler process during the timed bursts of ``bench.py``.

    python scripts/profile_bench.py [--out FILE] [bench.py args...]

Profiling is enabled only inside the timed steps (not start-up or warmup), and the top
functions by own time plus a grouped per-stage summary are printed / written to FILE."""
from __future__ import annotations

import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STAGES = [  # (stage, substrings of "file:function" that belong to it), first match wins
    ("watch decode + informer dispatch", ("informer.py", "kube/native.py:_drain", "json/")),
    ("pod event handlers", ("scheduler.py:on_pod", "pod.py", "labels.py", "queue.py:add", "queue.py:update",
                            "queue.py:_push", "queue.py:delete", "cache.py:add_pod", "cache.py:update_pod",
                            "cache.py:remove_pod", "cache.py:_add_bound", "queue.py:move_all")),
    ("scheduling cycle (native engine + bookkeeping)", ("scheduler.py:schedule", "scheduler.py:_batch",
                                                        "scheduler.py:_prepare", "scheduler.py:_finish",
                                                        "scheduler.py:_pod_gone", "native.py:pod_req",
                                                        "cache.py:assumed", "cache.py:_track", "runtime.py",
                                                        "queue.py:pop", "schedule_batch")),
    ("binding (submit + completion)", ("scheduler.py:_enqueue_bind", "scheduler.py:_native_bind",
                                       "scheduler.py:_after_bind", "scheduler.py:_bind_worker",
                                       "kube/native.py:bind", "defaults.py", "fastbind.py", "client.py:bind",
                                       "cache.py:finish_binding")),
    ("event recorder", ("events.py",)),
    ("asyncio / selectors", ("asyncio/", "selectors.py", "select.epoll")),
]


def main() -> int:
    args = sys.argv[1:]
    out = None
    if args[:1] == ["--out"]:
        out, args = args[1], args[2:]
    import bench
    from yoda_scheduler_amd.bench import harness as H
    if os.environ.get("YODA_PROF_SAMPLE"):
        return _sample(args, out, bench, H)
    if os.environ.get("YODA_NATIVE_PROF"):
        return _native(args, out, bench, H)
    # YODA_PROF_CPU=1: the interpreter thread's CPU time (waits on locks and the GIL excluded)
    pr = cProfile.Profile(__import__("time").thread_time) if os.environ.get("YODA_PROF_CPU") else cProfile.Profile()
    for cls in (H.Shard, H.HttpShard):
        orig = cls.burst

        def wrap(orig):
            async def burst(self, tag="b", timeout=600.0):
                if tag.startswith("s"):
                    pr.enable()
                try:
                    return await orig(self, tag, timeout)
                finally:
                    pr.disable()
            return burst
        cls.burst = wrap(orig)
    bench.main(args)
    if os.environ.get("YODA_PROF_DUMP"):
        pr.dump_stats(os.environ["YODA_PROF_DUMP"])
    st = pstats.Stats(pr)
    total = sum(v[2] for v in st.stats.values())
    groups = {name: 0.0 for name, _ in STAGES}
    groups["other"] = 0.0
    for (fn, _line, func), v in st.stats.items():
        key = f"{fn.replace(ROOT + '/', '')}:{func}"
        for name, pats in STAGES:
            if any(p in key for p in pats):
                groups[name] += v[2]
                break
        else:
            groups["other"] += v[2]
    s = io.StringIO()
    s.write(f"profiled CPU (own time, all functions): {total:.3f} s\n")
    for name, t in sorted(groups.items(), key=lambda kv: -kv[1]):
        s.write(f"  {100 * t / total:5.1f} %  {t:.3f} s  {name}\n")
    s.write("\n")
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
    if os.environ.get("YODA_PROF_CUM"):
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(int(os.environ["YODA_PROF_CUM"]))
    text = s.getvalue()
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text)
    return 0


def _sample(args, out, bench, H) -> int:
    """YODA_PROF_SAMPLE=1: a statistical profile instead of cProfile (no per-call
    overhead, so cheap functions are not inflated): a thread samples the interpreter
    thread's stack every ~0.5 ms during the timed bursts; prints self and inclusive
    sample shares per function."""
    import collections
    import threading
    import time

    main = threading.main_thread().ident
    on = [False]
    self_c, incl_c = collections.Counter(), collections.Counter()
    n = [0]

    def sampler():
        while not stop.is_set():
            time.sleep(0.0005)
            if not on[0]:
                continue
            f = sys._current_frames().get(main)
            if f is None:
                continue
            n[0] += 1
            seen = set()
            first = True
            while f is not None:
                co = f.f_code
                key = f"{co.co_filename.replace(ROOT + '/', '')}:{co.co_firstlineno}({co.co_name})"
                if first:
                    self_c[key] += 1
                    first = False
                if key not in seen:
                    incl_c[key] += 1
                    seen.add(key)
                f = f.f_back
    stop = threading.Event()
    sys.setswitchinterval(1e-4)      # let the sampler take the GIL between bytecodes
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    for cls in (H.Shard, H.HttpShard):
        orig = cls.burst

        def wrap(orig):
            async def burst(self, tag="b", timeout=600.0):
                on[0] = tag.startswith("s")
                try:
                    return await orig(self, tag, timeout)
                finally:
                    on[0] = False
            return burst
        cls.burst = wrap(orig)
    bench.main(args)
    stop.set()
    s = io.StringIO()
    s.write(f"samples: {n[0]}\n\nself %:\n")
    for k, v in self_c.most_common(40):
        s.write(f"  {100 * v / max(1, n[0]):5.1f}  {k}\n")
    s.write("\ninclusive %:\n")
    for k, v in incl_c.most_common(60):
        s.write(f"  {100 * v / max(1, n[0]):5.1f}  {k}\n")
    text = s.getvalue()
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text)
    return 0


def _native(args, out, bench, H) -> int:
    """YODA_NATIVE_PROF=<period us>: flat profile of the native threads (yoda-io, yoda-lane,
    yoda-engine) over the timed bursts (native/core/sampler.cpp, utils/native_prof.py)."""
    import tempfile
    from yoda_scheduler_amd.utils.native_prof import load_dump, maybe_sampler
    smp = maybe_sampler()
    # the native fake apiserver (http transport) samples itself for its whole life
    api_dump = os.path.join(tempfile.mkdtemp(prefix="yoda-apiprof-"), "apiserver.samples")
    os.environ["YODA_APISERVER_PROF"] = api_dump
    # YODA_NATIVE_PROF_PHASE=reset: sample only while the previous burst is being deleted
    reset_only = os.environ.get("YODA_NATIVE_PROF_PHASE") == "reset"
    for cls in (H.Shard, H.HttpShard):
        orig = cls.burst

        def wrap(orig):
            async def burst(self, tag="b", timeout=600.0):
                on = tag.startswith("s")
                if reset_only:
                    self.phase_hook = (lambda ph, started: (smp.start() if started else smp.stop())) if on else None
                    return await orig(self, tag, timeout)
                if on:
                    smp.start()
                try:
                    return await orig(self, tag, timeout)
                finally:
                    if on:
                        smp.stop()
            return burst
        cls.burst = wrap(orig)
    bench.main(args)
    top = int(os.environ.get("YODA_PROF_TOP", "35"))
    text = smp.report(top=top)
    if os.path.exists(api_dump):
        text += "\n\nfake apiserver process, whole life (start-up and warmup included):\n" + \
            load_dump(api_dump, period_us=smp.period_us).report(top=top)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
