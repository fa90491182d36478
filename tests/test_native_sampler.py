"""The native-thread CPU sampler (native/core/sampler.cpp, utils/native_prof.py)."""
import os
import threading

from yoda_scheduler_amd.utils.native_prof import NativeSampler, threads_by_name


def _spin(stop: threading.Event) -> None:
    x = 0
    while not stop.is_set():
        for i in range(10_000):
            x += i * i


def test_sampler_samples_a_named_busy_thread_and_symbolises_it():
    stop = threading.Event()
    th = threading.Thread(target=_spin, args=(stop,), name="spin")
    th.start()
    try:
        # Python names its threads in comm only on 3.12+: set it by tid here
        tid = th.native_id
        with open(f"/proc/self/task/{tid}/comm", "w") as f:
            f.write("yoda-spin")
        assert threads_by_name(["yoda-spin"]) == {tid: "yoda-spin"}
        for stacks in (False, True):
            s = NativeSampler(("yoda-spin",), period_us=500, stacks=stacks)
            s.start()
            t_end = os.times().elapsed + 0.6
            while os.times().elapsed < t_end:
                pass
            s.stop()
            assert s.samples, "no samples from a busy thread"
            rows = s.symbolise()
            assert {t for t, _, _ in rows} == {"yoda-spin"}
            assert sum(w for _, w, _ in rows) >= len(rows) >= 1
            # the spinning thread runs the interpreter loop
            mods = {syms[0][0] for _, _, syms in rows}
            assert any(m.startswith(("python", "libpython")) for m in mods), mods
            if stacks:
                assert any(len(syms) > 1 for _, _, syms in rows)
            rep = s.report(top=5)
            assert "[yoda-spin]" in rep
    finally:
        stop.set()
        th.join()
