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


def test_load_dump_symbolises_another_process_samples(tmp_path):
    """The fake apiserver writes its samples with yoda_sampler::dump (pc, tid|overrun<<24,
    callers; plus its maps); load_dump reads them back for report()."""
    from yoda_scheduler_amd.utils.native_prof import load_dump
    import ctypes
    # a PC inside this process's libc (its maps double as the other process's)
    pc = ctypes.cast(ctypes.CDLL(None).malloc, ctypes.c_void_p).value
    dump = tmp_path / "apiserver.samples"
    dump.write_text(f"# dropped 3\n{pc:x} {(2 << 24) | 4242:x}\n{pc + 1:x} {4242:x} {pc:x}\n")
    with open("/proc/self/maps") as f:
        (tmp_path / "apiserver.samples.maps").write_text(f.read())
    s = load_dump(str(dump), period_us=1000)
    assert s.dropped == 3 and len(s.samples) == 2 and s.stacks
    rows = s.symbolise()
    assert [w for _, w, _ in rows] == [3, 1]
    assert all(t == "apiserver" and syms[0][0].startswith("libc") for t, _, syms in rows)
    assert "[apiserver] 4 periods" in s.report()
