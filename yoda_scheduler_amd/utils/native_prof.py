"""Flat CPU profile of the scheduler's native threads (``native/core/sampler.cpp``).

The Python samplers (``scripts/profile_bench.py``) see only the interpreter thread; the
headline burst runs on ``yoda-io`` (transport, watch decode) and ``yoda-lane`` (pod lane,
engine). ``NativeSampler`` arms one CPU-time timer per named thread, and ``report()``
symbolises the sampled program counters with ``/proc/self/maps`` + ``addr2line``:
self-time shares per function, per thread.

    s = NativeSampler(("yoda-io", "yoda-lane"))
    s.start(); ...; s.stop()
    print(s.report())
"""
from __future__ import annotations

import collections
import os
import shutil
import subprocess
from typing import Iterable, Optional


def threads_by_name(names: Iterable[str]) -> dict[int, str]:
    """tid → name of this process's threads whose comm is one of ``names``."""
    want = set(names)
    out: dict[int, str] = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/comm") as f:
                nm = f.read().strip()
        except OSError:
            continue
        if nm in want:
            out[int(tid)] = nm
    return out


def _maps(path: str = "/proc/self/maps") -> list[tuple[int, int, int, str]]:
    """Executable mappings: (start, end, file offset, path)."""
    out = []
    with open(path) as f:
        for ln in f:
            parts = ln.split()
            if len(parts) < 6 or "x" not in parts[1] or not parts[5].startswith(("/", "[vdso]")):
                continue
            a, b = (int(x, 16) for x in parts[0].split("-"))
            out.append((a, b, int(parts[2], 16), parts[5]))
    return out


def _addr2line(path: str, offs: list[int]) -> dict[int, str]:
    tool = shutil.which("addr2line") or "/opt/rocm/lib/llvm/bin/llvm-addr2line"
    try:
        res = subprocess.run([tool, "-f", "-C", "-e", path, *[hex(o) for o in offs]],
                             capture_output=True, text=True, timeout=120)
    except (OSError, subprocess.TimeoutExpired):
        return {}
    lines = res.stdout.splitlines()
    return {o: lines[2 * i] for i, o in enumerate(offs) if 2 * i < len(lines)}


class NativeSampler:
    def __init__(self, names: Iterable[str] = ("yoda-io", "yoda-lane", "yoda-engine"), period_us: int = 200,
                 stacks: bool = False) -> None:
        from ..ops.native import core as core_module
        self._core = core_module()
        self.names = tuple(names)
        self.period_us = period_us
        self.stacks = stacks
        self.samples: list[tuple[int, int, list]] = []
        self.dropped = 0
        self.tids: dict[int, str] = {}
        self.maps_file = "/proc/self/maps"

    def start(self) -> None:
        self.tids.update(threads_by_name(self.names))
        self._core.sampler_start(list(self.tids), self.period_us, self.stacks)

    def stop(self) -> None:
        s, d = self._core.sampler_stop()
        self.samples.extend(s)
        self.dropped += d

    def _frames(self, pc: int, st: list) -> list[int]:
        """Interrupted PC, then its callers (return address - 1): the handler's own frame
        and the signal trampoline are dropped."""
        if not st:
            return [pc]
        try:
            k = st.index(pc)
            callers = st[k + 1:]
        except ValueError:
            callers = st[2:]
        return [pc] + [a - 1 for a in callers]

    def symbolise(self) -> list[tuple[str, int, list[tuple[str, str]]]]:
        """(thread, weight in periods, [(module basename, function), leaf first]) per sample."""
        maps = _maps(self.maps_file)
        where: dict[int, tuple[str, int]] = {}
        per_file: dict[str, set[int]] = collections.defaultdict(set)
        frames = [self._frames(pc, st) for pc, _tw, st in self.samples]
        for fr in frames:
            for pc in fr:
                if pc in where:
                    continue
                for a, b, off, path in maps:
                    if a <= pc < b:
                        o = pc - a + off
                        where[pc] = (path, o)
                        per_file[path].add(o)
                        break
                else:
                    where[pc] = ("?", pc)
        names: dict[tuple[str, int], str] = {}
        for path, offs in per_file.items():
            if not path.startswith("/"):
                continue                     # [vdso]: clock_gettime & co
            srt = sorted(offs)
            for i in range(0, len(srt), 2000):
                for o, fn in _addr2line(path, srt[i:i + 2000]).items():
                    names[(path, o)] = fn
        out = []
        for (pc, tw, _st), fr in zip(self.samples, frames):
            tid, w = tw & 0xFFFFFF, 1 + (tw >> 24)
            syms = []
            for a in fr:
                path, o = where[a]
                fn = names.get((path, o), "??")
                if fn == "??":
                    fn = f"?? ({os.path.basename(path)}+{o:#x})" if path != "?" else "??"
                syms.append((os.path.basename(path), fn))
            out.append((self.tids.get(tid, str(tid)), w, syms))
        return out

    def report(self, top: int = 30, width: int = 110) -> str:
        """Per thread: self time by module and by function (leaf frame), and, with stacks, by
        the first frame outside the C/C++ runtime (who called malloc, memcpy, ...)."""
        rows = self.symbolise()
        by_thread: collections.Counter = collections.Counter()
        for t, w, _ in rows:
            by_thread[t] += w
        s = [f"native samples: {len(rows)} (period {self.period_us} us of thread CPU, weighted by timer overruns; "
             f"dropped {self.dropped})"]
        for th, n in by_thread.most_common():
            s.append(f"\n[{th}] {n} periods = {n * self.period_us / 1e6:.3f} s CPU")
            mods: collections.Counter = collections.Counter()
            fns: collections.Counter = collections.Counter()
            owner: collections.Counter = collections.Counter()
            user: collections.Counter = collections.Counter()
            for t, w, syms in rows:
                if t != th:
                    continue
                mods[syms[0][0]] += w
                fns[syms[0][1]] += w
                if len(syms) > 1:
                    own = next((f for m, f in syms if not m.startswith(_RUNTIME)), syms[-1][1])
                    owner[own] += w
                    usr = next((f for m, f in syms if not m.startswith(_RUNTIME) and not _is_std(f)), syms[-1][1])
                    user[usr] += w
            s.append("  by module: " + ", ".join(f"{m} {100 * c / n:.1f}%" for m, c in mods.most_common(6)))
            s.append("  self (leaf function; stripped libc names are the nearest exported symbol):")
            for fn, c in fns.most_common(top):
                s.append(f"  {100 * c / n:5.1f}%  {fn[:width]}")
            if owner:
                s.append("  self with runtime calls charged to their caller:")
                for fn, c in owner.most_common(top):
                    s.append(f"  {100 * c / n:5.1f}%  {fn[:width]}")
                s.append("  self with runtime and std:: template calls charged to their caller:")
                for fn, c in user.most_common(top):
                    s.append(f"  {100 * c / n:5.1f}%  {fn[:width]}")
        return "\n".join(s)


def _is_std(fn: str) -> bool:
    f = fn[5:] if fn.startswith("void ") else fn
    return f.startswith(("std::", "__gnu_cxx::", "operator new", "operator delete"))


_RUNTIME = ("libc.so", "libstdc++.so", "libgcc_s.so", "ld-linux", "libm.so", "[vdso]", "?")


def load_dump(path: str, thread: str = "apiserver", period_us: int = 200) -> NativeSampler:
    """The samples another process wrote with ``yoda_sampler::dump`` (the native fake
    apiserver under ``YODA_APISERVER_PROF``), ready for ``report()``."""
    s = NativeSampler.__new__(NativeSampler)
    s.names, s.period_us, s.stacks, s.dropped = (thread,), period_us, False, 0
    s.samples, s.tids, s.maps_file = [], {}, path + ".maps"
    with open(path) as f:
        for ln in f:
            if ln.startswith("#"):
                s.dropped = int(ln.split()[-1])
                continue
            v = [int(x, 16) for x in ln.split()]
            if len(v) >= 2:
                s.samples.append((v[0], v[1], v[2:]))
                s.tids[v[1] & 0xFFFFFF] = thread
    s.stacks = any(st for _, _, st in s.samples)
    return s


def maybe_sampler() -> Optional[NativeSampler]:
    """A sampler when ``YODA_NATIVE_PROF`` is set (its value: period in µs, default 200);
    ``YODA_NATIVE_PROF_STACKS=1`` also records callers."""
    v = os.environ.get("YODA_NATIVE_PROF")
    if not v:
        return None
    return NativeSampler(period_us=int(v) if v.isdigit() and int(v) > 1 else 200,
                         stacks=bool(os.environ.get("YODA_NATIVE_PROF_STACKS")))
