#!/usr/bin/env python3
"""Build and run the native engine stress driver under sanitizers:
ASan+UBSan (memory errors, UB) and TSan (the ThreadPool used by the parallel filter).
Host code only — GPU sanitizers are not part of this pool."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORE = os.path.join(ROOT, "native", "core")
HIP = os.path.join(ROOT, "native", "hip")

VARIANTS = {
    "asan-ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}


SNIFFER = os.path.join(ROOT, "native", "sniffer")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def run_sniffer(variant: str = "asan-ubsan", iters: int = 3000) -> int:
    """The amd-smi collector's host code (JSON encoding fuzz + real sampling when a
    driver is present) under ASan+UBSan; the emitted JSON must parse."""
    import json
    out = os.path.join(tempfile.gettempdir(), f"yoda_sniffer_stress_{variant}")
    cmd = ["g++", "-std=c++17", "-O1", "-g", *VARIANTS[variant], f"-I{ROCM}/include",
           os.path.join(SNIFFER, "collector.cpp"), os.path.join(SNIFFER, "stress_main.cpp"), "-o", out,
           f"-L{ROCM}/lib", "-lamd_smi", f"-Wl,-rpath,{ROCM}/lib", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr)
        return r.returncode
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([out, str(iters)], capture_output=True, text=True, env=env, timeout=600)
    sys.stdout.write(f"[sniffer-{variant}] {r.stderr.strip()[-300:]}\n")
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-4000:])
        return r.returncode
    doc = json.loads(r.stdout.strip().splitlines()[-1])
    assert isinstance(doc, list) and len(doc) == 8, doc
    return 0


def run(variant: str, nodes: int = 700, steps: int = 2000, threads: int = 4) -> int:
    # > 512 nodes so the ThreadPool parallel filter/score paths run under TSan
    flags = VARIANTS[variant]
    out = os.path.join(tempfile.gettempdir(), f"yoda_stress_{variant}")
    cmd = ["g++", "-std=c++17", "-O1", "-g", *flags, f"-I{CORE}", f"-I{HIP}",
           os.path.join(CORE, "engine.cpp"), os.path.join(CORE, "stress_main.cpp"), "-o", out, "-lpthread", "-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr)
        return r.returncode
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    argv = [out, str(nodes), str(steps), str(threads)]
    if variant == "tsan" and shutil.which("setarch"):
        # TSan's shadow layout can collide with a randomised mmap base on recent kernels
        # ("unexpected memory mapping"); run the driver with ASLR off
        argv = ["setarch", os.uname().machine, "-R", *argv]
    r = subprocess.run(argv, capture_output=True, text=True, env=env, timeout=600)
    sys.stdout.write(f"[{variant}] {r.stdout}")
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-4000:])
    return r.returncode


KUBE = os.path.join(ROOT, "native", "kube")
COMMON = os.path.join(ROOT, "native", "common")


def run_lane(variant: str, bursts: int = 6, pods: int = 400) -> int:
    """The native pod lane (native/core/lane_stress.cpp): lane thread, a fake transport I/O
    thread answering Bindings and echoing pods, and the caller feeding bursts and deletions —
    the ledger must be exact after every burst and every deletion wave."""
    flags = VARIANTS[variant]
    out = os.path.join(tempfile.gettempdir(), f"yoda_lane_stress_{variant}")
    srcs = [os.path.join(CORE, f) for f in ("lane_stress.cpp", "lane.cpp", "engine.cpp")] + \
        [os.path.join(KUBE, f) for f in ("json.cpp", "flatjson.cpp", "project.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", *flags, f"-I{CORE}", f"-I{HIP}", f"-I{KUBE}", f"-I{COMMON}", *srcs,
           "-o", out, "-lpthread", "-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stderr)
        return r.returncode
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    argv = [out, str(bursts), str(pods), "64"]
    if variant == "tsan" and shutil.which("setarch"):
        argv = ["setarch", os.uname().machine, "-R", *argv]
    r = subprocess.run(argv, capture_output=True, text=True, env=env, timeout=600)
    sys.stdout.write(f"[lane-{variant}] {r.stdout}")
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-4000:])
    return r.returncode


def main() -> int:
    rc = 0
    for v in VARIANTS:
        rc |= run(v)
        rc |= run_lane(v)
    rc |= run_sniffer()
    return rc


if __name__ == "__main__":
    sys.exit(main())
