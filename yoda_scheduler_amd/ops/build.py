"""In-tree build of every native artefact (``python -m yoda_scheduler_amd.ops.build``).

* ``_yoda_core``    C++17 scheduling engine (pybind11, g++)            native/core/
* ``_yoda_sniffer`` C++ amd-smi collector (pybind11, links libamd_smi)  native/sniffer/
* ``yoda-sniffer``  standalone collector binary (JSON on stdout)        native/sniffer/
* ``libyoda_hip``   gfx950 HIP kernels: batched placement scorer, HBM /
                    xGMI probes (hipcc --offload-arch=gfx950, C ABI)    native/hip/

Outputs land in ``yoda_scheduler_amd/_native/`` so they travel with the repo snapshot
to the GPU box. Rebuilds are mtime-driven; ``--force`` rebuilds everything.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
NATIVE = ROOT / "native"
OUT = ROOT / "yoda_scheduler_amd" / "_native"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("YODA_HIP_ARCH", "gfx950")


def _pybind_includes() -> list[str]:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _stale(target: Path, sources: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(s.stat().st_mtime > t for s in sources)


def _run(cmd: list[str], what: str) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build of {what} failed: {' '.join(cmd)}")


def build_core(force: bool = False) -> Path:
    srcs = [NATIVE / "core" / "engine.cpp", NATIVE / "core" / "bindings.cpp"]
    deps = srcs + [NATIVE / "core" / "engine.hpp", NATIVE / "hip" / "yoda_dev_abi.h"]
    out = OUT / f"_yoda_core{EXT}"
    if force or _stale(out, deps):
        cxx = os.environ.get("CXX", "g++")
        _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-Wall",
              "-Wno-unused-function", *_pybind_includes(), f"-I{NATIVE / 'core'}", f"-I{NATIVE / 'hip'}",
              *map(str, srcs), "-o", str(out), "-lpthread", "-ldl"], "core")
    return out


def build_sniffer(force: bool = False) -> list[Path]:
    src = NATIVE / "sniffer"
    lib_srcs = [src / "collector.cpp"]
    deps = lib_srcs + [src / "collector.hpp", src / "bindings.cpp", src / "main.cpp"]
    outs = []
    inc = [f"-I{ROCM / 'include'}", f"-I{src}"]
    link = [f"-L{ROCM / 'lib'}", "-lamd_smi", f"-Wl,-rpath,{ROCM / 'lib'}"]
    mod = OUT / f"_yoda_sniffer{EXT}"
    if force or _stale(mod, deps):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", *inc,
              *_pybind_includes(), *map(str, lib_srcs), str(src / "bindings.cpp"), "-o", str(mod), *link],
             "sniffer module")
    outs.append(mod)
    exe = OUT / "yoda-sniffer"
    if force or _stale(exe, deps):
        _run(["g++", "-O2", "-std=c++17", *inc, *map(str, lib_srcs), str(src / "main.cpp"), "-o", str(exe),
              *link], "sniffer binary")
    outs.append(exe)
    return outs


def hipcc() -> str:
    h = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    return h


def build_hip(force: bool = False) -> Path:
    src = NATIVE / "hip"
    srcs = sorted(src.glob("*.hip"))
    deps = srcs + sorted(src.glob("*.h"))
    out = OUT / "libyoda_hip.so"
    if force or _stale(out, deps):
        _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-Wall", "-Wno-unused-result", "-Wno-unused-value", f"-I{src}", *map(str, srcs), "-o", str(out)], "hip kernels")
    return out


def build_all(force: bool = False, hip: bool = True, sniffer: bool = True) -> list[Path]:
    OUT.mkdir(parents=True, exist_ok=True)
    (OUT / "__init__.py").touch()
    jobs = [lambda: [build_core(force)]]
    if sniffer:
        jobs.append(lambda: build_sniffer(force))
    if hip:
        jobs.append(lambda: [build_hip(force)])
    outs: list[Path] = []
    with ThreadPoolExecutor(len(jobs)) as ex:
        for r in ex.map(lambda f: f(), jobs):
            outs.extend(r)
    return outs


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--no-hip", action="store_true")
    ap.add_argument("--no-sniffer", action="store_true")
    a = ap.parse_args(argv)
    for p in build_all(a.force, hip=not a.no_hip, sniffer=not a.no_sniffer):
        print(p.relative_to(ROOT))
    return 0


if __name__ == "__main__":
    sys.exit(main())
