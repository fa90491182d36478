"""In-tree build of every native artefact (``python -m yoda_scheduler_amd.ops.build``).

* ``_yoda_core``    C++17 scheduling engine (pybind11, g++)            native/core/
* ``_yoda_kube``    C++17 Kubernetes transport: pipelined HTTP/1.1 +
                    TLS, watch decoding, pod projection (pybind11)      native/kube/
* ``yoda-fake-apiserver-native`` epoll fake apiserver for HTTP benches  native/kube/
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


def build_kube(force: bool = False) -> list[Path]:
    """Native Kubernetes transport (pybind module) + the native fake apiserver binary."""
    src = NATIVE / "kube"
    common = [src / "json.cpp", src / "project.cpp"]
    deps = common + [src / "transport.cpp", src / "bindings.cpp", src / "json.hpp", src / "http.hpp",
                     src / "project.hpp", src / "transport.hpp"]
    flags = ["-O3", "-std=c++17", "-Wall", "-Wno-unused-function", f"-I{src}"]
    outs = []
    mod = OUT / f"_yoda_kube{EXT}"
    if force or _stale(mod, deps):
        _run([os.environ.get("CXX", "g++"), *flags, "-fPIC", "-shared", "-fvisibility=hidden", *_pybind_includes(),
              *map(str, common), str(src / "transport.cpp"), str(src / "bindings.cpp"), "-o", str(mod),
              "-lssl", "-lcrypto", "-lpthread"], "kube transport")
    outs.append(mod)
    fake_srcs = [src / "fakeapi.cpp", src / "fakeapi_main.cpp"]
    if all(p.exists() for p in fake_srcs):
        exe = OUT / "yoda-fake-apiserver-native"
        if force or _stale(exe, common + fake_srcs + [src / "fakeapi.hpp", src / "json.hpp", src / "http.hpp"]):
            _run([os.environ.get("CXX", "g++"), *flags, *map(str, common), *map(str, fake_srcs), "-o", str(exe),
                  "-lpthread"], "native fake apiserver")
        outs.append(exe)
    return outs


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
    jobs = [lambda: [build_core(force)], lambda: build_kube(force)]
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
