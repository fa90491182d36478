"""In-tree build of every native artefact (``python -m yoda_scheduler_amd.ops.build``).

* ``_yoda_core``    C++17 scheduling engine + native pod lane (pybind11)  native/core/
* ``_yoda_kube``    C++17 Kubernetes transport: pipelined HTTP/1.1 +
                    TLS, watch decoding, pod projection (pybind11)      native/kube/
* ``yoda-fake-apiserver-native`` epoll fake apiserver for HTTP benches  native/kube/
* ``_yoda_sniffer`` C++ amd-smi collector (pybind11, links libamd_smi)  native/sniffer/
* ``yoda-sniffer``  standalone collector binary (JSON on stdout)        native/sniffer/
* ``libyoda_hip``   gfx950 HIP kernels: batched placement scorer, HBM /
                    xGMI probes (hipcc --offload-arch=gfx950, C ABI)    native/hip/

Outputs land in ``yoda_scheduler_amd/_native/`` so they travel with the repo snapshot
to the GPU box.

Build provenance: each artefact's identity is :func:`source_hash` — a hash of its source
files' contents (relative paths + bytes) and its compile recipe. It is compiled in
(``-DYODA_BUILD_ID``: ``build_id()`` of the pybind modules, ``yoda_build_id()`` of the HIP
library, ``--build-id`` of the binaries) and written next to the artefact
(``<artefact>.buildid``). A rebuild happens when that hash changes — not on mtimes, which a
checkout or a copy to the GPU box rewrites — and :func:`verify_loaded` lets every importer
compare the id compiled into the library it actually loaded with the tree it runs from
(``YODA_BUILD_CHECK``: ``rebuild`` (default) | ``refuse`` | ``off``).
"""
from __future__ import annotations

import argparse
import hashlib
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

# Per artefact: output name, the sources compiled, every file whose contents define the
# artefact (sources + headers), and a recipe tag (bump it when the compile flags change).
CORE_SRCS = ["core/engine.cpp", "core/lane.cpp", "core/bindings.cpp", "core/sampler.cpp"]
KUBE_COMMON = ["kube/json.cpp", "kube/flatjson.cpp", "kube/project.cpp"]
ARTEFACTS: dict[str, dict] = {
    "core": {"out": f"_yoda_core{EXT}", "srcs": CORE_SRCS,
             "deps": CORE_SRCS + ["core/engine.hpp", "core/lane.hpp", "hip/yoda_dev_abi.h", "kube/project.hpp",
                                  "kube/json.hpp", "kube/flatjson.hpp", "kube/lane_port.hpp", "common/build_id.h"],
             "recipe": "g++ -O3 -std=c++17 -fPIC -shared -fvisibility=hidden v2"},
    "kube": {"out": f"_yoda_kube{EXT}", "srcs": KUBE_COMMON + ["kube/transport.cpp", "kube/bindings.cpp"],
             "deps": KUBE_COMMON + ["kube/transport.cpp", "kube/bindings.cpp", "kube/json.hpp", "kube/http.hpp",
                                    "kube/project.hpp", "kube/flatjson.hpp", "kube/transport.hpp", "kube/lane_port.hpp",
                                    "common/build_id.h"],
             "recipe": "g++ -O3 -std=c++17 -fPIC -shared -fvisibility=hidden -lssl -lcrypto v2"},
    "fakeapi": {"out": "yoda-fake-apiserver-native", "srcs": KUBE_COMMON + ["kube/fakeapi.cpp", "kube/fakeapi_main.cpp", "core/sampler.cpp"],
                "deps": KUBE_COMMON + ["kube/fakeapi.cpp", "kube/fakeapi_main.cpp", "core/sampler.cpp", "kube/fakeapi.hpp",
                                       "kube/json.hpp", "kube/flatjson.hpp", "kube/project.hpp", "kube/http.hpp",
                                       "common/build_id.h"],
                "recipe": "g++ -O3 -std=c++17 v2"},
    "sniffer": {"out": f"_yoda_sniffer{EXT}", "srcs": ["sniffer/collector.cpp", "sniffer/bindings.cpp"],
                "deps": ["sniffer/collector.cpp", "sniffer/collector.hpp", "sniffer/bindings.cpp",
                         "common/build_id.h"],
                "recipe": "g++ -O2 -std=c++17 -fPIC -shared -lamd_smi v2"},
    "sniffer_bin": {"out": "yoda-sniffer", "srcs": ["sniffer/collector.cpp", "sniffer/main.cpp"],
                    "deps": ["sniffer/collector.cpp", "sniffer/collector.hpp", "sniffer/main.cpp",
                             "common/build_id.h"],
                    "recipe": "g++ -O2 -std=c++17 -lamd_smi v2"},
    "hip": {"out": "libyoda_hip.so", "srcs": None, "deps": None,     # every native/hip/*.hip + *.h
            "recipe": f"hipcc --offload-arch={ARCH} -O3 -std=c++17 -fPIC -shared v2"},
}


class StaleArtefact(RuntimeError):
    """A loaded native library was not built from the sources of this tree."""


def _hip_files(native: Path) -> list[str]:
    src = native / "hip"
    return sorted(str(p.relative_to(native)) for p in list(src.glob("*.hip")) + list(src.glob("*.h")))


def deps_of(name: str, native: Path | None = None) -> list[str]:
    native = NATIVE if native is None else native
    a = ARTEFACTS[name]
    if name == "hip":
        return _hip_files(native) + ["common/build_id.h"]
    return list(a["deps"])


def source_hash(name: str, native: Path | None = None) -> str:
    """16-hex identity of artefact ``name`` as built from the sources under ``native``."""
    native = NATIVE if native is None else native
    h = hashlib.sha256()
    h.update(ARTEFACTS[name]["recipe"].encode())
    for rel in sorted(deps_of(name, native)):
        p = native / rel
        h.update(b"\0" + rel.encode() + b"\0")
        h.update(p.read_bytes() if p.exists() else b"<missing>")
    return h.hexdigest()[:16]


def out_path(name: str) -> Path:
    return OUT / ARTEFACTS[name]["out"]


def recorded_id(name: str) -> str:
    """The build id written next to the artefact when it was built ("" if none)."""
    p = out_path(name).with_name(out_path(name).name + ".buildid")
    try:
        return p.read_text().strip()
    except OSError:
        return ""


def _stale(name: str) -> bool:
    return not out_path(name).exists() or recorded_id(name) != source_hash(name)


def _record(name: str, bid: str) -> None:
    p = out_path(name)
    p.with_name(p.name + ".buildid").write_text(bid + "\n")


def _pybind_includes() -> list[str]:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _run(cmd: list[str], what: str) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build of {what} failed: {' '.join(cmd)}")


def _bid_flag(bid: str) -> str:
    return f'-DYODA_BUILD_ID="{bid}"'


def _srcs(name: str) -> list[str]:
    return [str(NATIVE / s) for s in ARTEFACTS[name]["srcs"]]


def build_core(force: bool = False) -> Path:
    out = out_path("core")
    if force or _stale("core"):
        bid = source_hash("core")
        cxx = os.environ.get("CXX", "g++")
        _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-Wall",
              "-Wno-unused-function", _bid_flag(bid), *_pybind_includes(), f"-I{NATIVE / 'core'}",
              f"-I{NATIVE / 'hip'}", f"-I{NATIVE / 'kube'}", f"-I{NATIVE / 'common'}", *_srcs("core"),
              "-o", str(out), "-lpthread", "-ldl", "-lrt"], "core")
        _record("core", bid)
    return out


def build_kube(force: bool = False) -> list[Path]:
    """Native Kubernetes transport (pybind module) + the native fake apiserver binary."""
    src = NATIVE / "kube"
    flags = ["-O3", "-std=c++17", "-Wall", "-Wno-unused-function", f"-I{src}", f"-I{NATIVE / 'common'}"]
    outs = []
    mod = out_path("kube")
    if force or _stale("kube"):
        bid = source_hash("kube")
        _run([os.environ.get("CXX", "g++"), *flags, _bid_flag(bid), "-fPIC", "-shared", "-fvisibility=hidden",
              *_pybind_includes(), *_srcs("kube"), "-o", str(mod), "-lssl", "-lcrypto", "-lpthread"],
             "kube transport")
        _record("kube", bid)
    outs.append(mod)
    if all((NATIVE / s).exists() for s in ARTEFACTS["fakeapi"]["srcs"]):
        exe = out_path("fakeapi")
        if force or _stale("fakeapi"):
            bid = source_hash("fakeapi")
            _run([os.environ.get("CXX", "g++"), *flags, _bid_flag(bid), *_srcs("fakeapi"), "-o", str(exe),
                  "-lpthread", "-lrt"], "native fake apiserver")
            _record("fakeapi", bid)
        outs.append(exe)
    return outs


def build_sniffer(force: bool = False) -> list[Path]:
    src = NATIVE / "sniffer"
    outs = []
    inc = [f"-I{ROCM / 'include'}", f"-I{src}", f"-I{NATIVE / 'common'}"]
    link = [f"-L{ROCM / 'lib'}", "-lamd_smi", f"-Wl,-rpath,{ROCM / 'lib'}"]
    mod = out_path("sniffer")
    if force or _stale("sniffer"):
        bid = source_hash("sniffer")
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", _bid_flag(bid), *inc,
              *_pybind_includes(), *_srcs("sniffer"), "-o", str(mod), *link], "sniffer module")
        _record("sniffer", bid)
    outs.append(mod)
    exe = out_path("sniffer_bin")
    if force or _stale("sniffer_bin"):
        bid = source_hash("sniffer_bin")
        _run(["g++", "-O2", "-std=c++17", _bid_flag(bid), *inc, *_srcs("sniffer_bin"), "-o", str(exe), *link],
             "sniffer binary")
        _record("sniffer_bin", bid)
    outs.append(exe)
    return outs


def hipcc() -> str:
    h = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    return h


def build_hip(force: bool = False) -> Path:
    src = NATIVE / "hip"
    srcs = sorted(src.glob("*.hip"))
    out = out_path("hip")
    if force or _stale("hip"):
        bid = source_hash("hip")
        _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", _bid_flag(bid),
              "-Wall", "-Wno-unused-result", "-Wno-unused-value", f"-I{src}", f"-I{NATIVE / 'common'}",
              *map(str, srcs), "-o", str(out)], "hip kernels")
        _record("hip", bid)
    return out


BUILDERS = {"core": lambda f: [build_core(f)], "kube": build_kube, "fakeapi": build_kube,
            "sniffer": build_sniffer, "sniffer_bin": build_sniffer, "hip": lambda f: [build_hip(f)]}


def verify_loaded(name: str, loaded_id: str, native: Path | None = None) -> None:
    """Compare the build id compiled into a library this process loaded with the tree's
    sources; raise :class:`StaleArtefact` on a mismatch (the caller decides whether to
    rebuild — only possible before the library is loaded — or to refuse)."""
    if os.environ.get("YODA_BUILD_CHECK", "rebuild") == "off":
        return
    want = source_hash(name, native)
    if loaded_id != want:
        raise StaleArtefact(f"{ARTEFACTS[name]['out']} was built from other sources (build id {loaded_id!r}, "
                            f"this tree {want!r}): rebuild with python -m yoda_scheduler_amd.ops.build")


def ensure_fresh(name: str) -> None:
    """Before loading artefact ``name``: rebuild it if its recorded build id does not match
    the sources (``YODA_BUILD_CHECK=rebuild``), or refuse (``refuse``)."""
    mode = os.environ.get("YODA_BUILD_CHECK", "rebuild")
    if mode == "off" or not (NATIVE / "common" / "build_id.h").exists():
        return                        # installed without sources: nothing to compare against
    if not _stale(name):
        return
    if mode == "refuse":
        raise StaleArtefact(f"{ARTEFACTS[name]['out']} is missing or stale against this tree's sources")
    OUT.mkdir(parents=True, exist_ok=True)
    (OUT / "__init__.py").touch()
    BUILDERS[name](False)


def build_ids() -> dict:
    """{artefact: (recorded build id, source hash)} for every artefact (smoke / diagnostics)."""
    return {n: (recorded_id(n), source_hash(n)) for n in ARTEFACTS}


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
    ap.add_argument("--ids", action="store_true", help="print recorded build id vs source hash per artefact")
    a = ap.parse_args(argv)
    if a.ids:
        for n, (rec, src) in build_ids().items():
            print(f"{n:12s} {rec or '-':16s} {src} {'ok' if rec == src else 'STALE'}")
        return 0
    for p in build_all(a.force, hip=not a.no_hip, sniffer=not a.no_sniffer):
        print(p.relative_to(ROOT))
    return 0


if __name__ == "__main__":
    sys.exit(main())
