"""ctypes binding of ``libyoda_hip.so`` (gfx950 kernels, C ABI).

Runtime note: PyTorch-ROCm wheels bundle their own ``libamdhip64.so`` with SONAME
``libamdhip64.so.7`` — the same SONAME as ``/opt/rocm``'s. Whichever is loaded first
serves both, so processes that use torch import it *before* this library: kernels
launched here and tensors allocated by torch then share one HIP runtime and device
context. Processes without torch (sniffer, scheduler) use ``/opt/rocm`` directly.

There is no silent fallback: if the library is missing it is built in-tree, and if
it cannot be loaded the call raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path
from typing import Optional

_LIB: Optional[ctypes.CDLL] = None
_lock = threading.Lock()
# YODA_HIP_LIB points at another build of the kernels (same-box A/B of kernel variants)
PATH = Path(os.environ.get("YODA_HIP_LIB") or Path(__file__).resolve().parents[1] / "_native" / "libyoda_hip.so")

c_int, c_uint, c_ull, c_double, c_float, c_char_p, c_void_p = (
    ctypes.c_int, ctypes.c_uint, ctypes.c_ulonglong, ctypes.c_double, ctypes.c_float, ctypes.c_char_p,
    ctypes.c_void_p)


class HipError(RuntimeError):
    pass


def _declare(lib: ctypes.CDLL) -> None:
    P = ctypes.POINTER
    sigs = {
        "yoda_hip_device_count": [P(c_int)],
        "yoda_hip_device_info": [c_int, c_char_p, c_int, P(c_int), P(c_ull), P(c_int)],
        "yoda_hbm_bandwidth": [c_int, c_ull, c_int, P(c_double), P(c_double)],
        "yoda_hbm_pattern_check": [c_int, c_ull, c_uint, P(c_ull), P(c_float)],
        "yoda_hbm_pattern_check2": [c_int, c_ull, c_uint, c_uint, P(c_ull), P(c_float)],
        "yoda_hip_pci_bus_id": [c_int, c_char_p, c_int],
        "yoda_peer_write_bandwidth": [c_int, c_int, c_ull, c_int, P(c_double), P(c_int)],
        "yoda_hip_occupy": [c_int, c_int, P(c_int)],
        "yoda_hip_occupy_wait": [c_int],
    }
    for name, args in sigs.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = c_int
    try:
        from . import device_scorer as _ds
    except ImportError:
        return
    _ds.declare(lib)


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    with _lock:
        if _LIB is None:
            # No torch import here: a scheduler process should not pay for torch. Processes
            # that use torch (bench, smoke, GPU tests) import it first, so the shared SONAME
            # resolves our NEEDED entry to torch's already-loaded runtime.
            from . import build
            if "YODA_HIP_LIB" not in os.environ:
                build.ensure_fresh("hip")         # missing or built from other sources: rebuild
            l = ctypes.CDLL(str(PATH), mode=ctypes.RTLD_GLOBAL)
            _declare(l)
            if "YODA_HIP_LIB" not in os.environ and (build.NATIVE / "common" / "build_id.h").exists():
                build.verify_loaded("hip", build_id(l))
            _LIB = l
    return _LIB


def build_id(l: Optional[ctypes.CDLL] = None) -> str:
    """Source hash compiled into the loaded ``libyoda_hip.so`` (``ops/build.py``)."""
    l = l if l is not None else lib()
    f = getattr(l, "yoda_build_id", None)
    if f is None:
        return ""
    f.argtypes, f.restype = [], c_char_p
    return (f() or b"").decode()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise HipError(f"{what} failed with hipError {rc}")


def device_count() -> int:
    n = c_int(0)
    rc = lib().yoda_hip_device_count(ctypes.byref(n))
    return 0 if rc else n.value


def device_info(device: int = 0) -> dict:
    arch = ctypes.create_string_buffer(64)
    cus, hbm, clk = c_int(0), c_ull(0), c_int(0)
    _check(lib().yoda_hip_device_info(device, arch, 64, ctypes.byref(cus), ctypes.byref(hbm), ctypes.byref(clk)),
           "hipGetDeviceProperties")
    return {"arch": arch.value.decode(), "cus": cus.value, "hbm_bytes": hbm.value, "clock_khz": clk.value}


def pci_bus_id(device: int = 0) -> str:
    """Lower-case PCI address of a HIP ordinal (amd-smi's ``bdf`` format)."""
    buf = ctypes.create_string_buffer(64)
    _check(lib().yoda_hip_pci_bus_id(device, buf, 64), "pci_bus_id")
    return buf.value.decode().strip().lower()


def hbm_bandwidth(device: int = 0, nbytes: int = 1 << 30, iters: int = 10) -> dict:
    r, c = c_double(0), c_double(0)
    _check(lib().yoda_hbm_bandwidth(device, nbytes, iters, ctypes.byref(r), ctypes.byref(c)), "hbm_bandwidth")
    return {"read_gbps": r.value, "copy_gbps": c.value, "bytes": nbytes, "iters": iters}


def hbm_pattern_check(device: int = 0, nbytes: int = 1 << 30, seed: int = 0x5eed,
                      verify_seed: int | None = None) -> dict:
    """Fill ``nbytes`` of HBM with a seeded pattern and count mismatching 32-bit words on
    read-back. ``verify_seed`` ≠ ``seed`` is the verifier's self-test (all words differ)."""
    err, ms = c_ull(0), c_float(0)
    vs = seed if verify_seed is None else verify_seed
    _check(lib().yoda_hbm_pattern_check2(device, nbytes, seed, vs, ctypes.byref(err), ctypes.byref(ms)),
           "hbm_pattern")
    return {"errors": err.value, "ms": ms.value, "bytes": nbytes, "words": nbytes // 4}


def peer_write_bandwidth(src: int, dst: int, nbytes: int = 256 << 20, iters: int = 10) -> dict:
    g, sup = c_double(0), c_int(0)
    _check(lib().yoda_peer_write_bandwidth(src, dst, nbytes, iters, ctypes.byref(g), ctypes.byref(sup)),
           "peer_write_bandwidth")
    return {"gbps": g.value, "supported": bool(sup.value)}


def occupy(device: int = 0, ms: int = 1000) -> int:
    """Hold every CU of ``device`` (its LDS and wave slots) for ``ms`` milliseconds with a
    bounded kernel on a stream of its own; returns the block count at once. Test utility: the
    "tenant kernel" the device scorer must survive (tests/test_gpu_device_scorer.py)."""
    blocks = c_int(0)
    _check(lib().yoda_hip_occupy(device, ms, ctypes.byref(blocks)), "occupy")
    return blocks.value


def occupy_wait(device: int = 0) -> None:
    _check(lib().yoda_hip_occupy_wait(device), "occupy_wait")
