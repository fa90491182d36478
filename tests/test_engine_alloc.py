"""The engine ledger allocates nothing for pods of known templates.

``native/core/alloc_probe.cpp`` replaces the global operator new with a counting one and
reserves / releases pods through ``Engine::reserve`` / ``Engine::release``: 10 000 one-at-a-time
cycles and ten 1000-pod bursts (the bench pattern: every step deletes the previous burst). Both
must make zero allocations once the slab, label-set table and node indices are warm. Round 5's
engine made 10 per churn cycle and ~5 per burst pod (a label copy per reserve, a LabSet
temporary per index update, a hash-map node per ledger entry) — the regression this pins.
"""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "native")


def test_reserve_release_of_templated_pods_allocates_nothing(tmp_path):
    exe = tmp_path / "alloc_probe"
    subprocess.run(["g++", "-std=c++17", "-O2", f"-I{NATIVE}/core", f"-I{NATIVE}/hip", f"-I{NATIVE}/kube",
                    f"-I{NATIVE}/common", f"{NATIVE}/core/engine.cpp", f"{NATIVE}/core/alloc_probe.cpp",
                    "-o", str(exe), "-lpthread", "-ldl"], check=True, timeout=300)
    out = subprocess.run([str(exe), "10000", "10"], check=True, capture_output=True, text=True, timeout=120)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["churn_allocs"] == 0, r
    assert r["burst_allocs"] == 0, r
    assert r["ledger"] == 0 and r["labsets"] == 4, r


def test_watch_event_record_stays_small():
    """Every pod watch event allocates one PodEv on the transport's I/O thread, fills it, and
    frees it on the lane thread, so each byte of it is paid on every event. Round 5 grew it from
    984 to 1184 bytes (PodScheduled condition strings, owner references by value). On one MI355X
    box that cost 143.5k vs 154.2k pods/s, and the reset grew from 1.46 to 1.94 ms (a same-box
    bisect, profiles/bench/r6/bisect/). Optional parts now live behind shared records: 528 bytes."""
    from yoda_scheduler_amd.ops.native import load_native
    k = load_native("kube", "yoda_scheduler_amd._native._yoda_kube")
    assert k.SIZEOF_POD_EV <= 576, k.SIZEOF_POD_EV
