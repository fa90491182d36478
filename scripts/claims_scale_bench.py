#!/usr/bin/env python3
"""Cost of keeping the native lane's claim table (plugins/volumes.py::LaneClaims) at cluster
scale: the first (full) refresh, and one PVC event's incremental refresh, against a full
recompute over every PVC (what a per-event recompute would cost).

    python scripts/claims_scale_bench.py
"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from types import SimpleNamespace
from yoda_scheduler_amd.plugins.volumes import LaneClaims, lane_claims

class H:
    def __init__(self, n):
        self.objs = {"persistentvolumeclaims": {}, "persistentvolumes": {}, "csinodes": {}, "storageclasses": {}}
        self.gen = collections.Counter()
        self.cache = SimpleNamespace(csi_limit_drivers={})
        for i in range(n):
            pv = {"metadata": {"name": f"pv{i}", "labels": {}}, "spec": {"csi": {"driver": "nfs", "volumeHandle": f"h{i}"},
                  **({"nodeAffinity": {"required": {"nodeSelectorTerms": [{"matchExpressions": [{"key": "kubernetes.io/hostname", "operator": "In", "values": [f"n{i%64}"]}]}]}}} if i % 2 else {})}}
            self.objs["persistentvolumes"][f"pv{i}"] = pv
            self.objs["persistentvolumeclaims"][f"default/c{i}"] = {"metadata": {"name": f"c{i}", "namespace": "default"}, "spec": {"volumeName": f"pv{i}"}}
    def lister(self, r): return self.objs[r]
    def generation(self, r): return self.gen[r]

for n in (1000, 10000, 50000):
    h = H(n)
    t = LaneClaims(h)
    t0 = time.perf_counter(); t.refresh(); full = time.perf_counter() - t0
    t1 = time.perf_counter()
    for i in range(1000):
        obj = h.objs["persistentvolumeclaims"][f"default/c{i}"]
        t.pvc_event(obj); t.refresh()
    ev = (time.perf_counter() - t1) / 1000
    t2 = time.perf_counter(); lane_claims(h); rec = time.perf_counter() - t2
    print(f"{n} claims: first refresh {full*1e3:.1f} ms, per PVC event {ev*1e6:.1f} us (a full recompute: {rec*1e3:.1f} ms)")
