"""GPU identity end to end on CPU: amd-smi index (BDF order) vs HIP ordinal (KFD order)
vs ROCr UUID, CPX partitions (several logical GPUs per physical GPU), probe attribution,
probe safety (busy-GPU skip, sizing, N-strike Unhealthy + recovery) and change-driven
telemetry publishing."""
from __future__ import annotations

import asyncio
import time

from yoda_scheduler_amd.fakeapi.client import InProcessClient
from yoda_scheduler_amd.fakeapi.server import FakeApiServer
from yoda_scheduler_amd.models.device import make_node
from yoda_scheduler_amd.models.scv import Scv
from yoda_scheduler_amd.sniffer.collector import FakeBackend, samples_to_scv
from yoda_scheduler_amd.sniffer.publisher import SnifferAgent, hip_to_index
from yoda_scheduler_amd.testing import FakeCluster, yoda_config

PERM = [3, 0, 6, 1, 7, 2, 5, 4]          # HIP ordinal of amd-smi index i


class FakeProber:
    """HIP probes of a node whose HIP order is ``hip_order``; ``bad_hip`` fail the pattern
    check; ``bus`` maps HIP ordinal → PCI address."""

    def __init__(self, backend: FakeBackend, bad_hip=(), bw: float = 6100.0) -> None:
        self.be, self.bad, self.bw = backend, set(bad_hip), bw
        self.calls: list[tuple] = []

    def count(self) -> int:
        return self.be.gpus

    def bus_id(self, d: int) -> str:
        return self.be._bdf(self.be.hip_order.index(d)).upper()

    def bandwidth_gbps(self, d: int, nbytes: int) -> float:
        self.calls.append(("bw", d, nbytes))
        return self.bw + d

    def pattern_errors(self, d: int, nbytes: int) -> int:
        self.calls.append(("pat", d, nbytes))
        return 17 if d in self.bad else 0


def test_hip_to_index_uses_hip_id_then_bus_id():
    be = FakeBackend(8, hip_order=PERM)
    s = be.sample()
    m = hip_to_index(s, 8)
    assert all(PERM[m[d]] == d for d in range(8))
    # without hipId (old driver): PCI bus ids join the two enumerations
    for x in s:
        x["hipId"] = -1
    prober = FakeProber(be)
    m2 = hip_to_index(s, 8, prober.bus_id)
    assert m2 == m
    # CPX: 16 logical GPUs, 2 per physical; function numbers keep BDFs unique
    cpx = FakeBackend(16, partitions_per_gpu=2, hip_order=list(reversed(range(16))))
    sc = cpx.sample()
    for x in sc:
        x["hipId"] = -1
    m3 = hip_to_index(sc, 16, FakeProber(cpx).bus_id)
    assert all(cpx.hip_order[m3[d]] == d for d in range(16))
    # ambiguous BDFs (partitions sharing one address, no hipId): left unmapped, never guessed
    for x in sc:
        x["bdf"] = x["bdf"].rsplit(".", 1)[0] + ".0"
    assert hip_to_index(sc, 16, FakeProber(cpx).bus_id) == {}


def test_scv_carries_identity_and_real_occupancy():
    be = FakeBackend(8, hip_order=PERM, node="n1")
    be.tenants[2] = (3, 128)                      # 3 processes holding 128 of 256 CUs
    scv = samples_to_scv("n1", be.sample())
    rt = Scv.from_json(scv.to_json())
    for i, c in enumerate(rt.status.card_list):
        assert c.hip_id == PERM[i] and c.uuid and c.hip_uuid.startswith("GPU-") and c.processes >= 0
    c2 = rt.status.card_list[2]
    assert c2.occupancy_source == "process-cus" and c2.cu_occupancy == 50.0 and c2.processes == 3
    # producers without a process list fall back to the GFX-activity proxy
    s = be.sample()
    for x in s:
        x["processes"] = -1
        x["gfxActivity"] = 40
    c = samples_to_scv("n1", s).status.card_list[0]
    assert c.occupancy_source == "gfx-activity" and c.cu_occupancy == 40.0


def test_probe_attribution_follows_hip_order_and_n_strike_health():
    be = FakeBackend(8, hip_order=PERM, node="n1")
    prober = FakeProber(be, bad_hip={2})
    agent = SnifferAgent(None, "n1", be, probe=True, prober=prober, fail_threshold=3, probe_bytes=1 << 30)
    bad_index = PERM.index(2)
    for k in range(3):
        res = agent.run_probes()
        health = {c.id: c.health for c in agent.build().status.card_list}
        if k < 2:
            assert all(h == "Healthy" for h in health.values()), (k, health)   # one bad check ≠ Unhealthy
    assert health[bad_index] == "Unhealthy" and sum(h != "Healthy" for h in health.values()) == 1
    # measured bandwidth landed on the card of the HIP ordinal that measured it
    bw = {c.id: c.bandwidth for c in agent.build().status.card_list}
    assert all(bw[i] == round(6100.0 + PERM[i]) for i in range(8))
    assert res[bad_index]["hip"] == 2 and res[bad_index]["fail_streak"] == 3
    # the fault clears: one clean check brings the card back
    prober.bad.clear()
    agent.run_probes()
    assert all(c.health == "Healthy" for c in agent.build().status.card_list)


def test_probe_skips_busy_gpus_and_sizes_from_free_hbm():
    be = FakeBackend(8, node="n1")
    be.tenants[1] = (1, 32)                       # a tenant process: never probed
    be.state[4].used_mb = 280_000                 # little free HBM left
    be.state[5].used_mb = 3000                    # over busy_vram_mb without a process
    prober = FakeProber(be)
    agent = SnifferAgent(None, "n1", be, probe=True, prober=prober, probe_bytes=1 << 30, busy_vram_mb=2048)
    res = agent.run_probes()
    probed = {d for kind, d, _ in prober.calls}
    assert 1 not in probed and "busy" in res[1]["skipped"]
    assert 5 not in probed and "busy" in res[5]["skipped"]
    assert 4 not in probed or all(n <= (0.25 * (be.spec.hbm_mb - 280_000)) * (1 << 20)
                                  for k, d, n in prober.calls if d == 4)
    assert all(n <= 1 << 30 for _, _, n in prober.calls)
    # a GPU that goes idle is probed on the next round
    be.tenants.pop(1)
    agent.run_probes()
    assert any(d == 1 for _, d, _ in prober.calls)


def test_change_driven_publish_and_heartbeat():
    now = [1000.0]
    srv = FakeApiServer()
    be = FakeBackend(8, node="n1")
    agent = SnifferAgent(InProcessClient(srv), "n1", be, interval=1.0, heartbeat=10.0, free_delta_mb=1024,
                         clock=lambda: now[0])

    async def go():
        await agent.publish_once(force=False)              # first: always
        for _ in range(5):                                  # idle node: nothing to write
            now[0] += 1
            await agent.publish_once(force=False)
        writes_idle = srv.calls["update"]
        be.state[0].used_mb += 512                          # below the delta: still quiet
        now[0] += 1
        await agent.publish_once(force=False)
        be.state[0].used_mb += 1024                         # meaningful change
        now[0] += 1
        await agent.publish_once(force=False)
        changed = srv.calls["update"]
        now[0] += 11                                        # heartbeat
        await agent.publish_once(force=False)
        be.state[3].ecc_uncorrectable = 1                   # health flips immediately
        now[0] += 1
        await agent.publish_once(force=False)
        return writes_idle, changed, srv.calls["update"], srv.calls["get"] if "get" in srv.calls else 0
    idle, changed, total, gets = asyncio.run(go())
    assert idle == 1 and changed == 2 and total == 4
    assert agent.skipped == 6 and agent.published == 4
    obj = srv.get("scvs", "n1")
    assert obj["spec"]["updateInterval"] == 10_000          # staleness follows the heartbeat
    assert Scv.from_json(obj).status.card_list[3].health == "Unhealthy"


def test_binding_pins_by_rocr_uuid_with_permuted_hip_order():
    """A 2-GPU pod on a node whose HIP order is a permutation of BDF order (and one on a
    CPX node): the Binding's visible-devices annotation names exactly the assigned cards'
    ROCr UUIDs, whatever their ordinals."""
    async def go():
        c = FakeCluster(yoda_config())
        for name, be in (("perm", FakeBackend(8, hip_order=PERM, node="perm")),
                         ("cpx", FakeBackend(16, partitions_per_gpu=2, hip_order=list(reversed(range(16))),
                                             node="cpx"))):
            c.server.create("nodes", make_node(name))
            s = samples_to_scv(name, be.sample(), interval_ms=600_000)
            c.server.create("scvs", s.to_json())
        await c.start()
        c.add_pod("a", {"scv/number": "2", "scv/memory": "1000"}, nodeSelector={"kubernetes.io/hostname": "perm"})
        c.add_pod("b", {"scv/number": "4", "scv/memory": "1000"}, nodeSelector={"kubernetes.io/hostname": "cpx"})
        assert await c.wait_bound(2)
        out = {}
        for p in ("a", "b"):
            pod = c.pod(p)
            scv = Scv.from_json(c.scv_obj(pod["spec"]["nodeName"]))
            ann = pod["metadata"]["annotations"]
            cards = [int(x) for x in ann["scv.amd.com/gpus"].split(",")]
            out[p] = (ann["scv.amd.com/visible-devices"].split(","),
                      [scv.status.card_list[k].hip_uuid for k in cards],
                      ann["scv.amd.com/gpu-uuids"].split(","), [scv.status.card_list[k].uuid for k in cards])
        await c.stop()
        return out
    out = asyncio.run(go())
    for p, (vis, want, uuids, want_u) in out.items():
        assert vis == want and uuids == want_u and all(v.startswith("GPU-") for v in vis), p
    assert len(out["b"][0]) == 4
