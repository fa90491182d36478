"""``yoda-sniffer`` — the per-node amd-smi telemetry agent (DaemonSet), replacing the
reference's external NVML-based SCV sniffer (``readme.md:9-10,15``).

Samples every GPU of the node with the C++ amd-smi collector every ``--interval`` seconds
and publishes the node's ``Scv`` status when something the scheduler acts on changed
(or every ``--heartbeat`` seconds). With ``--probe`` the gfx950 HBM probes run on idle
GPUs every ``--probe-interval`` seconds (measured bandwidth → ``Card.Bandwidth``,
``--probe-fail-threshold`` consecutive pattern failures → ``Card.Health`` Unhealthy).
``--print`` samples once and prints the Scv JSON (no apiserver needed).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import sys
from typing import Optional, Sequence

from ..utils import klog


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="yoda-sniffer", description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--node", default=os.environ.get("NODE_NAME", socket.gethostname()))
    p.add_argument("--kubeconfig", default="")
    p.add_argument("--master", default="")
    p.add_argument("--interval", type=float, default=1.0, help="sample period (s)")
    p.add_argument("--heartbeat", type=float, default=10.0,
                   help="publish at least this often (s); also the Scv updateInterval staleness is based on")
    p.add_argument("--free-delta-mb", type=int, default=1024, help="publish when a GPU's free HBM moved this much")
    p.add_argument("--load-delta", type=float, default=0.05, help="publish when an xGMI link load moved this much")
    p.add_argument("--backend", choices=["amd-smi", "fake"], default="amd-smi")
    p.add_argument("--fake-gpus", type=int, default=8)
    p.add_argument("--probe", action="store_true", help="run the HIP HBM bandwidth/pattern probes on idle GPUs")
    p.add_argument("--probe-bytes", type=int, default=1 << 30, help="upper bound (also ≤ 25%% of free HBM)")
    p.add_argument("--probe-interval", type=float, default=600.0, help="re-probe idle GPUs every N seconds")
    p.add_argument("--probe-fail-threshold", type=int, default=3,
                   help="consecutive failed pattern checks before a GPU is marked Unhealthy")
    p.add_argument("--print", dest="print_only", action="store_true", help="sample once, print the Scv, exit")
    p.add_argument("--count", type=int, default=0, help="publish N samples then exit (0 = forever)")
    p.add_argument("--v", type=int, default=0)
    return p


def make_backend(name: str, gpus: int = 8):
    from ..sniffer.collector import AmdSmiBackend, FakeBackend
    return FakeBackend(gpus) if name == "fake" else AmdSmiBackend()


def main(argv: Optional[Sequence[str]] = None) -> int:
    a = build_parser().parse_args(argv)
    klog.setup(a.v)
    from ..sniffer.publisher import SnifferAgent
    backend = make_backend(a.backend, a.fake_gpus)
    if a.print_only:
        agent = SnifferAgent(None, a.node, backend, a.interval, probe=a.probe, probe_bytes=a.probe_bytes,
                             heartbeat=a.heartbeat, fail_threshold=a.probe_fail_threshold)
        if a.probe:
            agent.run_probes()
        print(json.dumps(agent.build().to_json(), indent=2))
        return 0
    from ..kube.client import KubeClient, KubeConfig

    async def run() -> None:
        client = KubeClient(KubeConfig.load(a.kubeconfig, a.master))
        agent = SnifferAgent(client, a.node, backend, a.interval, probe=a.probe, probe_bytes=a.probe_bytes,
                             heartbeat=a.heartbeat, free_delta_mb=a.free_delta_mb, load_delta=a.load_delta,
                             probe_interval=a.probe_interval, fail_threshold=a.probe_fail_threshold)
        try:
            await agent.run(count=a.count or None)
        finally:
            await client.close()

    asyncio.run(run())
    return 0


if __name__ == "__main__":
    sys.exit(main())
