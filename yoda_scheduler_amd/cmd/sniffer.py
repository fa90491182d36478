"""``yoda-sniffer`` — the per-node amd-smi telemetry agent (DaemonSet), replacing the
reference's external NVML-based SCV sniffer (``readme.md:9-10,15``).

Samples every GPU of the node with the C++ amd-smi collector, optionally runs the gfx950
HBM probes once at start (measured bandwidth → ``Card.Bandwidth``, pattern errors →
``Card.Health``) and publishes the node's ``Scv`` status every ``--interval`` seconds.
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
    p.add_argument("--interval", type=float, default=1.0)
    p.add_argument("--backend", choices=["amd-smi", "fake"], default="amd-smi")
    p.add_argument("--fake-gpus", type=int, default=8)
    p.add_argument("--probe", action="store_true", help="run the HIP HBM bandwidth/pattern probes at start")
    p.add_argument("--probe-bytes", type=int, default=1 << 30)
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
        agent = SnifferAgent(None, a.node, backend, a.interval, probe=a.probe, probe_bytes=a.probe_bytes)
        if a.probe:
            agent.run_probes()
        print(json.dumps(agent.build().to_json(), indent=2))
        return 0
    from ..kube.client import KubeClient, KubeConfig

    async def run() -> None:
        client = KubeClient(KubeConfig.load(a.kubeconfig, a.master))
        agent = SnifferAgent(client, a.node, backend, a.interval, probe=a.probe, probe_bytes=a.probe_bytes)
        try:
            await agent.run(count=a.count or None)
        finally:
            await client.close()

    asyncio.run(run())
    return 0


if __name__ == "__main__":
    sys.exit(main())
