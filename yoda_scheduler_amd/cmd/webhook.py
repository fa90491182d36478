"""``yoda-webhook`` — admission webhook for the scv label API (see ``webhook/``)."""
from __future__ import annotations

import argparse
import asyncio
import signal
import ssl
import sys
from typing import Optional, Sequence

from ..utils import klog
from ..webhook.admission import AdmissionPolicy
from ..webhook.server import WebhookServer


def main(argv: Optional[Sequence[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="yoda-webhook", description=__doc__)
    p.add_argument("--bind-address", default="0.0.0.0")
    p.add_argument("--port", type=int, default=9443)
    p.add_argument("--tls-cert-file", default="")
    p.add_argument("--tls-private-key-file", default="")
    p.add_argument("--scheduler-name", default="yoda-scheduler", help="profile pods with scv labels are sent to")
    p.add_argument("--no-mutate-scheduler-name", action="store_true")
    p.add_argument("--no-inject-visible-devices", action="store_true",
                   help="do not add HIP/ROCR_VISIBLE_DEVICES (downward API of scv.amd.com/gpus) to yoda pods")
    p.add_argument("--max-gpus-per-pod", type=int, default=64)
    p.add_argument("--max-memory-mb", type=int, default=288 * 1024)
    p.add_argument("--v", type=int, default=0)
    a = p.parse_args(argv)
    klog.setup(a.v)
    ctx = None
    if a.tls_cert_file:
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(a.tls_cert_file, a.tls_private_key_file or None)
    pol = AdmissionPolicy(a.max_gpus_per_pod, a.max_memory_mb, a.scheduler_name, not a.no_mutate_scheduler_name,
                          not a.no_inject_visible_devices)

    async def run() -> int:
        srv = WebhookServer(a.bind_address, a.port, pol, ctx)
        port = await srv.start()
        print(f"yoda-webhook serving on {a.bind_address}:{port} ({'https' if ctx else 'http'})", flush=True)
        stop = asyncio.Event()
        loop = asyncio.get_event_loop()
        for sig in (signal.SIGINT, signal.SIGTERM):
            try:
                loop.add_signal_handler(sig, stop.set)
            except (NotImplementedError, RuntimeError):
                pass
        await stop.wait()
        await srv.stop()
        return 0

    return asyncio.run(run())


if __name__ == "__main__":
    sys.exit(main())
