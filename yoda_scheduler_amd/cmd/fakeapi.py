"""``yoda-fake-apiserver`` — serve the in-process fake apiserver over HTTP (dev/testing),
optionally pre-populated with synthetic 8×MI355X nodes and their Scv objects."""
from __future__ import annotations

import argparse
import asyncio
import sys
import time
from typing import Optional, Sequence


def main(argv: Optional[Sequence[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="yoda-fake-apiserver")
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--port", type=int, default=8001)
    p.add_argument("--nodes", type=int, default=0)
    p.add_argument("--gpus", type=int, default=8)
    p.add_argument("--bench-config", type=int, default=0, help="populate BASELINE config N and serve /debug/bench/*")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--template", default="", help="JSON card template (real amd-smi fields) for MI355X nodes")
    p.add_argument("--port-file", default="", help="write the bound port here once listening")
    a = p.parse_args(argv)
    from ..fakeapi.http import serve_forever
    from ..fakeapi.server import FakeApiServer
    from ..models.device import make_node, make_scv
    srv = FakeApiServer()
    workload = None
    if a.bench_config:
        import json

        from ..bench.workloads import make_workload, populate
        workload = make_workload(a.bench_config, seed=a.seed)
        populate(srv, workload, json.loads(a.template) if a.template else None,
                 link_load=0.2 if a.bench_config == 5 else 0.0, seed=a.seed)
    for i in range(a.nodes):
        srv.create("nodes", make_node(f"mi355x-{i}"))
        s = make_scv(f"mi355x-{i}", gpus=a.gpus, update_time=time.time())
        s.update_interval_ms = 3_600_000
        srv.create("scvs", s.to_json())
    try:
        asyncio.run(serve_forever(a.host, a.port, srv, workload=workload, port_file=a.port_file))
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
