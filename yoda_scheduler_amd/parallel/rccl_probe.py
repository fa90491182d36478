"""RCCL all-reduce probe: measures the collective bandwidth a GPU set actually achieves
(SURVEY §2.5/§7 phase 6 — validation workload for gang placements, not scheduler hot path).

Launch one process per GPU of the set (``torch.distributed.run``); backend ``nccl`` is RCCL
on ROCm and runs over xGMI between the node's MI355X GPUs. Reports, per message size,
algorithm bandwidth (bytes / time) and bus bandwidth (× 2(n−1)/n for a ring all-reduce),
which on an MI355X full mesh is bounded by the per-link rate (~153.6 GB/s) times the links
RCCL's channels use — the quantity the gang objective's link-quality term models.

    python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 \
        -m yoda_scheduler_amd.parallel.rccl_probe --sizes 1M,64M,512M
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import Optional, Sequence


def parse_size(s: str) -> int:
    s = s.strip().upper()
    mul = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(s[-1:], 1)
    return int(float(s[:-1]) * mul) if s[-1:] in "KMG" else int(s)


def allreduce_bandwidth(sizes: Sequence[int], iters: int = 20, warmup: int = 5, dtype: str = "bfloat16",
                        device: Optional[str] = None, group=None) -> list[dict]:
    """Run inside an initialised process group (every rank of ``group``, default the whole
    world); returns one dict per size (rank-local timing, max over the group's ranks)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = torch.device(device) if device else (torch.device("cuda", torch.cuda.current_device())
                                                if torch.cuda.is_available() else torch.device("cpu"))
    dt = getattr(torch, dtype)
    esz = torch.tensor([], dtype=dt).element_size()
    out = []
    for nbytes in sizes:
        n = max(1, nbytes // esz)
        x = torch.ones(n, dtype=dt, device=dev)
        for _ in range(warmup):
            dist.all_reduce(x, group=group)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x, group=group)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        el = time.perf_counter() - t0
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        el = float(t.item())
        algbw = n * esz * iters / el / 1e9
        out.append({"bytes": n * esz, "world": world, "us_per_iter": round(el / iters * 1e6, 2),
                    "algbw_gbps": round(algbw, 3), "busbw_gbps": round(algbw * 2 * (world - 1) / max(world, 1), 3)})
    return out


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1M,16M,256M")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="bfloat16")
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", 0))
    cuda = torch.cuda.is_available()
    if cuda:
        torch.cuda.set_device(local % torch.cuda.device_count())
    if cuda:
        dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    else:
        dist.init_process_group("gloo")
    res = allreduce_bandwidth([parse_size(s) for s in a.sizes.split(",")], a.iters,
                              dtype=a.dtype if cuda else "float32")
    if dist.get_rank() == 0:
        for r in res:
            print(json.dumps({"probe": "rccl_allreduce" if cuda else "gloo_allreduce", **r}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
