"""GPU: RCCL (torch.distributed "nccl" on ROCm) all-reduce probe and the xGMI peer-write
probe (gang-placement validation workloads)."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_allreduce_probe_single_rank(require_gpu):
    import torch
    import torch.distributed as dist
    from yoda_scheduler_amd.parallel.rccl_probe import allreduce_bandwidth
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", world_size=1, rank=0,
                            device_id=torch.device("cuda", 0))
    try:
        res = allreduce_bandwidth([1 << 20, 64 << 20], iters=5, warmup=2)
    finally:
        dist.destroy_process_group()
    assert [r["bytes"] for r in res] == [1 << 20, 64 << 20]
    assert all(r["algbw_gbps"] > 0 for r in res)


def test_xgmi_peer_write_probe(require_gpu):
    from yoda_scheduler_amd.ops import hip
    n = hip.device_count()
    if n >= 2:
        r = hip.peer_write_bandwidth(0, 1, 256 << 20, 5)
        assert r["supported"] and r["gbps"] > 20, r
    else:
        r = hip.peer_write_bandwidth(0, 0, 1 << 20, 1)   # single-GPU box: no peer, no error
        assert r["supported"] is False and r["gbps"] == 0.0
