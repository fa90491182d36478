"""Multi-process paths on CPU (gloo, world_size 2): the bench.py weak-scaling contract
(one scheduler shard per rank, max-over-ranks timing, aggregate value) and the all-reduce
probe used to validate gang placements."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(args, nproc=2, timeout=240):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), *args]
    return subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, env=env, timeout=timeout)


def test_bench_two_ranks_weak_scaling_contract():
    r = _torchrun(["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # exactly one JSON line, from rank 0
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["pods_bound"] == 2 * 2 * 1000 and d["config"]["global_batch"] == 2000
    assert abs(d["value"] - d["pods_bound"] / (d["ms_per_step"] * d["steps"] / 1000.0)) / d["value"] < 0.01
    assert d["higher_is_better"] is True and d["p99_latency_ms"] > 0


def test_allreduce_probe_gloo():
    r = _torchrun(["-m", "yoda_scheduler_amd.parallel.rccl_probe", "--sizes", "64K,1M", "--iters", "3"])
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [x["bytes"] for x in rows] == [65536, 1 << 20]
    assert all(x["world"] == 2 and x["busbw_gbps"] > 0 for x in rows)


def test_gang_validation_harness_picks_low_load_set_gloo():
    """parallel/validate_gangs under torch.distributed.run (4 gloo ranks, FakeBackend with
    an injected hot xGMI link): the engine's placement of a 2-GPU pod avoids the loaded
    pair, agrees with the Python reference objective, the worst-ranked set is the loaded
    pair, and rank 0 emits one JSON line with both sets' all-reduce bandwidth."""
    r = _torchrun(["-m", "yoda_scheduler_amd.parallel.validate_gangs", "--fake", "--k", "2",
                   "--fake-load", "0-1:0.9", "--sizes", "64K", "--iters", "2"], nproc=4)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["k"] == 2 and d["world"] == 4 and d["engine_matches_spec"] is True
    assert d["best"] == [2, 3] and d["worst"] == [0, 1]
    assert d["best_objective"] < d["worst_objective"] and d["best_link_bad"] < d["worst_link_bad"]
    assert d["sampled_link_load"]["0-1"] == 0.9
    assert d["busbw_best"][0]["world"] == 2 and d["busbw_worst"][0]["busbw_gbps"] > 0
    assert d["busbw_ratio_best_over_worst"] > 0 and "no xGMI" in d["backend"]


def test_bench_eight_ranks_each_rank_owns_its_gpu_gloo():
    """8 gloo ranks, each on a fake amd-smi node of 8 distinct cards (HIP order reversed
    against amd-smi order): rank r's scheduler config pins the device scorer to GPU r, its
    telemetry template comes from the card whose HIP ordinal is r (a distinct BDF per rank),
    and the one JSON line aggregates 8 × the per-rank pods."""
    env_extra = {"YODA_BENCH_FAKE_SMI": "8"}
    old = {k: os.environ.get(k) for k in env_extra}
    os.environ.update(env_extra)
    try:
        r = _torchrun(["bench.py", "--gpus", "8", "--steps", "1", "--warmup", "0", "--config", "2",
                       "--alt", "none"], nproc=8, timeout=600)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["pods_bound"] == 8 * 100 and d["config"]["global_batch"] == 800
    ranks = sorted(d["ranks"], key=lambda x: x["rank"])
    assert [x["rank"] for x in ranks] == list(range(8))
    for x in ranks:
        assert x["gpu_index"] == x["local_rank"] == x["rank"]
        assert x["device_scorer_device"] == x["rank"]        # yodaRuntime.deviceScorer.device
        assert x["telemetry_hip_id"] == x["rank"]            # its own card, by HIP ordinal
        assert x["pods_bound"] == 100
    assert len({x["telemetry_bdf"] for x in ranks}) == 8     # eight distinct cards
    assert sum(x["pods_bound"] for x in ranks) == d["pods_bound"]
