"""core.BatchWorker: engine batches on a native thread that never takes the GIL, results
collected by the event loop through an eventfd (framework/scheduler.py
``_submit_engine_batch``)."""
import asyncio
import select

import pytest

import random

from yoda_scheduler_amd.ops import device_scorer as ds
from yoda_scheduler_amd.ops.native import core


def _engine(nodes=24):
    eng = core().Engine(False, 1)
    ds.synthetic_cluster(eng, nodes, seed=3, busy=0.3)
    return eng


def _pods(eng, n, tag):
    rng = random.Random(7)
    ids, reqs = [], []
    for i in range(n):
        pi, req = ds.random_request(eng, rng, f"{tag}{i}")
        ids.append(pi.num_id)
        reqs.append(req)
    return ids, reqs


def test_batch_worker_matches_inline_batches_and_signals_fd():
    a, b = _engine(), _engine()
    ids, reqs = _pods(a, 40, "p")
    inline = b.schedule_batch(*_pods(b, 40, "p"))
    assert sum(r[0] >= 0 for r in inline) >= 20
    w = core().BatchWorker(a)
    try:
        j1 = w.submit(ids[:25], reqs[:25])
        j2 = w.submit(ids[25:], reqs[25:])
        got = {}
        while len(got) < 2:
            r, _, _ = select.select([w.fileno()], [], [], 10.0)
            assert r, "no completion signalled"
            for jid, res, err, t0, t1 in w.collect():
                assert err is None and t1 >= t0
                got[jid] = res
        assert [r[0] for r in got[j1] + got[j2]] == [r[0] for r in inline]
        assert a.ledger_size == b.ledger_size > 0
        assert w.pending == 0
    finally:
        w.close()


def test_batch_worker_rejects_mismatched_batch_and_closes_cleanly():
    eng = _engine()
    ids, reqs = _pods(eng, 3, "q")
    w = core().BatchWorker(eng)
    with pytest.raises(ValueError):
        w.submit(ids, reqs[:2])
    w.close()
    with pytest.raises(RuntimeError):
        w.submit(ids, reqs)
    w.close()   # idempotent


def test_batch_worker_from_event_loop():
    eng = _engine()
    ids, reqs = _pods(eng, 10, "r")

    async def go():
        loop = asyncio.get_event_loop()
        w = core().BatchWorker(eng)
        fut = loop.create_future()

        def on_ready():
            for jid, res, err, _t0, _t1 in w.collect():
                fut.set_result(res)
        loop.add_reader(w.fileno(), on_ready)
        w.submit(ids, reqs)
        res = await asyncio.wait_for(fut, 10.0)
        loop.remove_reader(w.fileno())
        w.close()
        return res
    res = asyncio.run(go())
    assert len(res) == 10 and any(r[0] >= 0 for r in res)
