"""`bench.py --mix-preempt N`: a full cluster — every GPU held by a bound
low-priority pod — and a burst of priority-100 pods that each need most of a card. Every
preemptor fails the filters, DefaultPreemption (native search) nominates a node and deletes one
victim through the API, and the pod binds on its retry after upstream's initial backoff."""
import asyncio


def test_preemption_burst_on_a_full_cluster_binds_every_preemptor():
    from yoda_scheduler_amd.bench.harness import Shard
    from yoda_scheduler_amd.bench.workloads import make_workload
    from yoda_scheduler_amd.plugins.defaults import DefaultPreemption

    w = make_workload(5, seed=0, mix_preempt=8)
    assert w.wait_bound and len(w.pods) == 8
    fillers = [o for res, o in w.objects if res == "pods"]
    assert len(fillers) == 4 * 8 and all(o["spec"]["nodeName"] for o in fillers)
    before = dict(DefaultPreemption.stats)

    async def run():
        sh = Shard(w, device="off")
        await sh.start()
        try:
            r = await sh.burst("p", timeout=30)
            left = [k for k in sh.server._objs["pods"] if k.startswith("default/filler-")]
            nodes = set(sh.server.bind_node.values())
            return r, left, nodes
        finally:
            await sh.stop()

    r, left, nodes = asyncio.run(run())
    assert r.bound == 8, r
    assert len(left) == 32 - 8                      # one victim per preemptor
    assert nodes <= {f"node-{i}" for i in range(4)}
    S = DefaultPreemption.stats
    assert S["nominated"] - before["nominated"] == 8
    assert S["victims"] - before["victims"] == 8
    assert 0.9 < max(r.latencies_s) < 10            # bound on the retry after the 1 s backoff
