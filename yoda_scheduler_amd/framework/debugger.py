"""Cache debugger (upstream ``pkg/scheduler/internal/cache/debugger``): on ``SIGUSR2`` the
scheduler compares its cache with the informers' view of the cluster and dumps the cache
and the scheduling queue to the log; ``/debug/cache`` serves the same report as JSON.

What is compared (the drift a long-running scheduler must not accumulate):

* nodes — informer store vs the scheduler cache vs the native engine's node table;
* bound pods — informer pods with ``spec.nodeName`` (not terminal) vs the cache's
  non-assumed pods, and each cached pod's reservation in the engine's HBM ledger;
* pending pods — informer pods this scheduler is responsible for vs the queue plus the
  assumed / binding pods.
"""
from __future__ import annotations

import logging
import signal

log = logging.getLogger("yoda.debugger")


class CacheDebugger:
    def __init__(self, sched) -> None:
        self.s = sched

    def _store(self, res: str) -> dict:
        inf = self.s.informers.get(res)
        return inf.store if inf is not None else {}

    def compare(self) -> dict:
        s = self.s
        inf_nodes = {o["metadata"]["name"] for o in self._store("nodes").values()}
        cache_nodes = set(s.cache.nodes)
        eng_nodes = {n for n in cache_nodes if s.engine.node_index(n) >= 0}
        bound, pending = {}, set()
        for o in self._store("pods").values():
            uid = (o.get("metadata") or {}).get("uid")
            if s._terminal(o):
                continue
            if s._assigned(o):
                bound[uid] = (o.get("spec") or {}).get("nodeName")
            elif s._responsible(o):
                pending.add(uid)
        cached = {uid: ps for uid, ps in s.cache.pods.items() if not ps.assumed}
        assumed = {uid for uid, ps in s.cache.pods.items() if ps.assumed}
        queued = set(s.queue._pods) | {uid for fw in s.frameworks.values() for uid in fw.waiting}
        wrong_node = sorted(uid for uid, node in bound.items() if uid in cached and cached[uid].node != node)
        no_ledger = sorted(uid for uid, ps in s.cache.pods.items() if not s.engine.has_pod(ps.info.num_id))
        return {
            "nodes": {"missed": sorted(inf_nodes - cache_nodes), "redundant": sorted(cache_nodes - inf_nodes),
                      "not_in_engine": sorted(cache_nodes - eng_nodes)},
            "pods": {"missed": sorted(set(bound) - set(cached) - assumed),
                     "redundant": sorted(set(cached) - set(bound)), "wrong_node": wrong_node,
                     "no_ledger_entry": no_ledger},
            "pending": {"missed": sorted(pending - queued - assumed),
                        "redundant": sorted(queued - pending - assumed)},
        }

    def dump(self) -> dict:
        s = self.s
        nodes = {}
        for name in s.cache.nodes:
            uids = s.cache.node_pods.get(name, ())
            nodes[name] = {"pods": sorted(s.cache.pods[u].info.key for u in uids if u in s.cache.pods),
                           "gpus": s.cache.node_gpu_state(name), "stale": bool(s.cache._stale.get(name))}
        q = s.queue
        return {"nodes": nodes,
                "queue": {"active": sorted(q._pods[u].key for u in q._active_entries if u in q._pods),
                          "backoff": sorted(p.key for p in q._backoff_pods.values()),
                          "unschedulable": sorted(p.key for p, _t in q._unsched.values())},
                "nominations": {uid: node for uid, (node, _i, _t) in s.nominations.items()}}

    def report(self) -> dict:
        return {"comparison": self.compare(), "dump": self.dump()}

    def drift(self) -> dict:
        """Only the non-empty differences of :meth:`compare`."""
        out = {}
        for k, v in self.compare().items():
            d = {kk: vv for kk, vv in v.items() if vv}
            if d:
                out[k] = d
        return out

    def log_report(self) -> None:
        drift = self.drift()
        if drift:
            log.warning("cache comparer: drift %s", drift)
        else:
            log.info("cache comparer: cache matches the informers")
        d = self.dump()
        for name, n in d["nodes"].items():
            log.info("cache dump: node %s pods=%d gpus(reserved,free)=%s stale=%s", name, len(n["pods"]),
                     [(g["reserved"], g["free"]) for g in n["gpus"]], n["stale"])
        log.info("cache dump: queue %s", {k: len(v) for k, v in d["queue"].items()})

    def install(self, loop) -> bool:
        try:
            loop.add_signal_handler(signal.SIGUSR2, self.log_report)
            return True
        except (NotImplementedError, RuntimeError, ValueError):
            return False
