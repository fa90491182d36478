"""Coscheduling (gang scheduling of pod groups) — all-or-nothing placement of a
multi-pod job, e.g. an 8-node × 8-MI355X data-parallel training run whose ranks are
useless unless all of them start.

API (the sig-scheduling lightweight coscheduling labels): pods carry
``pod-group.scheduling.sigs.k8s.io: <group>`` and
``pod-group.scheduling.sigs.k8s.io/min-available: "<n>"``.

* PreFilter: a member is unschedulable (unresolvable) while fewer than ``min-available``
  members of its group exist at all;
* Permit: each placed member is assumed and held (WAIT) until ``min-available`` members of
  the group are assumed or bound — then every waiting member is allowed and they bind
  together; ``permitWaitingTimeSeconds`` (default 60) bounds the wait;
* Unreserve: when one member is rejected or times out, every waiting member of the group is
  rejected too, releasing their GPUs so the group retries as a whole.

Not part of the upstream default profile: enable it in ``plugins.preFilter/permit/reserve``.
Pods without the group label are unaffected (and stay on the native path).
"""
from __future__ import annotations

from ..framework.interfaces import (Code, CycleState, PermitPlugin, PreFilterPlugin, ReservePlugin, Status)
from ..models.pod import LABEL_POD_GROUP, LABEL_POD_GROUP_MIN, PF_POD_GROUP
from ..utils.gonum import atoi_or_zero


def _group(pod):
    g = pod.labels.get(LABEL_POD_GROUP)
    if not g:
        return None
    return pod.namespace, g, max(1, atoi_or_zero(pod.labels.get(LABEL_POD_GROUP_MIN, "1")))


class Coscheduling(PreFilterPlugin, PermitPlugin, ReservePlugin):
    name = "Coscheduling"
    pod_flags = PF_POD_GROUP
    reads_flags = PF_POD_GROUP  # other pods' features this plugin reads (needs_lane_mirror)

    def __init__(self, args=None, handle=None) -> None:
        super().__init__(args, handle)
        self.timeout = float(self.args.get("permitWaitingTimeSeconds", 60))

    def is_noop_for(self, pod) -> bool:
        return LABEL_POD_GROUP not in pod.labels

    def _members_total(self, ns: str, group: str) -> int:
        n = 0
        for o in self.handle.lister("pods").values():
            m = o.get("metadata") or {}
            if m.get("namespace", "default") == ns and (m.get("labels") or {}).get(LABEL_POD_GROUP) == group and \
                    (o.get("status") or {}).get("phase") not in ("Succeeded", "Failed") and not m.get("deletionTimestamp"):
                n += 1
        return n

    def _members_placed(self, ns: str, group: str) -> int:
        return sum(1 for ps in self.handle.cache.pods.values()
                   if ps.info.namespace == ns and ps.info.labels.get(LABEL_POD_GROUP) == group)

    def pre_filter(self, state: CycleState, pod) -> Status:
        g = _group(pod)
        if g is None:
            return Status.ok()
        ns, name, need = g
        have = self._members_total(ns, name)
        if have < need:
            return Status(Code.UNSCHEDULABLE_AND_UNRESOLVABLE,
                          [f"pod group {name}: {have} member(s) exist, min-available is {need}"], self.name)
        return Status.ok()

    def permit(self, state: CycleState, pod, node_name: str) -> tuple[Status, float]:
        g = _group(pod)
        if g is None:
            return Status.ok(), 0.0
        ns, name, need = g
        if self._members_placed(ns, name) >= need:      # this pod is already assumed
            for wp in self.handle.iterate_waiting_pods():
                wg = _group(wp.pod)
                if wg is not None and wg[:2] == (ns, name):
                    wp.allow(self.name)
            return Status.ok(), 0.0
        return Status(Code.WAIT, [f"waiting for pod group {name}"], self.name), self.timeout

    def reserve(self, state: CycleState, pod, node_name: str) -> Status:
        return Status.ok()

    def unreserve(self, state: CycleState, pod, node_name: str) -> None:
        g = _group(pod)
        if g is None:
            return
        for wp in self.handle.iterate_waiting_pods():
            wg = _group(wp.pod)
            if wg is not None and wg[:2] == g[:2] and wp.pod.uid != pod.uid:
                wp.reject(self.name, f"pod group {g[1]}: a member was rejected")
