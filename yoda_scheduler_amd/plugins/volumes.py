"""Volume plugins of the upstream default profile (the reference's profile only
lists ``yoda``, so kube-scheduler v1.20's volume Filter/Reserve/PreBind plugins stay on):

* ``VolumeRestrictions`` — in-tree disks that cannot be mounted twice on one node
  (GCE PD / AWS EBS / RBD / iSCSI conflict rules).
* ``VolumeZone`` — a bound PV's zone/region labels must match the node's.
* ``VolumeBinding`` — PVCs must exist; bound PVs' node affinity must admit the node;
  ``WaitForFirstConsumer`` claims get a matching static PV (smallest that fits) or dynamic
  provisioning on that node; Reserve assumes the choice, PreBind writes it to the
  apiserver and waits until the PV controller reports the claims bound.
* ``NodeVolumeLimits`` (CSI attach limits from ``CSINode``) and the in-tree
  ``EBSLimits`` / ``GCEPDLimits`` / ``AzureDiskLimits`` counters.

All of them are no-ops for pods without the relevant volumes (``is_noop_for``), so GPU
pods without PVCs keep the fully native scheduling cycle. A pod whose claims are all bound
is a no-op for each of them too when its bound volumes give that plugin nothing to check —
no PV node affinity (VolumeBinding), no zone labels on the PVs (VolumeZone), no attach
limit anywhere or no attachable volume of the plugin's kind (the limits plugins) — so a pod
that mounts a pre-provisioned dataset / checkpoint share takes the native cycle as well.
Each test is the plugin's own Filter / PreBind reasoning applied to the current listers,
so it can only answer "no-op" where every extension point would pass untouched. The
objects come from informers the scheduler starts only because these plugins declare
``watches``.
"""
from __future__ import annotations

import asyncio
import re
import time
from typing import Optional

from ..framework.interfaces import (Code, CycleState, FilterPlugin, PreBindPlugin, PreFilterPlugin, ReservePlugin,
                                    StateData, Status)
from ..models.pod import FIELD_NODE_NAME, PF_CLAIMS, PF_DISKS
from ..models.selectors import LabelSelector, NodeSelector
from ..utils.quantity import bytes_of

ZONE_LABELS = ("topology.kubernetes.io/zone", "topology.kubernetes.io/region",
               "failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region")
ANN_SELECTED_NODE = "volume.kubernetes.io/selected-node"
NO_PROVISIONER = "kubernetes.io/no-provisioner"
WFFC = "WaitForFirstConsumer"
_EMPTY: dict = {}

ERR_DISK_CONFLICT = "node(s) had no available disk"
ERR_ZONE_CONFLICT = "node(s) had no available volume zone"
ERR_NODE_CONFLICT = "node(s) had volume node affinity conflict"
ERR_NO_PV = "node(s) didn't find available persistent volumes to bind"
ERR_UNBOUND_IMMEDIATE = "pod has unbound immediate PersistentVolumeClaims"
ERR_MAX_VOLUMES = "node(s) exceed max volume count"


def _volumes(pod) -> list:
    return (pod.obj.get("spec") or {}).get("volumes") or []


def _claim_names(pod) -> list[str]:
    out = []
    for v in _volumes(pod):
        if "persistentVolumeClaim" in v:
            out.append((v["persistentVolumeClaim"] or {}).get("claimName", ""))
        elif "ephemeral" in v:                      # generic ephemeral volume → <pod>-<volume>
            out.append(f"{pod.name}-{v.get('name', '')}")
    return out


def _unresolvable(msg: str, plugin: str) -> Status:
    return Status(Code.UNSCHEDULABLE_AND_UNRESOLVABLE, [msg], plugin)


class _VolFacts:
    """What the volume plugins' no-op tests read of one pod, resolved in one pass:

    * ``claims`` — the claim names (PVC volumes and generic ephemeral volumes' claims);
    * ``bound`` — the PV of every claim when each claim exists, is not being deleted and
      names a PV that exists; None otherwise;
    * ``inline`` — the attachable-disk kinds among the pod's inline volumes;
    * ``pv_kinds`` — the attachable-disk kinds of the PVs its PVC volumes are bound to;
    * ``csi`` — the CSI drivers whose attach limit its PVC volumes count against (a bound
      CSI PV's driver, an unbound claim's provisioner) — NodeVolumeLimits' own rule."""
    __slots__ = ("claims", "bound", "inline", "pv_kinds", "csi")

    def __init__(self, plugin: "_VolumeBase", pod) -> None:
        vols = _volumes(pod)
        self.claims = _claim_names(pod)
        self.inline = {k for v in vols for k in _ATTACHABLE_KINDS if k in v}
        self.pv_kinds: set = set()
        self.csi: set = set()
        for v in vols:
            if "persistentVolumeClaim" not in v:
                continue
            pvc = plugin._pvc(pod.namespace, (v["persistentVolumeClaim"] or _EMPTY).get("claimName", ""))
            if pvc is None:
                continue
            spec = pvc.get("spec") or _EMPTY
            pv = plugin._pv(spec.get("volumeName", ""))
            if pv is not None:
                ps = pv.get("spec") or _EMPTY
                csi = ps.get("csi")
                if csi:
                    self.csi.add(csi.get("driver", ""))
                self.pv_kinds.update(k for k in _ATTACHABLE_KINDS if ps.get(k))
                continue
            sc = plugin._sc(spec.get("storageClassName", ""))
            if sc is not None and sc.get("provisioner", NO_PROVISIONER) != NO_PROVISIONER:
                self.csi.add(sc["provisioner"])
        self.bound = plugin._bound_claims(pod, self.claims) if self.claims else []


class _VolumeBase:
    watches = ("persistentvolumeclaims", "persistentvolumes", "storageclasses")

    def _lister(self, res: str) -> dict:
        return self.handle.lister(res)

    def _pvc(self, ns: str, name: str) -> Optional[dict]:
        return self._lister("persistentvolumeclaims").get(f"{ns}/{name}")

    def _pv(self, name: str) -> Optional[dict]:
        return self._lister("persistentvolumes").get(name) if name else None

    def _sc(self, name: str) -> Optional[dict]:
        return self._lister("storageclasses").get(name) if name else None

    def _node_labels(self, node: str) -> dict:
        n = self.handle.cache.nodes.get(node)
        return n.labels if n is not None else {}

    def _facts(self, pod) -> "_VolFacts":
        """The pod's claims resolved against the PVC / PV / StorageClass listers, once for
        every volume plugin that asks about the pod, until one of those listers changes
        (their generations move on every event; the pod's volumes are fixed)."""
        gen = getattr(self.handle, "generation", None)
        if gen is None or not hasattr(pod, "vol_memo"):
            return _VolFacts(self, pod)
        key = (gen("persistentvolumeclaims"), gen("persistentvolumes"), gen("storageclasses"))
        m = pod.vol_memo
        if m is None or m[0] != key:
            m = pod.vol_memo = (key, _VolFacts(self, pod))
        return m[1]

    def _bound_claims(self, pod, claims: list) -> Optional[list]:
        """The claims' bound PVs when every claim exists, is not being deleted and names a PV
        that exists; None otherwise (the plugin's own checks decide)."""
        out = []
        for claim in claims:
            pvc = self._pvc(pod.namespace, claim)
            if pvc is None or (pvc.get("metadata") or {}).get("deletionTimestamp"):
                return None
            pv = self._pv((pvc.get("spec") or {}).get("volumeName", ""))
            if pv is None:
                return None
            out.append(pv)
        return out

    def _node_pod_objs(self, node: str):
        cache = self.handle.cache
        for uid in cache.node_pods.get(node, ()):
            ps = cache.pods.get(uid)
            if ps is not None:
                yield ps.info.obj


# ================================================================= VolumeRestrictions
def _disk_conflict(a: dict, b: dict) -> bool:
    if "gcePersistentDisk" in a and "gcePersistentDisk" in b:
        x, y = a["gcePersistentDisk"] or {}, b["gcePersistentDisk"] or {}
        return x.get("pdName") == y.get("pdName") and not (x.get("readOnly") and y.get("readOnly"))
    if "awsElasticBlockStore" in a and "awsElasticBlockStore" in b:
        return (a["awsElasticBlockStore"] or {}).get("volumeID") == (b["awsElasticBlockStore"] or {}).get("volumeID")
    if "iscsi" in a and "iscsi" in b:
        x, y = a["iscsi"] or {}, b["iscsi"] or {}
        return x.get("iqn") == y.get("iqn") and not (x.get("readOnly") and y.get("readOnly"))
    if "rbd" in a and "rbd" in b:
        x, y = a["rbd"] or {}, b["rbd"] or {}
        share_mon = bool(set(x.get("monitors") or []) & set(y.get("monitors") or []))
        return (share_mon and x.get("pool", "rbd") == y.get("pool", "rbd") and x.get("image") == y.get("image")
                and not (x.get("readOnly") and y.get("readOnly")))
    return False


_EXCLUSIVE_KINDS = ("gcePersistentDisk", "awsElasticBlockStore", "iscsi", "rbd")


class VolumeRestrictions(_VolumeBase, FilterPlugin):
    name = "VolumeRestrictions"
    watches = ()
    pod_flags = PF_DISKS
    reads_flags = PF_DISKS  # other pods' features this plugin reads (needs_lane_mirror)

    def is_noop_for(self, pod) -> bool:
        return not any(k in v for v in _volumes(pod) for k in _EXCLUSIVE_KINDS)

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        mine = [v for v in _volumes(pod) if any(k in v for k in _EXCLUSIVE_KINDS)]
        for obj in self._node_pod_objs(node_name):
            for ev in (obj.get("spec") or {}).get("volumes") or ():
                for v in mine:
                    if _disk_conflict(v, ev):
                        return Status.unschedulable(ERR_DISK_CONFLICT, plugin=self.name)
        return Status.ok()


# ================================================================= VolumeZone
class VolumeZone(_VolumeBase, FilterPlugin):
    name = "VolumeZone"
    pod_flags = PF_CLAIMS
    claim_inert_ok = True   # the lane's claim table covers it (claim_lane): a no-op or an engine filter
    reads_flags = 0  # other pods' features this plugin reads (needs_lane_mirror)

    def is_noop_for(self, pod) -> bool:
        # no claims, or every claim bound to a PV without zone / region labels (the filter
        # then passes on every node)
        f = self._facts(pod)
        return not f.claims or f.bound is not None and not any(
            k in ((pv.get("metadata") or _EMPTY).get("labels") or _EMPTY) for pv in f.bound for k in ZONE_LABELS)

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        labels = self._node_labels(node_name)
        node_zone = {k: labels[k] for k in ZONE_LABELS if k in labels}
        if not node_zone:
            return Status.ok()          # a node without zone labels takes any volume
        for claim in _claim_names(pod):
            pvc = self._pvc(pod.namespace, claim)
            if pvc is None:
                return _unresolvable(f'persistentvolumeclaim "{claim}" not found', self.name)
            pv_name = (pvc.get("spec") or {}).get("volumeName", "")
            if not pv_name:
                scn = (pvc.get("spec") or {}).get("storageClassName", "")
                if not scn:
                    return _unresolvable("PersistentVolumeClaim had no pv name and storageClass name", self.name)
                sc = self._sc(scn)
                if sc is None:
                    return _unresolvable(f'StorageClass "{scn}" claimed by PersistentVolumeClaim "{claim}" not found',
                                         self.name)
                if sc.get("volumeBindingMode") == WFFC:
                    continue            # VolumeBinding decides where it is provisioned
                return _unresolvable("PersistentVolume had no name", self.name)
            pv = self._pv(pv_name)
            if pv is None:
                return _unresolvable(f'persistentvolume "{pv_name}" not found', self.name)
            pv_labels = (pv.get("metadata") or {}).get("labels") or {}
            for k in ZONE_LABELS:
                if k not in pv_labels:
                    continue
                allowed = set(pv_labels[k].split("__"))
                if k not in node_zone or node_zone[k] not in allowed:
                    return _unresolvable(ERR_ZONE_CONFLICT, self.name)
        return Status.ok()


# ================================================================= VolumeBinding
def _pvc_key(pvc: dict) -> str:
    m = pvc.get("metadata") or {}
    return f"{m.get('namespace') or 'default'}/{m.get('name', '')}"


def _storage(obj: dict, *path) -> int:
    cur = obj
    for p in path:
        cur = (cur or {}).get(p)
    return bytes_of(cur or "0")


def _pv_class(pv: dict) -> str:
    return (pv.get("spec") or {}).get("storageClassName", "") or ""


def _pv_node_ok(pv: dict, node: str, labels: dict) -> bool:
    req = ((pv.get("spec") or {}).get("nodeAffinity") or {}).get("required")
    return req is None or NodeSelector(req).matches(node, labels)


class _BindingState(StateData):
    def __init__(self, bound, delayed, candidates) -> None:
        self.bound = bound                  # [(pvc, pv)] already bound claims
        self.delayed = delayed              # [pvc] unbound WaitForFirstConsumer claims
        self.candidates = candidates        # pvc key → [pv] static candidates, smallest first
        self.decisions: dict[str, tuple[list, list]] = {}   # node → ([(pvc, pv name)], [pvc to provision])

    def clone(self) -> "_BindingState":
        return self


class VolumeBinding(_VolumeBase, PreFilterPlugin, FilterPlugin, ReservePlugin, PreBindPlugin):
    name = "VolumeBinding"
    KEY = "PreFilterVolumeBinding"
    pod_flags = PF_CLAIMS
    # other pods' features this plugin reads (needs_lane_mirror): none — it reads the PVC / PV /
    # StorageClass listers and its own assumed PVs, never another pod
    reads_flags = 0
    claim_inert_ok = True   # the lane's claim table covers it (claim_lane): a no-op or an engine filter

    def __init__(self, args=None, handle=None) -> None:
        super().__init__(args, handle)
        self.bind_timeout = float((args or {}).get("bindTimeoutSeconds", 600))
        self._assumed: dict[str, str] = {}      # pv name → pvc key (chosen, not yet bound)
        self._pod_choice: dict[str, tuple[list, list]] = {}   # pod uid → decision

    def is_noop_for(self, pod) -> bool:
        # no claims, or every claim bound to an existing PV without required node affinity:
        # PreFilter finds nothing to bind, Filter passes on every node, Reserve assumes
        # nothing and PreBind has no claim to wait for
        f = self._facts(pod)
        return not f.claims or f.bound is not None and all(
            ((pv.get("spec") or _EMPTY).get("nodeAffinity") or _EMPTY).get("required") is None for pv in f.bound)

    def pre_filter(self, state: CycleState, pod) -> Status:
        bound, delayed, immediate = [], [], 0
        for claim in _claim_names(pod):
            pvc = self._pvc(pod.namespace, claim)
            if pvc is None:
                return _unresolvable(f'persistentvolumeclaim "{claim}" not found', self.name)
            if (pvc.get("metadata") or {}).get("deletionTimestamp"):
                return _unresolvable(f'persistentvolumeclaim "{claim}" is being deleted', self.name)
            spec = pvc.get("spec") or {}
            if spec.get("volumeName"):
                bound.append((pvc, self._pv(spec["volumeName"])))
                continue
            sc = self._sc(spec.get("storageClassName", ""))
            if sc is not None and sc.get("volumeBindingMode") == WFFC:
                delayed.append(pvc)
            else:
                immediate += 1
        if immediate:
            return _unresolvable(ERR_UNBOUND_IMMEDIATE, self.name)
        candidates = {_pvc_key(p): self._static_candidates(p) for p in delayed}
        state.write(self.KEY, _BindingState(bound, delayed, candidates))
        return Status.ok()

    def _static_candidates(self, pvc: dict) -> list[dict]:
        spec = pvc.get("spec") or {}
        key = _pvc_key(pvc)
        want = _storage(pvc, "spec", "resources", "requests", "storage")
        modes = set(spec.get("accessModes") or [])
        vmode = spec.get("volumeMode") or "Filesystem"
        scn = spec.get("storageClassName", "") or ""
        sel = LabelSelector(spec["selector"]) if spec.get("selector") else None
        uid = (pvc.get("metadata") or {}).get("uid")
        out = []
        for pv in self._lister("persistentvolumes").values():
            ps = pv.get("spec") or {}
            name = (pv.get("metadata") or {}).get("name", "")
            ref = ps.get("claimRef")
            if ref and not (ref.get("uid") == uid or (not ref.get("uid") and
                                                      f"{ref.get('namespace')}/{ref.get('name')}" == key)):
                continue
            if self._assumed.get(name, key) != key:
                continue
            if _pv_class(pv) != scn or (ps.get("volumeMode") or "Filesystem") != vmode:
                continue
            if (pv.get("status") or {}).get("phase", "Available") not in ("Available", "Pending", ""):
                continue
            if _storage(pv, "spec", "capacity", "storage") < want or not modes <= set(ps.get("accessModes") or []):
                continue
            if sel is not None and not sel.matches((pv.get("metadata") or {}).get("labels")):
                continue
            out.append(pv)
        out.sort(key=lambda p: (_storage(p, "spec", "capacity", "storage"), p["metadata"]["name"]))
        return out

    def _can_provision(self, pvc: dict, node: str, labels: dict) -> bool:
        sc = self._sc((pvc.get("spec") or {}).get("storageClassName", ""))
        if sc is None or sc.get("provisioner", NO_PROVISIONER) == NO_PROVISIONER:
            return False
        topo = sc.get("allowedTopologies")
        if not topo:
            return True
        for term in topo:
            exprs = term.get("matchLabelExpressions") or []
            if all(labels.get(e.get("key")) in (e.get("values") or []) for e in exprs):
                return True
        return False

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        try:
            s: _BindingState = state.read(self.KEY)
        except KeyError:
            return Status.ok()
        labels = self._node_labels(node_name)
        for pvc, pv in s.bound:
            if pv is None:
                return _unresolvable(f'persistentvolume "{pvc["spec"]["volumeName"]}" not found', self.name)
            if not _pv_node_ok(pv, node_name, labels):
                return _unresolvable(ERR_NODE_CONFLICT, self.name)
        static, provision, taken = [], [], set()
        for pvc in s.delayed:
            pick = None
            for pv in s.candidates[_pvc_key(pvc)]:
                name = pv["metadata"]["name"]
                if name not in taken and _pv_node_ok(pv, node_name, labels):
                    pick = name
                    break
            if pick is not None:
                taken.add(pick)
                static.append((pvc, pick))
            elif self._can_provision(pvc, node_name, labels):
                provision.append(pvc)
            else:
                return Status.unschedulable(ERR_NO_PV, plugin=self.name)
        with state.lock():
            s.decisions[node_name] = (static, provision)
        return Status.ok()

    def reserve(self, state: CycleState, pod, node_name: str) -> Status:
        try:
            s: _BindingState = state.read(self.KEY)
        except KeyError:
            return Status.ok()
        static, provision = s.decisions.get(node_name, ([], []))
        for pvc, pv_name in static:
            owner = self._assumed.get(pv_name)
            if owner is not None and owner != _pvc_key(pvc):
                self.unreserve(state, pod, node_name)
                return Status.error(f"persistentvolume {pv_name} was assumed by {owner}", plugin=self.name)
            self._assumed[pv_name] = _pvc_key(pvc)
        self._pod_choice[pod.uid] = (static, provision)
        return Status.ok()

    def unreserve(self, state: CycleState, pod, node_name: str) -> None:
        static, _ = self._pod_choice.pop(pod.uid, ([], []))
        for pvc, pv_name in static:
            if self._assumed.get(pv_name) == _pvc_key(pvc):
                self._assumed.pop(pv_name, None)

    async def pre_bind(self, state: CycleState, pod, node_name: str) -> Status:
        choice = self._pod_choice.get(pod.uid)
        if choice is None:
            return Status.ok()
        static, provision = choice
        client = self.handle.client
        try:
            for pvc, pv_name in static:
                m = pvc["metadata"]
                ref = {"kind": "PersistentVolumeClaim", "apiVersion": "v1", "namespace": m.get("namespace", "default"),
                       "name": m["name"], "uid": m.get("uid", "")}
                await client.patch("persistentvolumes", pv_name, {"spec": {"claimRef": ref}})
            for pvc in provision:
                m = pvc["metadata"]
                await client.patch("persistentvolumeclaims", m["name"],
                                   {"metadata": {"annotations": {ANN_SELECTED_NODE: node_name}}},
                                   namespace=m.get("namespace", "default"))
            keys = [_pvc_key(p) for p, _ in static] + [_pvc_key(p) for p in provision]
            deadline = time.monotonic() + self.bind_timeout
            pvcs = self._lister("persistentvolumeclaims")
            while True:
                if all(((pvcs.get(k) or {}).get("status") or {}).get("phase") == "Bound" for k in keys):
                    break
                if time.monotonic() > deadline:
                    return Status.error(f"binding volumes: timed out waiting for {len(keys)} claim(s)",
                                        plugin=self.name)
                await asyncio.sleep(0.01)
        except Exception as e:  # noqa: BLE001 - apiserver errors fail the bind (pod is retried)
            return Status.error(f"binding volumes: {e}", plugin=self.name)
        finally:
            self.unreserve(state, pod, node_name)
        return Status.ok()


# ================================================================= attach limits
class _LimitsBase(_VolumeBase, FilterPlugin):
    """Counts unique attachable volumes per (driver) on the node plus the pod's new ones."""

    new_only = False   # CSI: skip drivers the pod adds no new volume to (NodeVolumeLimits)

    def _pod_ids(self, ns: str, spec: dict) -> dict[str, set[str]]:
        raise NotImplementedError

    def _limits(self, node: str) -> dict[str, int]:
        raise NotImplementedError

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        mine = self._pod_ids(pod.namespace, pod.obj.get("spec") or {})
        if not any(mine.values()):
            return Status.ok()
        limits = self._limits(node_name)
        if not limits:
            return Status.ok()
        attached: dict[str, set[str]] = {}
        for obj in self._node_pod_objs(node_name):
            ns = (obj.get("metadata") or {}).get("namespace", "default")
            for d, ids in self._pod_ids(ns, obj.get("spec") or {}).items():
                attached.setdefault(d, set()).update(ids)
        for d, ids in mine.items():
            lim = limits.get(d)
            have = attached.get(d, set())
            if self.new_only and ids <= have:
                continue      # upstream CSILimits compares only drivers the pod adds volumes to
            if lim is not None and len(have | ids) > lim:
                return Status.unschedulable(ERR_MAX_VOLUMES, plugin=self.name)
        return Status.ok()


class NodeVolumeLimits(_LimitsBase):
    """CSI attach limits: ``CSINode.spec.drivers[].allocatable.count`` (or node allocatable
    ``attachable-volumes-csi-<driver>``). As upstream v1.20 CSILimits, a driver whose volumes
    of the pod are all attached on the node already is not compared (the in-tree limits are:
    existing + new > limit rejects even with nothing new)."""
    name = "NodeVolumeLimits"
    new_only = True
    pod_flags = PF_CLAIMS
    claim_inert_ok = True   # the lane's claim table covers it (claim_lane): a no-op or an engine filter
    reads_flags = PF_CLAIMS  # other pods' features this plugin reads (needs_lane_mirror)
    watches = ("persistentvolumeclaims", "persistentvolumes", "storageclasses", "csinodes")

    def __init__(self, args=None, handle=None) -> None:
        super().__init__(args, handle)
        self._csinode_limits = (-1, frozenset())   # (csinodes generation, drivers a CSINode limits)

    def is_noop_for(self, pod) -> bool:
        # no claims, or none of the CSI drivers its claims count against has an attach limit on
        # any node (the filter only compares drivers with a limit)
        f = self._facts(pod)
        return not f.claims or not f.csi or not (f.csi & self._limited_drivers())

    def _limited_drivers(self) -> set:
        gen = self.handle.generation("csinodes") if hasattr(self.handle, "generation") else -2
        g, drivers = self._csinode_limits
        if g != gen or gen == -2:
            drivers = frozenset(_csinode_drivers(self._lister("csinodes")))
            self._csinode_limits = (gen, drivers)
        return drivers | set(getattr(self.handle.cache, "csi_limit_drivers", ()))

    def _pod_ids(self, ns: str, spec: dict) -> dict[str, set[str]]:
        out: dict[str, set[str]] = {}
        for v in spec.get("volumes") or ():
            if "persistentVolumeClaim" not in v:
                continue
            claim = (v["persistentVolumeClaim"] or {}).get("claimName", "")
            pvc = self._pvc(ns, claim)
            if pvc is None:
                continue
            pv = self._pv((pvc.get("spec") or {}).get("volumeName", ""))
            if pv is not None:
                csi = (pv.get("spec") or {}).get("csi")
                if csi:
                    d = csi.get("driver", "")
                    out.setdefault(d, set()).add(f"{d}/{csi.get('volumeHandle', '')}")
                continue
            sc = self._sc((pvc.get("spec") or {}).get("storageClassName", ""))
            if sc is not None and sc.get("provisioner", NO_PROVISIONER) != NO_PROVISIONER:
                d = sc["provisioner"]
                out.setdefault(d, set()).add(f"{d}/{ns}/{claim}")
        return out

    def _limits(self, node: str) -> dict[str, int]:
        out: dict[str, int] = {}
        n = self.handle.cache.nodes.get(node)
        if n is not None:
            alloc = (n.obj.get("status") or {}).get("allocatable") or {}
            for k, v in alloc.items():
                if k.startswith("attachable-volumes-csi-"):
                    out[k[len("attachable-volumes-csi-"):]] = int(v)
        csinode = self._lister("csinodes").get(node)
        for d in ((csinode or {}).get("spec") or {}).get("drivers") or ():
            cnt = (d.get("allocatable") or {}).get("count")
            if cnt is not None:
                out[d.get("name", "")] = int(cnt)
        return out


class _InTreeLimits(_LimitsBase):
    kind = ""
    id_field = ""
    alloc_key = ""
    default_max = 0
    pod_flags = PF_CLAIMS | PF_DISKS
    reads_flags = PF_CLAIMS | PF_DISKS  # other pods' features this plugin reads (needs_lane_mirror)
    claim_inert_ok = True   # a no-op for a pod whose claims are all in the lane's claim table (PF_DISKS: not)

    def is_noop_for(self, pod) -> bool:
        # no inline volume of this kind and no PVC bound to one: the filter has nothing to count
        f = self._facts(pod)
        return self.kind not in f.inline and self.kind not in f.pv_kinds

    def _pod_ids(self, ns: str, spec: dict) -> dict[str, set[str]]:
        ids: set[str] = set()
        for v in spec.get("volumes") or ():
            if self.kind in v:
                ids.add(str((v[self.kind] or {}).get(self.id_field, "")))
            elif "persistentVolumeClaim" in v:
                pvc = self._pvc(ns, (v["persistentVolumeClaim"] or {}).get("claimName", ""))
                pv = self._pv(((pvc or {}).get("spec") or {}).get("volumeName", ""))
                src = ((pv or {}).get("spec") or {}).get(self.kind)
                if src:
                    ids.add(str(src.get(self.id_field, "")))
        return {self.kind: ids} if ids else {}

    def _limits(self, node: str) -> dict[str, int]:
        n = self.handle.cache.nodes.get(node)
        alloc = ((n.obj.get("status") or {}).get("allocatable") or {}) if n is not None else {}
        return {self.kind: int(alloc.get(self.alloc_key, self.default_max))}


class EBSLimits(_InTreeLimits):
    name = "EBSLimits"
    kind, id_field, alloc_key, default_max = "awsElasticBlockStore", "volumeID", "attachable-volumes-aws-ebs", 39


class GCEPDLimits(_InTreeLimits):
    name = "GCEPDLimits"
    kind, id_field, alloc_key, default_max = "gcePersistentDisk", "pdName", "attachable-volumes-gce-pd", 16


class AzureDiskLimits(_InTreeLimits):
    name = "AzureDiskLimits"
    kind, id_field, alloc_key, default_max = "azureDisk", "diskName", "attachable-volumes-azure-disk", 16


class CinderLimits(_InTreeLimits):
    """Not in the v1.20 default profile; enabled by configs that name it."""
    name = "CinderLimits"
    kind, id_field, alloc_key, default_max = "cinder", "volumeID", "attachable-volumes-cinder", 256


def _csinode_drivers(csinodes: dict) -> set:
    """CSI drivers some CSINode reports an attach limit for (``drivers[].allocatable.count``)."""
    return {d.get("name", "") for cn in csinodes.values() for d in ((cn.get("spec") or _EMPTY).get("drivers") or ())
            if (d.get("allocatable") or _EMPTY).get("count") is not None}


def claim_inert(pvc: dict, pvs: dict, limited: set) -> bool:
    """One PersistentVolumeClaim every volume plugin has nothing to check for: not being
    deleted, bound to a PV that exists and has no required node affinity, no zone / region
    labels and no in-tree attachable disk, and either not a CSI volume or one whose driver has
    no attach limit on any node (``limited``: the drivers that have one). A pod whose claims
    are all inert is a no-op for VolumeBinding, VolumeZone, NodeVolumeLimits and the in-tree
    limits (each claim satisfies the per-claim half of their ``is_noop_for``)."""
    if claim_lane(pvc, pvs) is not None:
        return False
    csi = (pvs[pvc["spec"]["volumeName"]].get("spec") or _EMPTY).get("csi")
    return not (csi and csi.get("driver", "") in limited)


NOT_LANE = "not-lane"                     # claim_lane: the claim needs the Python volume plugins
_LANE_NODE_OPS = ("In", "NotIn", "Exists", "DoesNotExist")
_GO_INT = re.compile(r"[+-]?[0-9]+\Z")


def _go_int64(s: str) -> bool:
    """``strconv.ParseInt(s, 10, 64)`` succeeds (the engine's Gt / Lt threshold)."""
    return bool(_GO_INT.match(s)) and -(1 << 63) <= int(s) < (1 << 63)


def claim_lane(pvc: dict, pvs: dict):
    """What the native lane needs to run a pod that mounts this claim: ``NOT_LANE`` when the
    claim needs the Python volume plugins, else the constraints its bound PV puts on nodes —
    None or ``(node_terms | None, zone_terms | None)``:

    * ``node_terms`` — the PV's ``nodeAffinity.required`` (VolumeBinding's filter for a bound
      claim: any term matches; a term without requirements matches nothing), only with the
      operators In / NotIn / Exists / DoesNotExist, Gt / Lt on one Go int64, and ``matchFields`` only as In / NotIn on ``metadata.name``;
    * ``zone_terms`` — VolumeZone's filter as two OR'ed terms: the node has none of the zone /
      region labels, or it has every label the PV has with a value the PV allows ("__"-separated).

    A lane-able claim is not being deleted, is bound to a PV that exists and has no in-tree
    attachable disk. CSI attach limits are counted by the engine (``claim_volume``)."""
    if (pvc.get("metadata") or _EMPTY).get("deletionTimestamp"):
        return NOT_LANE
    name = (pvc.get("spec") or _EMPTY).get("volumeName", "")
    pv = pvs.get(name) if name else None
    if pv is None:
        return NOT_LANE
    ps = pv.get("spec") or _EMPTY
    if any(ps.get(k) for k in _ATTACHABLE_KINDS):
        return NOT_LANE
    node = None
    req = (ps.get("nodeAffinity") or _EMPTY).get("required")
    if req is not None:
        if not isinstance(req, dict):
            return NOT_LANE
        terms = []
        for t in req.get("nodeSelectorTerms") or []:
            if not isinstance(t, dict):
                return NOT_LANE
            exprs = []
            for f in t.get("matchFields") or []:      # the node name; other fields fail the term
                if f.get("key") != "metadata.name" or f.get("operator", "In") not in ("In", "NotIn"):
                    return NOT_LANE
                exprs.append((FIELD_NODE_NAME, f.get("operator", "In"), tuple(str(v) for v in f.get("values") or [])))
            for e in t.get("matchExpressions") or []:
                op = e.get("operator", "In")
                vals = tuple(str(v) for v in e.get("values") or [])
                if op in ("Gt", "Lt"):
                    # one Go int64 value (strconv.ParseInt), else the Python plugin decides
                    if len(vals) != 1 or not _go_int64(vals[0]):
                        return NOT_LANE
                elif op not in _LANE_NODE_OPS:
                    return NOT_LANE
                exprs.append((e.get("key", ""), op, vals))
            terms.append(tuple(exprs))
        node = tuple(terms)
    labels = (pv.get("metadata") or _EMPTY).get("labels") or _EMPTY
    keys = [k for k in ZONE_LABELS if k in labels]
    zone = None
    if keys:
        zone = (tuple((k, "DoesNotExist", ()) for k in ZONE_LABELS),
                tuple((k, "In", tuple(str(labels[k]).split("__"))) for k in keys))
    return None if node is None and zone is None else (node, zone)


def limited_drivers(handle) -> set:
    """CSI drivers some node limits (node allocatable ``attachable-volumes-csi-<driver>`` or a
    CSINode ``allocatable.count``): NodeVolumeLimits counts those drivers' volumes."""
    return _csinode_drivers(handle.lister("csinodes")) | set(getattr(handle.cache, "csi_limit_drivers", ()))


def lane_claims(handle) -> dict:
    """The claim table over the whole PVC lister: key ("namespace/name") → ``claim_lane``
    value, for every lane-able claim."""
    pvs = handle.lister("persistentvolumes")
    out = {}
    for key, pvc in handle.lister("persistentvolumeclaims").items():
        v = claim_lane(pvc, pvs)
        if v is not NOT_LANE:
            out[key] = v
    return out


def inert_claims(handle) -> set:
    """Every inert claim ("namespace/name", ``claim_inert``) of the PVC lister."""
    pvs, limited = handle.lister("persistentvolumes"), limited_drivers(handle)
    return {k for k, pvc in handle.lister("persistentvolumeclaims").items() if claim_inert(pvc, pvs, limited)}


def claim_volume(key: str, pvc: dict, pvs: dict, scs: dict) -> Optional[tuple]:
    """(driver, unique volume id) NodeVolumeLimits counts for a pod volume on this claim
    (``_pod_ids``): a bound CSI PV's (driver, "<driver>/<volumeHandle>"); with no PV yet and a
    provisioning StorageClass, (provisioner, "<provisioner>/<namespace>/<claim>"); else None."""
    spec = pvc.get("spec") or _EMPTY
    name = spec.get("volumeName", "")
    pv = pvs.get(name) if name else None
    if pv is not None:
        csi = (pv.get("spec") or _EMPTY).get("csi")
        if csi:
            d = csi.get("driver", "")
            return d, f"{d}/{csi.get('volumeHandle', '')}"
        return None
    scn = spec.get("storageClassName", "")
    sc = scs.get(scn) if scn else None
    if sc is not None and sc.get("provisioner", NO_PROVISIONER) != NO_PROVISIONER:
        d = sc["provisioner"]
        return d, f"{d}/{key}"
    return None


def claim_volumes(handle) -> dict:
    """``claim_volume`` of every PVC of the lister that has one."""
    pvs, scs = handle.lister("persistentvolumes"), handle.lister("storageclasses")
    out = {}
    for key, pvc in handle.lister("persistentvolumeclaims").items():
        v = claim_volume(key, pvc, pvs, scs)
        if v is not None:
            out[key] = v
    return out


def node_csi_limits(node_obj: Optional[dict], csinode: Optional[dict]) -> dict:
    """NodeVolumeLimits._limits: attach limits per CSI driver from the node's allocatable
    (``attachable-volumes-csi-<driver>``), overridden by its CSINode's ``allocatable.count``.
    None when a value is not an integer (the Python plugin decides there)."""
    out = {}
    try:
        alloc = ((node_obj or _EMPTY).get("status") or _EMPTY).get("allocatable") or _EMPTY
        for k, v in alloc.items():
            if k.startswith("attachable-volumes-csi-"):
                out[k[len("attachable-volumes-csi-"):]] = int(v)
        for d in ((csinode or _EMPTY).get("spec") or _EMPTY).get("drivers") or ():
            cnt = (d.get("allocatable") or _EMPTY).get("count")
            if cnt is not None:
                out[d.get("name", "")] = int(cnt)
    except (TypeError, ValueError, AttributeError):
        return None
    return out


def pvc_claim_keys(pod) -> list:
    """"namespace/claim" of a pod's persistentVolumeClaim volumes (what NodeVolumeLimits counts
    of it: ``_pod_ids`` skips ephemeral volumes)."""
    return [f"{pod.namespace}/{(v['persistentVolumeClaim'] or _EMPTY).get('claimName', '')}"
            for v in _volumes(pod) if "persistentVolumeClaim" in v]


class LaneClaims:
    """The native lane's claim table (``lane_claims``) and the engine's claim volumes
    (``claim_volumes``) kept up to date per event instead of recomputed over every PVC: a PVC
    event re-evaluates that claim, a PV event the claims bound to it (an index PV name → claim
    keys), a StorageClass event all of them. ``refresh`` returns the changes since the last
    call: ``(table | None, changed, removed, volumes | None, volumes changed, volumes removed)``
    — a whole table instead of None on the first call and after a StorageClass event."""

    def __init__(self, handle) -> None:
        self.handle = handle
        self.table: dict = {}
        self.vols: dict = {}
        self._pv_of: dict[str, str] = {}          # claim key → the PV name it is bound to
        self._claims_of: dict[str, set] = {}      # PV name → claim keys bound to it
        self._dirty: set = set()
        self._all = True                          # first refresh: every claim

    @property
    def keys(self):
        return self.table.keys()

    def pvc_event(self, obj: dict) -> None:
        m = obj.get("metadata") or _EMPTY
        self._dirty.add(f"{m.get('namespace') or 'default'}/{m.get('name', '')}")

    def pv_event(self, obj: dict) -> None:
        self._dirty |= self._claims_of.get((obj.get("metadata") or _EMPTY).get("name", ""), set())

    def sc_event(self, obj: dict) -> None:
        self._all = True

    def _index(self, key: str, pv: str) -> None:
        old = self._pv_of.get(key)
        if old == pv:
            return
        if old is not None:
            ks = self._claims_of.get(old)
            if ks is not None:
                ks.discard(key)
                if not ks:
                    del self._claims_of[old]
        if pv:
            self._pv_of[key] = pv
            self._claims_of.setdefault(pv, set()).add(key)
        else:
            self._pv_of.pop(key, None)

    @staticmethod
    def _diff(old: dict, new: dict) -> tuple:
        return {k: v for k, v in new.items() if old.get(k, NOT_LANE) != v}, set(old) - set(new)

    def refresh(self):
        h = self.handle
        pvcs, pvs, scs = h.lister("persistentvolumeclaims"), h.lister("persistentvolumes"), h.lister("storageclasses")
        if self._all:
            self._all, self._dirty = False, set()
            self._pv_of, self._claims_of = {}, {}
            table, vols = {}, {}
            for key, pvc in pvcs.items():
                self._index(key, (pvc.get("spec") or _EMPTY).get("volumeName", "") or "")
                v = claim_lane(pvc, pvs)
                if v is not NOT_LANE:
                    table[key] = v
                cv = claim_volume(key, pvc, pvs, scs)
                if cv is not None:
                    vols[key] = cv
            changed, removed = self._diff(self.table, table)
            vchanged, vremoved = self._diff(self.vols, vols)
            self.table, self.vols = table, vols
            return table, changed, removed, vols, vchanged, vremoved
        changed, removed, vchanged, vremoved = {}, set(), {}, set()
        dirty, self._dirty = self._dirty, set()
        for key in dirty:
            pvc = pvcs.get(key)
            self._index(key, ((pvc.get("spec") or _EMPTY).get("volumeName", "") or "") if pvc is not None else "")
            v = NOT_LANE if pvc is None else claim_lane(pvc, pvs)
            if v is NOT_LANE:
                if key in self.table:
                    del self.table[key]
                    removed.add(key)
            elif self.table.get(key, NOT_LANE) != v:
                self.table[key] = v
                changed[key] = v
            cv = None if pvc is None else claim_volume(key, pvc, pvs, scs)
            if cv is None:
                if key in self.vols:
                    del self.vols[key]
                    vremoved.add(key)
            elif self.vols.get(key) != cv:
                self.vols[key] = cv
                vchanged[key] = cv
        return None, changed, removed, None, vchanged, vremoved


# the in-tree attach-limit plugins' volume kinds (what _VolFacts resolves for them)
_ATTACHABLE_KINDS = tuple(c.kind for c in (EBSLimits, GCEPDLimits, AzureDiskLimits, CinderLimits))

VOLUME_PLUGINS = (VolumeRestrictions, VolumeZone, VolumeBinding, NodeVolumeLimits, EBSLimits, GCEPDLimits,
                  AzureDiskLimits, CinderLimits)
