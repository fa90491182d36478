"""``ImageLocality`` and ``NodePreferAvoidPods`` — the two remaining score plugins of the
upstream v1.20 default profile that the reference's scheduler runs next to
``yoda`` (weights 1 and 10000).

Both are no-ops for the common case and keep pods on the native cycle: ImageLocality
when no node reports any of the pod's images (every node would score 0), and
NodePreferAvoidPods when the pod has no ReplicationController/ReplicaSet owner or no
node carries the annotation (every node would score 100).
"""
from __future__ import annotations

import json

from ..framework.interfaces import CycleState, ScorePlugin, Status, MAX_NODE_SCORE
from ..models.pod import PF_CONTROLLER, normalize_image

MB = 1024 * 1024
MIN_THRESHOLD = 23 * MB           # upstream: below this an image is "not there"
MAX_CONTAINER_THRESHOLD = 1000 * MB


def _images(pod) -> list[str]:
    spec = pod.obj.get("spec") or {}
    return [normalize_image(c.get("image", "")) for c in spec.get("containers") or () if c.get("image")]


class ImageLocality(ScorePlugin):
    """score = 100·(clamp(Σ size·spread) − 23MB)/(1000MB·#containers − 23MB), where
    spread = (#nodes holding the image)/(#nodes) damps images present everywhere."""
    name = "ImageLocality"
    pod_flags = 0
    reads_flags = 0  # other pods' features this plugin reads (needs_lane_mirror)

    def cluster_active(self) -> bool:
        return bool(self.handle.cache.image_nodes)

    def is_noop_for(self, pod) -> bool:
        have = self.handle.cache.image_nodes
        return not have or not any(im in have for im in _images(pod))

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        cache = self.handle.cache
        node = cache.nodes.get(node_name)
        if node is None:
            return 0, Status.ok()
        total = max(1, len(cache.nodes))
        containers = (pod.obj.get("spec") or {}).get("containers") or ()
        s = 0
        for im in _images(pod):
            size = node.images.get(im)
            if size:
                s += int(size * (cache.image_nodes.get(im, 0) / total))
        hi = MAX_CONTAINER_THRESHOLD * max(1, len(containers))
        s = min(max(s, MIN_THRESHOLD), hi)
        return MAX_NODE_SCORE * (s - MIN_THRESHOLD) // (hi - MIN_THRESHOLD), Status.ok()


def _controller(pod):
    for ref in (pod.obj.get("metadata") or {}).get("ownerReferences") or ():
        if ref.get("controller") and ref.get("kind") in ("ReplicationController", "ReplicaSet"):
            return ref.get("kind"), ref.get("uid")
    return None


class NodePreferAvoidPods(ScorePlugin):
    """0 on nodes whose ``scheduler.alpha.kubernetes.io/preferAvoidPods`` annotation names
    the pod's controller, 100 elsewhere."""
    name = "NodePreferAvoidPods"
    pod_flags = PF_CONTROLLER
    reads_flags = 0  # other pods' features this plugin reads (needs_lane_mirror)

    def is_noop_for(self, pod) -> bool:
        return not self.handle.cache.avoid_nodes or _controller(pod) is None

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        node = self.handle.cache.nodes.get(node_name)
        ctl = _controller(pod)
        if node is None or ctl is None or not node.avoid:
            return MAX_NODE_SCORE, Status.ok()
        try:
            avoids = json.loads(node.avoid).get("preferAvoidPods") or []
        except (ValueError, AttributeError):
            return MAX_NODE_SCORE, Status.ok()
        for a in avoids:
            pc = ((a.get("podSignature") or {}).get("podController")) or {}
            if (pc.get("kind"), pc.get("uid")) == ctl:
                return 0, Status.ok()
        return MAX_NODE_SCORE, Status.ok()
