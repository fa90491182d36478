"""``ImageLocality`` and ``NodePreferAvoidPods`` — two score plugins of the upstream v1.20
default profile that the reference's scheduler runs next to ``yoda`` in the same
compiled cycle (weights 1 and 10000; ``/root/reference/deploy/yoda-scheduler.yaml:21-31`` keeps
the defaults, ``/root/reference/pkg/yoda/scheduler.go:76-130`` is the cycle they share).

Both score natively (``native/core/engine.cpp`` ``S_IMAGE_LOCALITY`` / ``S_PREFER_AVOID``): the
engine keeps every node's ``status.images``, the per-image node count and the preferAvoidPods
controllers, and each pod's normalized images and RC / RS controller, so a real cluster —
every kubelet reports its images — keeps its pods on the native cycle and the native lane.
The Python ``score`` methods below are the executable spec the native terms are pinned
against (``tests/test_native_default_plugins.py``).
"""
from __future__ import annotations

import json

from ..framework.interfaces import CycleState, NativeBinding, ScorePlugin, Status, MAX_NODE_SCORE
from ..models.pod import normalize_image
from ..ops.native import core

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
    reads_flags = 0  # other pods' features this plugin reads (needs_lane_mirror)

    def native(self):
        return NativeBinding(score_index=core().S_IMAGE_LOCALITY)

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
    reads_flags = 0  # other pods' features this plugin reads (needs_lane_mirror)

    def native(self):
        return NativeBinding(score_index=core().S_PREFER_AVOID)

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        node = self.handle.cache.nodes.get(node_name)
        ctl = _controller(pod)
        if node is None or ctl is None or not node.avoid:
            return MAX_NODE_SCORE, Status.ok()
        try:
            avoids = json.loads(node.avoid).get("preferAvoidPods") or []
        except (ValueError, AttributeError):
            return MAX_NODE_SCORE, Status.ok()
        for a in avoids if isinstance(avoids, list) else ():
            if not isinstance(a, dict):
                continue
            pc = ((a.get("podSignature") or {}).get("podController")) or {}
            if (pc.get("kind"), pc.get("uid")) == ctl:
                return 0, Status.ok()
        return MAX_NODE_SCORE, Status.ok()
