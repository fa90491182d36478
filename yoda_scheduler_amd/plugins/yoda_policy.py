"""Pure-Python reference of the Yoda policy — the executable spec the native core is
parity-tested against.

Two semantics:

* ``compat=True`` reproduces the reference bit-exactly, quirks included:
  - Filter counts memory-fit and clock-fit cards independently (Q3,
    ``pkg/yoda/filter/filter.go:18-58``), clock is ``==`` in Filter but ``>=`` in
    Score/collection, and Score/collection skip the health check
    (``pkg/yoda/score/algorithm.go:48``, ``pkg/yoda/collection/collection.go:46``);
  - the clock term is normalised by ``MaxBandwidth`` (Q2, ``algorithm.go:60``);
  - Allocate sums the ``scv/memory`` label of pods on the node once per pod
    (``algorithm.go:74-87``), Actual uses the sniffed ``FreeMemorySum`` (``:70-72``);
  - all arithmetic is uint64 with truncating division.
  The only deviation is Q4: a zero ``TotalMemorySum`` scores 0 instead of panicking.

* ``compat=False`` (default) is the corrected MI355X policy: per-card conjunction of
  health ∧ free ≥ m ∧ clock match, the same eligibility in every path, clock term
  normalised by ``MaxClock``, effective free memory = min(sniffed free, total −
  reserved) so in-flight pods are never double-booked (Q10), Allocate from the
  per-GPU reservation ledger (m × n per pod).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence

from ..models.labels import GpuRequest
from ..models.scv import HEALTHY, Card
from ..utils.gonum import U64, idiv_trunc, u64, udiv, uint64_to_int64, wrap_i64

# compile-time weights of the reference (algorithm.go:16-26)
BANDWIDTH_W, CLOCK_W, CORE_W, POWER_W = 1, 1, 1, 1
FREE_MEMORY_W, TOTAL_MEMORY_W = 2, 1
ACTUAL_W, ALLOCATE_W = 2, 3
MAX_NODE_SCORE = 100


@dataclass
class MaxValue:
    """``collection.MaxValue`` (collection.go:14-21); every maximum starts at 1."""
    bandwidth: int = 1
    clock: int = 1
    core: int = 1
    free_memory: int = 1
    power: int = 1
    total_memory: int = 1

    def absorb(self, c: Card, free: int | None = None) -> None:
        f = c.free_memory if free is None else free
        self.free_memory = max(self.free_memory, f)
        self.clock = max(self.clock, c.clock)
        self.total_memory = max(self.total_memory, c.total_memory)
        self.bandwidth = max(self.bandwidth, c.bandwidth)
        self.core = max(self.core, c.core)
        self.power = max(self.power, c.power)


@dataclass
class NodeView:
    """What the policy sees of one node: sniffed cards + the scheduler's ledger."""
    name: str
    cards: Sequence[Card]
    card_number: int
    free_memory_sum: int
    total_memory_sum: int
    reserved_mb: Sequence[int] = ()      # per card, from assumed/bound pods (fixed mode)
    pending_mb: Sequence[int] = ()       # part of reserved the last sample cannot reflect yet
    label_memory_sum: int = 0            # Σ scv/memory label of pods on node (compat Allocate)
    stale: bool = False

    def eff_free(self, i: int) -> int:
        """min(sampled free − pending, total − reserved), floored at 0."""
        c = self.cards[i]
        if not self.reserved_mb:
            return c.free_memory
        pend = self.pending_mb[i] if self.pending_mb else 0
        return max(0, min(c.free_memory - pend, c.total_memory - self.reserved_mb[i]))


# ------------------------------------------------------------------ predicates
def pod_fits_number(req: GpuRequest, node: NodeView) -> tuple[bool, int]:
    """filter.go:11-16"""
    if req.has_number:
        return req.number <= node.card_number, req.number
    return node.card_number > 0, 1


def card_eligible(req: GpuRequest, node: NodeView, i: int, memory: int, clock: int) -> bool:
    """Fixed-mode per-card conjunction used by Filter, PreScore and Score alike."""
    c = node.cards[i]
    if c.health != HEALTHY:
        return False
    if node.eff_free(i) < memory:
        return False
    if req.has_clock and c.clock != clock:
        return False
    if req.clock_min and c.clock < req.clock_min:
        return False
    return True


def filter_node(req: GpuRequest, node: NodeView, compat: bool = False) -> tuple[bool, int, int, int]:
    """Returns (fits, number, memory, clock). compat = (*Yoda).Filter (scheduler.go:85-92)."""
    ok, n = pod_fits_number(req, node)
    m = req.memory if req.has_memory else 0
    c = req.clock if req.has_clock else 0
    if not ok:
        return False, n, m, c
    if compat:
        fm = True
        if req.has_memory:
            cnt = sum(1 for card in node.cards if card.health == HEALTHY and card.free_memory >= m)
            fm = cnt >= n
        fc = True
        if req.has_clock:
            cnt = sum(1 for card in node.cards if card.health == HEALTHY and card.clock == c)
            fc = cnt >= n
        return fm and fc, n, m, c
    if node.stale:
        return False, n, m, c
    cnt = sum(1 for i in range(len(node.cards)) if card_eligible(req, node, i, m, c))
    return cnt >= n, n, m, c


def _score_cards(req: GpuRequest, node: NodeView, m: int, c: int, compat: bool):
    """Indices of cards that contribute to Max collection / Basic score."""
    if compat:
        return [i for i, card in enumerate(node.cards) if card.free_memory >= m and card.clock >= c]
    return [i for i in range(len(node.cards)) if card_eligible(req, node, i, m, c)]


def collect_max(req: GpuRequest, nodes: Sequence[NodeView], compat: bool = False) -> MaxValue:
    """collection.CollectMaxValues (collection.go:30-57). In fixed mode this runs in
    PreScore over the feasible nodes (Q1 fix); compat iterates every Scv."""
    mv = MaxValue()
    for node in nodes:
        fits, n, m, c = filter_node(req, node, compat)
        if not fits:
            continue
        for i in _score_cards(req, node, m, c, compat):
            mv.absorb(node.cards[i], None if compat else node.eff_free(i))
    return mv


def card_score(mv: MaxValue, card: Card, compat: bool, free: int | None = None) -> int:
    """score.CalculateCardScore (algorithm.go:57-68)."""
    f = card.free_memory if free is None else free
    bw = udiv(u64(card.bandwidth * 100), mv.bandwidth)
    clk = udiv(u64(card.clock * 100), mv.bandwidth if compat else mv.clock)
    core = udiv(u64(card.core * 100), mv.core)
    pw = udiv(u64(card.power * 100), mv.power)
    fm = udiv(u64(f * 100), mv.free_memory)
    tm = udiv(u64(card.total_memory * 100), mv.total_memory)
    return u64(u64(bw * BANDWIDTH_W + clk * CLOCK_W + core * CORE_W + pw * POWER_W)
               + fm * FREE_MEMORY_W + tm * TOTAL_MEMORY_W)


def basic_score(mv: MaxValue, req: GpuRequest, node: NodeView, compat: bool = False) -> int:
    fits, n, m, c = filter_node(req, node, compat)
    if not fits:
        return 0
    s = 0
    for i in _score_cards(req, node, m, c, compat):
        s = u64(s + card_score(mv, node.cards[i], compat, None if compat else node.eff_free(i)))
    return s


def actual_score(node: NodeView, compat: bool = False) -> int:
    """algorithm.go:70-72 (Q4 guarded)."""
    total = node.total_memory_sum if compat else sum(c.total_memory for c in node.cards)
    if total == 0:
        return 0
    free = node.free_memory_sum if compat else sum(node.eff_free(i) for i in range(len(node.cards)))
    return u64(udiv(u64(free * 100), total) * ACTUAL_W)


def allocate_score(node: NodeView, compat: bool = False) -> int:
    """algorithm.go:74-87 (Q4 guarded)."""
    if compat:
        total, alloc = node.total_memory_sum, node.label_memory_sum & U64
    else:
        total = sum(c.total_memory for c in node.cards)
        alloc = sum(node.reserved_mb) if node.reserved_mb else 0
    if total == 0 or total < alloc:
        return 0
    return u64(udiv(u64((total - alloc) * 100), total) * ALLOCATE_W)


def calculate_score(mv: MaxValue, req: GpuRequest, node: NodeView, compat: bool = False) -> int:
    """score.CalculateScore → Uint64ToInt64 (scheduler.go:124-128)."""
    s = u64(basic_score(mv, req, node, compat) + allocate_score(node, compat) + actual_score(node, compat))
    return uint64_to_int64(s)


def gang_bonus(req: GpuRequest, node: NodeView, link_q: Sequence[int], nphys: int, w=None) -> int:
    """Fixed-mode node-score bonus for multi-GPU pods: best achievable xGMI quality of a
    k-GPU set on the node (``parallel/gang.py``), × ``gangWeights.score``."""
    from ..parallel.gang import GangWeights, GpuView, select
    w = w or GangWeights()
    if not (req.has_number and 1 < req.number <= len(node.cards)):
        return 0
    m = req.memory if req.has_memory else 0
    c = req.clock if req.has_clock else 0
    views = [GpuView(node.eff_free(i), cd.total_memory, cd.phys, cd.numa_node, int(round(cd.cu_occupancy * 100)))
             for i, cd in enumerate(node.cards)]
    elig = [i for i in range(len(node.cards)) if card_eligible(req, node, i, m, c)]
    ok, _sel, q = select(views, elig, req.number, m, link_q, nphys, w)
    return (q // 100) * w.gang_score if ok else 0


def normalize_scores(scores: list[int]) -> list[int]:
    """(*Yoda).NormalizeScore (scheduler.go:132-157): highest seeded 0, lowest seeded
    scores[0], equal → lowest−1 (every node 100). int64 arithmetic."""
    if not scores:
        return []
    highest, lowest = 0, scores[0]
    for s in scores:
        lowest = min(lowest, s)
        highest = max(highest, s)
    if highest == lowest:
        lowest -= 1
    den = wrap_i64(highest - lowest)
    return [idiv_trunc(wrap_i64(wrap_i64(s - lowest) * MAX_NODE_SCORE), den) for s in scores]


def queue_less(prio_a: int, prio_b: int) -> bool:
    """sort.Less (sort.go:8-10)."""
    return prio_a > prio_b
