"""xGMI-aware gang (multi-GPU) placement inside one MI355X node — Python reference of
``Engine::select_gpus`` / ``gang_objective`` (native/core/engine.cpp), bit-exact.

An MI355X node is a full xGMI mesh (7 links/GPU, ~153 GB/s each): every pair is one
hop, so what differentiates GPU sets is *link load* (a TP/SP ring is bound by its
slowest link), NUMA locality of the host side and how much HBM headroom is left.
The reference has no notion of this (``scv/number`` only counts cards,
``pkg/yoda/filter/filter.go:11-50``).

Objective (lower is better), integer arithmetic with truncating division:

    P        = k(k−1)/2 pairs
    link_bad = (P·10000 − Σ_pairs q(a,b)) · 100 / P          q = 9000·(1−load) over xGMI, same phys → 10000
    min_bad  = (10000 − min_pairs q(a,b)) · 100               bottleneck: a ring is as fast as its slowest link
    numa_bad = (#NUMA nodes − 1) · 10^6 / (k−1)
    leftover = Σ(eff_free − m) · 10^6 / Σ total                 spread: 10^6 − leftover
    occ_bad  = Σ occupancy(1e-4) · 100 / k
    obj      = w_link·link_bad + w_minlink·min_bad + w_numa·numa_bad + w_fit·fit + w_occ·occ_bad

All k-subsets of eligible cards are enumerated in lexicographic order when there are at
most ``enum_limit`` of them (C(8,4)=70 on an SPX node); the first minimum wins.
Larger (CPX-partitioned) nodes fall back to greedy growth.
"""
from __future__ import annotations

from dataclasses import dataclass
from itertools import combinations
from math import comb
from typing import Sequence


@dataclass
class GangWeights:
    link: int = 4
    numa: int = 2
    fit: int = 1
    occ: int = 1
    binpack: bool = False
    gang_score: int = 3
    enum_limit: int = 5000
    minlink: int = 2


@dataclass
class GpuView:
    eff_free: int
    total: int
    phys: int
    numa: int
    occ_q: int


def _trunc_div(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def objective(cards: Sequence[GpuView], link_q: Sequence[int], nphys: int, subset: Sequence[int], m: int,
              w: GangWeights) -> tuple[int, int]:
    k = len(subset)
    P = k * (k - 1) // 2
    qsum, qmin = 0, 10000
    numa = set()
    free_after = total = occ = 0
    for ai in range(k):
        a = cards[subset[ai]]
        numa.add(a.numa & 63)
        free_after += a.eff_free - m
        total += a.total
        occ += a.occ_q
        for bi in range(ai + 1, k):
            b = cards[subset[bi]]
            q = 10000
            if a.phys != b.phys and a.phys < nphys and b.phys < nphys:
                q = link_q[a.phys * nphys + b.phys]
            qsum += q
            qmin = min(qmin, q)
    link_bad = _trunc_div((P * 10000 - qsum) * 100, P) if P else 0
    min_bad = (10000 - qmin) * 100 if P else 0
    numa_bad = _trunc_div((len(numa) - 1) * 1_000_000, k - 1) if k > 1 else 0
    leftover = _trunc_div(free_after * 1_000_000, total) if total else 0
    fit = leftover if w.binpack else 1_000_000 - leftover
    occ_bad = _trunc_div(occ * 100, k) if k else 0
    return w.link * link_bad + w.minlink * min_bad + w.numa * numa_bad + w.fit * fit + w.occ * occ_bad, link_bad


def select(cards: Sequence[GpuView], eligible: Sequence[int], k: int, m: int, link_q: Sequence[int], nphys: int,
           w: GangWeights) -> tuple[bool, list[int], int]:
    """Returns (ok, chosen card indices, quality 0..10000)."""
    if k == 0:
        return True, [], 10000
    E = list(eligible)
    if len(E) < k:
        return False, [], 10000
    best, best_link, out = None, 0, []
    if comb(len(E), k) <= w.enum_limit:
        for sub in combinations(E, k):
            obj, lb = objective(cards, link_q, nphys, sub, m, w)
            if best is None or obj < best:
                best, best_link, out = obj, lb, list(sub)
    else:
        cur: list[int] = []
        used = set()
        for _ in range(k):
            bo, bi = None, -1
            for e in E:
                if e in used:
                    continue
                obj, _ = objective(cards, link_q, nphys, cur + [e], m, w)
                if bo is None or obj < bo:
                    bo, bi = obj, e
            used.add(bi)
            cur.append(bi)
        out = sorted(cur)
        _, best_link = objective(cards, link_q, nphys, out, m, w)
    return True, out, 10000 - _trunc_div(best_link, 100)
