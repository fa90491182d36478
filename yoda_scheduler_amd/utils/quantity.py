"""Kubernetes resource.Quantity parsing (the subset schedulers need).

Parsed values are memoised: a burst of pods repeats the same few request strings
("100m", "128Mi"), and Decimal parsing is the slow part of decoding a pod.
"""
from __future__ import annotations

from decimal import Decimal, InvalidOperation
from functools import lru_cache

_BIN = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}
_DEC = {"n": Decimal("1e-9"), "u": Decimal("1e-6"), "m": Decimal("1e-3"),
        "k": Decimal("1e3"), "M": Decimal("1e6"), "G": Decimal("1e9"), "T": Decimal("1e12"),
        "P": Decimal("1e15"), "E": Decimal("1e18")}


def parse_quantity(q) -> Decimal:
    if q is None:
        return Decimal(0)
    if isinstance(q, (int, float)):
        return Decimal(str(q))
    s = str(q).strip()
    if not s:
        return Decimal(0)
    try:
        for suf, mul in _BIN.items():
            if s.endswith(suf):
                return Decimal(s[: -len(suf)]) * mul
        if s[-1] in _DEC:
            return Decimal(s[:-1]) * _DEC[s[-1]]
        return Decimal(s)          # plain number or exponent form (1e3)
    except InvalidOperation as e:
        raise ValueError(f"invalid quantity {q!r}") from e


def _ceil(d: Decimal) -> int:
    i = int(d)
    return i + (1 if d > i else 0)


@lru_cache(maxsize=4096)
def _cpu_millis_str(s: str) -> int:
    return _ceil(parse_quantity(s) * 1000)


@lru_cache(maxsize=4096)
def _bytes_str(s: str) -> int:
    return _ceil(parse_quantity(s))


def cpu_millis(q) -> int:
    """CPU quantity → millicores (rounded up like MilliValue)."""
    if isinstance(q, str):
        return _cpu_millis_str(q)
    return _ceil(parse_quantity(q) * 1000)


def bytes_of(q) -> int:
    if isinstance(q, str):
        return _bytes_str(q)
    return _ceil(parse_quantity(q))
