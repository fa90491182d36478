"""Kubernetes resource.Quantity parsing (the subset schedulers need)."""
from __future__ import annotations

from decimal import Decimal, InvalidOperation

_BIN = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}
_DEC = {"n": Decimal("1e-9"), "u": Decimal("1e-6"), "m": Decimal("1e-3"), "": Decimal(1),
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
    for suf, mul in _BIN.items():
        if s.endswith(suf):
            return Decimal(s[: -len(suf)]) * mul
    # exponent form 1e3 / 1E3
    try:
        if s[-1] in _DEC and s[-1] != "":
            suf = s[-1]
            if suf.isalpha():
                return Decimal(s[:-1]) * _DEC[suf]
        return Decimal(s)
    except (InvalidOperation, KeyError) as e:
        raise ValueError(f"invalid quantity {q!r}") from e


def cpu_millis(q) -> int:
    """CPU quantity → millicores (rounded up like MilliValue)."""
    d = parse_quantity(q) * 1000
    i = int(d)
    return i + (1 if d > i else 0)


def bytes_of(q) -> int:
    d = parse_quantity(q)
    i = int(d)
    return i + (1 if d > i else 0)
