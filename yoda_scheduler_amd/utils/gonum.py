"""Go integer semantics used by the reference policy code.

The reference parses every ``scv/*`` label with ``strconv.Atoi`` and silently maps
errors to 0 (``pkg/yoda/filter/filter.go:60-82``); negative values are then cast to
``uint``/``uint64`` and wrap (quirk Q5). All score arithmetic is unsigned 64-bit with
truncating division (``pkg/yoda/score/algorithm.go:57-87``) and ``NormalizeScore``
works in int64 (``pkg/yoda/scheduler.go:132-157``). These helpers reproduce that
bit-exactly so the compat mode and the native core can be parity-tested.
"""
from __future__ import annotations

U64 = (1 << 64) - 1
I64_MAX = (1 << 63) - 1
I64_MIN = -(1 << 63)


def atoi(s: str) -> tuple[int, bool]:
    """Go ``strconv.Atoi``: base-10, optional sign, int64 range. Returns (value, ok)."""
    if not isinstance(s, str) or not s:
        return 0, False
    body = s
    if body[0] in "+-":
        body = body[1:]
    if not body or not all("0" <= c <= "9" for c in body):
        return 0, False
    v = int(s)
    if v > I64_MAX or v < I64_MIN:
        return 0, False
    return v, True


def atoi_or_zero(s: str) -> int:
    v, ok = atoi(s)
    return v if ok else 0


def str_to_uint(s: str) -> int:
    """``filter.strToUint`` / ``StrToUint64``: Atoi, error → 0, negative wraps mod 2^64."""
    return atoi_or_zero(s) & U64


def str_to_int64(s: str) -> int:
    return atoi_or_zero(s)


def uint64_to_int64(v: int) -> int:
    """``filter.Uint64ToInt64`` (filter.go:84): format + Atoi; > MaxInt64 → 0."""
    v &= U64
    return v if v <= I64_MAX else 0


def u64(v: int) -> int:
    return v & U64


def udiv(a: int, b: int) -> int:
    """Unsigned 64-bit division; the Go code would panic on b == 0 — callers guard."""
    return (a & U64) // (b & U64)


def wrap_i64(v: int) -> int:
    v &= U64
    return v - (1 << 64) if v > I64_MAX else v


def idiv_trunc(a: int, b: int) -> int:
    """Go int64 division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q
