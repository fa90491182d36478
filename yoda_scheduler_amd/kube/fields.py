"""Field selectors (``fieldSelector=spec.nodeName=,status.phase!=Failed``), as the
apiserver applies them to lists and watches.

Upstream kube-scheduler v1.20 watches pods with
``status.phase!=Succeeded,status.phase!=Failed`` so completed pods never reach it;
SURVEY U9 (informers). Requirements are AND'ed; ``=``/``==`` and ``!=`` on a dotted
field path; a missing field reads as ``""``. Selectors compile to one closure.
"""
from __future__ import annotations

from typing import Callable, Optional

Matcher = Callable[[dict], bool]


def _getter(path: str):
    keys = tuple(path.split("."))
    if len(keys) == 2:                 # spec.nodeName, status.phase, metadata.name: unrolled
        k0, k1 = keys

        def get2(obj: dict) -> str:
            v = obj.get(k0)
            if not isinstance(v, dict):
                return ""
            v = v.get(k1)
            if v is None:
                return ""
            return v if isinstance(v, str) else str(v)
        return get2

    def get(obj: dict) -> str:
        v = obj
        for k in keys:
            if not isinstance(v, dict):
                return ""
            v = v.get(k)
            if v is None:
                return ""
        return v if isinstance(v, str) else str(v)
    return get


class FieldSelector:
    __slots__ = ("text", "reqs", "matches")

    def __init__(self, text: str) -> None:
        self.text = text
        self.reqs: list[tuple[str, str, str]] = []
        for part in (p.strip() for p in text.split(",")):
            if not part:
                continue
            if "!=" in part:
                k, v = part.split("!=", 1)
                op = "!="
            elif "==" in part:
                k, v = part.split("==", 1)
                op = "="
            elif "=" in part:
                k, v = part.split("=", 1)
                op = "="
            else:
                raise ValueError(f"invalid field selector requirement {part!r}")
            self.reqs.append((k.strip(), op, v.strip()))
        self.matches: Matcher = self._compile()

    def _compile(self) -> Matcher:
        # group by path: one lookup per distinct field, then set membership tests
        by_path: dict[str, tuple[set, set]] = {}
        for k, op, v in self.reqs:
            eq, ne = by_path.setdefault(k, (set(), set()))
            (eq if op == "=" else ne).add(v)
        checks = [(_getter(k), frozenset(eq), frozenset(ne)) for k, (eq, ne) in by_path.items()]
        if not checks:
            return lambda obj: True

        def matches(obj: dict) -> bool:
            for get, eq, ne in checks:
                v = get(obj)
                if v in ne or (eq and (len(eq) > 1 or v not in eq)):
                    return False
            return True
        return matches

    def __bool__(self) -> bool:
        return bool(self.reqs)

    def __repr__(self) -> str:
        return f"FieldSelector({self.text!r})"


def parse(text: Optional[str]) -> Optional[FieldSelector]:
    if not text:
        return None
    sel = FieldSelector(text)
    return sel if sel else None


def filter_event(sel: FieldSelector, typ: str, obj: dict, old: Optional[dict]) -> Optional[tuple[str, dict]]:
    """Watch event as seen through a field selector (apiserver watch filtering): an object
    that starts matching arrives as ADDED, one that stops matching as DELETED (with its new
    state); events of objects matching neither before nor after are dropped."""
    m = sel.matches
    if typ == "ADDED" or typ == "DELETED":
        return (typ, obj) if m(obj) else None
    if typ != "MODIFIED":
        return typ, obj
    now = m(obj)
    before = old is not None and m(old)
    if now and before:
        return "MODIFIED", obj
    if now:
        return "ADDED", obj
    if before:
        return "DELETED", obj
    return None
