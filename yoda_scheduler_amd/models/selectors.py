"""metav1.LabelSelector matching (matchLabels + matchExpressions)."""
from __future__ import annotations

import re
from typing import Mapping, Optional

_GO_INT = re.compile(r"[+-]?[0-9]+\Z")   # strconv.ParseInt(s, 10, 64) syntax


class LabelSelector:
    __slots__ = ("labels", "exprs", "empty", "nothing")

    def __init__(self, sel: Optional[dict]) -> None:
        # nil selector matches nothing; {} matches everything (upstream semantics)
        self.nothing = sel is None
        sel = sel or {}
        self.labels = dict(sel.get("matchLabels") or {})
        self.exprs = [(e.get("key", ""), e.get("operator", "In"), set(str(v) for v in e.get("values") or []))
                      for e in sel.get("matchExpressions") or []]
        self.empty = not self.labels and not self.exprs

    def native(self, namespaces=None) -> tuple:
        """The selector (+ the namespaces it applies in, None = all) as a native ``MatchTerm``
        (``core.Lane.count_matching`` / lane gate terms)."""
        return (None if namespaces is None else tuple(namespaces), self.nothing, tuple(self.labels.items()),
                tuple((k, op, tuple(sorted(vals))) for k, op, vals in self.exprs))

    def native_query(self, namespaces=None) -> list:
        return [self.native(namespaces)]

    def matches(self, labels: Optional[Mapping[str, str]]) -> bool:
        if self.nothing:
            return False
        labels = labels or {}
        for k, v in self.labels.items():
            if labels.get(k) != v:
                return False
        for k, op, vals in self.exprs:
            has = k in labels
            if op == "In":
                if not has or labels[k] not in vals:
                    return False
            elif op == "NotIn":
                if has and labels[k] in vals:
                    return False
            elif op == "Exists":
                if not has:
                    return False
            elif op == "DoesNotExist":
                if has:
                    return False
            else:
                raise ValueError(f"unknown selector operator {op!r}")
        return True


class NodeSelector:
    """core/v1 NodeSelector (``nodeSelectorTerms`` OR'ed, expressions AND'ed), as used by
    PV ``spec.nodeAffinity.required``. Operators In/NotIn/Exists/DoesNotExist/Gt/Lt on
    labels and ``matchFields`` on ``metadata.name``. A term with no requirements matches
    nothing (upstream)."""
    __slots__ = ("terms",)

    def __init__(self, sel: Optional[dict]) -> None:
        self.terms = []
        for t in (sel or {}).get("nodeSelectorTerms") or []:
            exprs = [(e.get("key", ""), e.get("operator", "In"), [str(v) for v in e.get("values") or []])
                     for e in t.get("matchExpressions") or []]
            fields = [(e.get("key", ""), e.get("operator", "In"), [str(v) for v in e.get("values") or []])
                      for e in t.get("matchFields") or []]
            self.terms.append((exprs, fields))

    @staticmethod
    def _req(op: str, has: bool, val: str, vals: list) -> bool:
        if op == "In":
            return has and val in vals
        if op == "NotIn":
            return not has or val not in vals
        if op == "Exists":
            return has
        if op == "DoesNotExist":
            return not has
        if op in ("Gt", "Lt"):
            # upstream parses both sides with strconv.ParseInt: no spaces or '_' (Python's int takes them)
            if not has or len(vals) != 1 or not _GO_INT.match(val) or not _GO_INT.match(vals[0]):
                return False
            a, b = int(val), int(vals[0])
            return a > b if op == "Gt" else a < b
        raise ValueError(f"unknown node selector operator {op!r}")

    def matches(self, node_name: str, labels: Optional[Mapping[str, str]]) -> bool:
        labels = labels or {}
        for exprs, fields in self.terms:
            if not exprs and not fields:
                continue
            if all(self._req(op, k in labels, labels.get(k, ""), vals) for k, op, vals in exprs) and \
                    all(self._field(k, op, vals, node_name) for k, op, vals in fields):
                return True
        return False

    @staticmethod
    def _field(key: str, op: str, vals: list, node_name: str) -> bool:
        """upstream v1.20 NodeSelectorRequirementsAsFieldSelector over {metadata.name: node}: In /
        NotIn with exactly one value (anything else errors, failing the term); an unknown field
        reads as ""."""
        if op not in ("In", "NotIn") or len(vals) != 1:
            return False
        eq = vals[0] == (node_name if key == "metadata.name" else "")
        return eq if op == "In" else not eq
