"""metav1.LabelSelector matching (matchLabels + matchExpressions)."""
from __future__ import annotations

from typing import Mapping, Optional


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
