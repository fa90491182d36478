"""klog-compatible logging: ``--v=N`` verbosity gates V(N) lines (the reference logs
every Filter call at V(3), ``pkg/yoda/scheduler.go:77``, and every normalized score at
Info, ``:154`` — here both are V(4)+ so production verbosity stays cheap)."""
from __future__ import annotations

import logging
import sys

_verbosity = 0


def set_verbosity(v: int) -> None:
    global _verbosity
    _verbosity = int(v)


def V(level: int) -> bool:
    return _verbosity >= level


def setup(v: int = 0, stream=sys.stderr) -> None:
    set_verbosity(v)
    fmt = logging.Formatter("%(levelname).1s%(asctime)s.%(msecs)03d %(process)d %(name)s] %(message)s",
                            datefmt="%m%d %H:%M:%S")
    h = logging.StreamHandler(stream)
    h.setFormatter(fmt)
    root = logging.getLogger()
    root.handlers[:] = [h]
    root.setLevel(logging.DEBUG if v >= 4 else logging.INFO)
