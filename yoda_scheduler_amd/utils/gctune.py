"""Garbage-collector tuning for the long-running scheduler process.

A 1000-pod burst allocates ~50 k container objects per 1000 pods; with CPython's default
thresholds (700, 10, 10) that triggers ~50 young collections and periodic full
collections that stall the event loop for 30-90 ms — the whole p99 of a burst. Like
other latency-sensitive Python servers, the scheduler freezes everything allocated at
start-up (informer caches, plugin tables) into the permanent generation and raises the
young-generation threshold; cyclic garbage is still collected, just in larger batches.
Configured with ``yodaRuntime.gcThreshold`` (``[]`` disables tuning).
"""
from __future__ import annotations

import gc

DEFAULT_THRESHOLD = (50_000, 50, 1000)


def tune(threshold=DEFAULT_THRESHOLD, freeze: bool = True) -> None:
    if not threshold:
        return
    if freeze:
        gc.collect()
        gc.freeze()
    gc.set_threshold(*threshold)
