"""asyncio helpers.

``wait_for``: ``asyncio.wait_for`` on Python < 3.12 loses an outer cancellation when the
inner awaitable completes in the same loop iteration (CPython gh-86296): the caller gets
the result instead of ``CancelledError`` and keeps running. A bind worker hit that during
scheduler shutdown and never exited. This version cancels the inner task from a timer
instead, so a cancellation of the caller always propagates.
"""
from __future__ import annotations

import asyncio


async def wait_for(aw, timeout: float):
    task = asyncio.ensure_future(aw)
    if timeout is None:
        return await task
    timed_out = False

    def expire() -> None:
        nonlocal timed_out
        if not task.done():
            timed_out = True
            task.cancel()

    h = asyncio.get_running_loop().call_later(max(0.0, timeout), expire)
    try:
        return await task
    except asyncio.CancelledError:
        if timed_out:
            raise asyncio.TimeoutError() from None
        raise
    finally:
        h.cancel()
