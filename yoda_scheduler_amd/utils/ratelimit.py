"""Token-bucket rate limiter (client-go ``flowcontrol.NewTokenBucketRateLimiter``).

The reference inherits kube-scheduler's default client QPS 50 / burst 100,
which is what bounds its burst throughput to ≈50 binds/s. The limiter
here reproduces that when configured the same way; ``qps <= 0`` disables limiting.
"""
from __future__ import annotations

import asyncio
import time


class TokenBucket:
    def __init__(self, qps: float, burst: int, clock=time.monotonic) -> None:
        self.qps = float(qps)
        self.burst = max(int(burst), 1)
        self.tokens = float(self.burst)
        self.clock = clock
        self.last = clock()
        self.waited = 0.0

    @property
    def unlimited(self) -> bool:
        return self.qps <= 0

    def _refill(self) -> None:
        now = self.clock()
        self.tokens = min(self.burst, self.tokens + (now - self.last) * self.qps)
        self.last = now

    def try_acquire(self) -> bool:
        if self.unlimited:
            return True
        self._refill()
        if self.tokens >= 1.0:
            self.tokens -= 1.0
            return True
        return False

    async def acquire(self) -> None:
        if self.unlimited:
            return
        self._refill()
        self.tokens -= 1.0                 # reserve; may go negative = queue position
        if self.tokens < 0:
            delay = -self.tokens / self.qps
            self.waited += delay
            await asyncio.sleep(delay)
