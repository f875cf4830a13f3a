"""Tiny thread-safe metrics registry with Prometheus text exposition (counters + summary
quantiles).  The reference has no metrics at all."""
from __future__ import annotations

import collections
import threading


class Metrics:
    def __init__(self, prefix: str, window: int = 2048):
        self.prefix = prefix
        self._c: dict[str, float] = collections.defaultdict(float)
        self._o: dict[str, collections.deque] = collections.defaultdict(lambda: collections.deque(maxlen=window))
        self._lock = threading.Lock()

    def inc(self, name: str, v: float = 1.0) -> None:
        with self._lock:
            self._c[name] += v

    def set(self, name: str, v: float) -> None:
        """Set a counter to an absolute value (mirrors a counter kept elsewhere)."""
        with self._lock:
            self._c[name] = float(v)

    def observe(self, name: str, v: float) -> None:
        with self._lock:
            self._o[name].append(float(v))

    def values(self, name: str) -> list[float]:
        with self._lock:
            return list(self._o.get(name, ()))

    def quantile(self, name: str, q: float) -> float | None:
        with self._lock:
            xs = sorted(self._o.get(name, ()))
        if not xs:
            return None
        return xs[min(len(xs) - 1, int(q * len(xs)))]

    def render(self) -> str:
        lines = []
        with self._lock:
            for k, v in sorted(self._c.items()):
                lines.append(f"# TYPE {self.prefix}_{k} counter")
                lines.append(f"{self.prefix}_{k} {v}")
            obs = {k: sorted(v) for k, v in self._o.items()}
        for k, xs in sorted(obs.items()):
            lines.append(f"# TYPE {self.prefix}_{k} summary")
            for q in (0.5, 0.9, 0.99):
                lines.append(f'{self.prefix}_{k}{{quantile="{q}"}} {xs[min(len(xs) - 1, int(q * len(xs)))]}')
            lines.append(f"{self.prefix}_{k}_count {len(xs)}")
            lines.append(f"{self.prefix}_{k}_sum {sum(xs)}")
        return "\n".join(lines) + "\n"
