"""Event summarizer (reference core/_private/cluster/event_summarizer.py:6): the scaler emits
many near-identical messages per iteration ("Adding 1 node(s) of type gpu" x N); this
aggregates them into one line per template per cycle and rate-limits repeated warnings."""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional


class EventSummarizer:
    def __init__(self):
        self.events_by_key: Dict[str, int] = {}
        self.messages_to_send: List[str] = []
        self.throttled_messages: Dict[str, float] = {}

    def add(self, template: str, *, quantity: int, aggregate: Callable[[int, int], int] = lambda a, b: a + b):
        """template contains "{}" for the quantity, e.g. "Adding {} node(s) of type gpu"."""
        self.events_by_key[template] = aggregate(self.events_by_key.get(template, 0), quantity) \
            if template in self.events_by_key else quantity

    def add_once_per_interval(self, message: str, key: str, interval_s: float, now: Optional[float] = None):
        now = time.time() if now is None else now
        if now >= self.throttled_messages.get(key, 0.0):
            self.throttled_messages[key] = now + interval_s
            self.messages_to_send.append(message)

    def summary(self) -> List[str]:
        out = [t.format(q) for t, q in self.events_by_key.items()] + list(self.messages_to_send)
        return out

    def clear(self):
        self.events_by_key.clear()
        self.messages_to_send.clear()
