"""Cluster-creation event callbacks (reference core/_private/event_system.py:8-144, exposed
through ``Cluster.register_callback``).

Handlers are registered per event (optionally per cluster name) and called with an
event-data dict (``cluster_name``, ``node_id``, ``command``...).  A failing handler is
logged and never aborts the cluster operation.
"""
from __future__ import annotations

import enum
import logging
import threading
from typing import Any, Callable, Dict, List, Optional, Tuple

logger = logging.getLogger(__name__)


class CreateClusterEvent(enum.Enum):
    up_started = "up_started"
    acquiring_new_head_node = "acquiring_new_head_node"
    head_node_acquired = "head_node_acquired"
    ssh_control_acquired = "ssh_control_acquired"
    run_initialization_cmd = "run_initialization_cmd"
    run_setup_cmd = "run_setup_cmd"
    start_cloudtik_runtime = "start_cloudtik_runtime"
    cluster_booting_completed = "cluster_booting_completed"
    cluster_booting_failed = "cluster_booting_failed"


class _EventSystem:
    def __init__(self):
        self._lock = threading.Lock()
        self._handlers: Dict[CreateClusterEvent, List[Tuple[Optional[str], Callable]]] = {}

    def add_callback_handler(self, event: CreateClusterEvent, callback: Callable[[Dict[str, Any]], None],
                             cluster_name: Optional[str] = None):
        if not callable(callback):
            raise TypeError("callback must be callable")
        with self._lock:
            self._handlers.setdefault(event, []).append((cluster_name, callback))

    def execute_callback(self, event: CreateClusterEvent, event_data: Optional[Dict[str, Any]] = None):
        data = dict(event_data or {})
        data.setdefault("event_name", event)
        cluster = data.get("cluster_name")
        with self._lock:
            handlers = [cb for (c, cb) in self._handlers.get(event, []) if c is None or c == cluster]
        for cb in handlers:
            try:
                cb(data)
            except Exception:  # noqa: BLE001
                logger.exception("event handler for %s failed", event.value)

    def clear_callbacks_for_event(self, event: CreateClusterEvent):
        with self._lock:
            self._handlers.pop(event, None)

    def clear_callbacks_for_cluster(self, cluster_name: str):
        with self._lock:
            for ev in list(self._handlers):
                self._handlers[ev] = [(c, cb) for (c, cb) in self._handlers[ev] if c != cluster_name]


global_event_system = _EventSystem()
