"""Locked JSON file store for node state of the local / virtual / on-premise schedulers
(reference core/_private/state/file_state_store.py:11-148): nodes, their tags and
running/terminated state survive CLI invocations and are shared between processes with
an advisory file lock."""
from __future__ import annotations

import json
import os
import threading
from contextlib import contextmanager
from typing import Any, Dict

from filelock import FileLock


class FileStateStore:
    def __init__(self, path: str):
        self.path = os.path.expanduser(path)
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        self._flock = FileLock(self.path + ".lock")
        self._tlock = threading.RLock()
        if not os.path.exists(self.path):
            with self.transaction() as st:
                st.setdefault("nodes", {})

    def _read(self) -> Dict[str, Any]:
        try:
            with open(self.path) as f:
                return json.load(f)
        except (OSError, ValueError):
            return {"nodes": {}}

    def _write(self, state: Dict[str, Any]):
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(state, f, indent=1, sort_keys=True)
        os.replace(tmp, self.path)

    @contextmanager
    def transaction(self):
        with self._tlock, self._flock:
            st = self._read()
            yield st
            self._write(st)

    def get(self) -> Dict[str, Any]:
        with self._tlock, self._flock:
            return self._read()

    # convenience node API
    def get_nodes(self) -> Dict[str, Any]:
        return self.get().get("nodes", {})

    def get_node(self, node_id: str):
        return self.get_nodes().get(node_id)

    def put_node(self, node_id: str, node: Dict[str, Any]):
        with self.transaction() as st:
            st.setdefault("nodes", {})[node_id] = node

    def update_node_tags(self, node_id: str, tags: Dict[str, str]):
        with self.transaction() as st:
            n = st["nodes"][node_id]
            n.setdefault("tags", {}).update(tags)

    def delete_node(self, node_id: str):
        with self.transaction() as st:
            st.get("nodes", {}).pop(node_id, None)
