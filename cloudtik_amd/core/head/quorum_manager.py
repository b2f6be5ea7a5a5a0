"""Quorum constraints for runtimes that need a minimal node set before any member is set
up (ZooKeeper, etcd, Consul, MinIO, MongoDB, Kafka; reference
core/_private/cluster/quorum_manager.py:29-534 and ``Runtime.get_node_constraints``).

Until ``minimal`` workers have been launched, the scaler launches but does not set up
workers of such a cluster (every member must know the full initial membership when its
service is configured).  Once enough exist, the first ``minimal`` get one quorum id and
``join=init`` tags and are set up together; when they are up they are marked
``join=success`` and later nodes join the existing quorum directly.  A member that fails
setup marks the quorum attempt failed so a fresh quorum can form.
"""
from __future__ import annotations

import uuid
from typing import Any, Dict, List, Optional

from cloudtik_amd.core import tags as T


def quorum_minimal_nodes(config: Dict[str, Any]) -> int:
    from cloudtik_amd.core import runtime_factory as rf
    from cloudtik_amd.core.cluster_config import get_runtime_types
    minimal = 0
    for t in get_runtime_types(config):
        rc = config.get("runtime", {}).get(t, {}) or {}
        rt = rf.get_runtime(t, rc)
        if rt.get_node_constraints(config) is not None:
            minimal = max(minimal, int(rc.get("minimal_nodes", 3)))
    return minimal


class QuorumManager:
    def __init__(self, config: Dict[str, Any], provider):
        self.provider = provider
        self.reset(config)

    def reset(self, config):
        self.config = config
        self.minimal = quorum_minimal_nodes(config)

    @property
    def enabled(self) -> bool:
        return self.minimal > 0

    def _formed(self, workers) -> Optional[str]:
        for w in workers:
            t = self.provider.node_tags(w)
            if t.get(T.CLOUDTIK_TAG_QUORUM_JOIN) == T.QUORUM_JOIN_STATUS_SUCCESS:
                return t.get(T.CLOUDTIK_TAG_QUORUM_ID)
        return None

    def updatable(self, workers: List[str]) -> List[str]:
        """Workers the scaler may start setting up now."""
        if not self.enabled:
            return list(workers)
        qid = self._formed(workers)
        if qid is not None:
            for w in workers:                      # late joiners of a formed quorum
                t = self.provider.node_tags(w)
                if not t.get(T.CLOUDTIK_TAG_QUORUM_ID):
                    self.provider.set_node_tags(w, {T.CLOUDTIK_TAG_QUORUM_ID: qid,
                                                    T.CLOUDTIK_TAG_QUORUM_JOIN: T.QUORUM_JOIN_STATUS_INIT})
            return list(workers)
        pending = [w for w in workers if self.provider.node_tags(w).get(T.CLOUDTIK_TAG_QUORUM_JOIN)
                   == T.QUORUM_JOIN_STATUS_INIT]
        if pending:
            return pending
        if len(workers) < self.minimal:
            return []                              # wait for the minimal membership
        qid = uuid.uuid4().hex[:12]
        members = sorted(workers, key=lambda w: int(self.provider.node_tags(w).get(T.CLOUDTIK_TAG_NODE_SEQ_ID, 0)
                                                    or 0))[:self.minimal]
        for w in members:
            self.provider.set_node_tags(w, {T.CLOUDTIK_TAG_QUORUM_ID: qid,
                                            T.CLOUDTIK_TAG_QUORUM_JOIN: T.QUORUM_JOIN_STATUS_INIT})
        return members

    def on_update_done(self, node_id: str, success: bool):
        if not self.enabled:
            return
        t = self.provider.node_tags(node_id)
        if t.get(T.CLOUDTIK_TAG_QUORUM_JOIN) == T.QUORUM_JOIN_STATUS_INIT:
            self.provider.set_node_tags(node_id, {T.CLOUDTIK_TAG_QUORUM_JOIN: T.QUORUM_JOIN_STATUS_SUCCESS if success
                                                  else T.QUORUM_JOIN_STATUS_FAILED})
