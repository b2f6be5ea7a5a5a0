"""Node constraints, quorums and launch priorities of the head scaler (reference
core/_private/cluster/quorum_manager.py:29-534; ``Runtime.get_node_constraints`` /
``node_constraints_reached``).

Per WORKER NODE TYPE (not per cluster): a node type whose runtimes report node constraints
(ZooKeeper, etcd, Consul, MinIO, MongoDB, Kafka -- runtime/catalog.py QUORUM_CONSTRAINTS) and
that has ``min_workers > 0`` gets ``NodeConstraints(minimal=min_workers, quorum, scalable,
runtimes)``.  The runtime config of a node type is the cluster ``runtime`` section deep-merged
with the node type's own ``runtime`` section, so only the node types that actually run such a
runtime are constrained.

Each scaler round:

1. ``update(workers, tags, pending)`` snapshots the workers and the quorum id -> members map.
2. ``terminate_for_quorum(type, node)``: a member of a quorum that has lost its majority
   (fewer than ``minimal // 2 + 1`` members left) is terminated -- that quorum can never
   regain consensus; a new one forms from fresh nodes.
3. ``is_launch_allowed(type)`` -> (allowed, quorum id):
   * quorum types: while a quorum with a majority is running, a NON-scalable quorum (MinIO)
     launches nothing; a scalable one (ZooKeeper) launches ONE node at a time, tagged with the
     running quorum's id and ``quorum-join=init``, and nothing more until that join finished
     (and no launch of the type is pending);
   * ``options.launch_with_strong_priority`` with worker types of different
     ``launch_priority``: a type waits until every type of a LOWER priority value (launched
     first) has all its nodes up to date and none pending (e.g. storage before compute).
4. ``wait_for_update()`` -> True holds back every node update of the round while a
   constrained type has fewer than ``minimal`` nodes or nodes without an IP.  Once satisfied,
   the members are published (state-server KV ``cluster_nodes_info_<type>``) and a quorum
   type without a running quorum commits a new one (id = hash of the member set) on the
   nodes not in any quorum; the runtimes get ``node_constraints_reached(config, node_type,
   head_info, nodes_info, quorum_id)`` whenever the published member set changes (also for a
   joining node of a running quorum).
5. ``on_update_done(node, ok)``: a joining node's ``quorum-join`` becomes success / failed.
"""
from __future__ import annotations

import copy
import hashlib
import json
import logging
from typing import Any, Dict, List, NamedTuple, Optional, Tuple

from cloudtik_amd.core import tags as T

logger = logging.getLogger(__name__)

NODES_INFO_KEY = "cluster_nodes_info_{}"
NODES_INFO_NAMESPACE = "cluster"


class NodeConstraints(NamedTuple):
    minimal: int
    quorum: bool
    scalable: bool
    runtimes: List[str]


def _merge(a, b):
    out = copy.deepcopy(a)
    for k, v in (b or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def node_type_runtime_config(config: Dict[str, Any], node_type: str) -> Dict[str, Any]:
    """Cluster runtime config merged with the node type's own ``runtime`` section
    (reference utils.py:1234 _get_node_type_specific_runtime_config)."""
    nt = (config.get("available_node_types") or {}).get(node_type) or {}
    return _merge(config.get("runtime") or {}, nt.get("runtime") or {})


def node_constraints_for_node_type(config: Dict[str, Any], node_type: str) -> Optional[NodeConstraints]:
    from cloudtik_amd.core import runtime_factory as rf
    rc = node_type_runtime_config(config, node_type)
    runtimes, quorum, scalable = [], False, False
    for t in rc.get("types") or []:
        try:
            rt = rf.get_runtime(t, rc.get(t, {}) or {})
            c = _constraints_of(rt, config, node_type)
        except Exception:  # noqa: BLE001 - unknown runtime types are validated elsewhere
            continue
        if c is None:
            continue
        needs_minimal, q, s = c
        if needs_minimal:
            runtimes.append(t)
            if q:
                quorum = True
                scalable = scalable or bool(s)
    if not runtimes:
        return None
    minimal = int(((config.get("available_node_types") or {}).get(node_type) or {}).get("min_workers", 0) or 0)
    return NodeConstraints(minimal, quorum, scalable, runtimes) if minimal > 0 else None


def _constraints_of(rt, config, node_type):
    try:
        return rt.get_node_constraints(config, node_type)
    except TypeError:                       # runtimes with the one-argument form
        return rt.get_node_constraints(config)


def quorum_minimal_nodes(config: Dict[str, Any]) -> int:
    """Largest minimal node count over the constrained worker node types (0: none)."""
    out = 0
    for nt in config.get("available_node_types") or {}:
        if nt == config.get("head_node_type"):
            continue
        c = node_constraints_for_node_type(config, nt)
        if c is not None:
            out = max(out, c.minimal)
    return out


def _hash(s: str) -> str:
    return hashlib.sha1(s.encode()).hexdigest()[:16]


class QuorumManager:
    def __init__(self, config: Dict[str, Any], provider, state_client=None):
        self.provider = provider
        self.state = state_client
        self.published_hashes: Dict[str, str] = {}
        self.notifications: List[Dict[str, Any]] = []      # what the runtimes were told (status/tests)
        self.workers: List[str] = []
        self.tags: Dict[str, Dict[str, str]] = {}
        self.pending: Dict[str, int] = {}
        self.quorums: Dict[str, Dict[str, set]] = {}       # node type -> quorum id -> members
        self.nodes_info: Dict[str, Dict[str, Dict[str, Any]]] = {}
        self.reset(config)

    # ------------------------------------------------------------------ config
    def reset(self, config: Dict[str, Any], provider=None):
        self.config = config
        if provider is not None:
            self.provider = provider
        head = config.get("head_node_type")
        types = config.get("available_node_types") or {}
        self.constraints: Dict[str, NodeConstraints] = {}
        for nt in types:
            if nt == head:
                continue
            c = node_constraints_for_node_type(config, nt)
            if c is not None:
                self.constraints[nt] = c
        prios = {nt: int(v.get("launch_priority", 0) or 0) for nt, v in types.items() if nt != head}
        opts = config.get("options") or {}
        self.strong_priority = bool(opts.get("launch_with_strong_priority", config.get("launch_with_strong_priority")))
        if self.strong_priority and not (len(prios) > 1 and len(set(prios.values())) > 1):
            self.strong_priority = False
        self.launch_priority = prios

    @property
    def enabled(self) -> bool:
        return bool(self.constraints)

    # ------------------------------------------------------------------ per round
    def update(self, workers: List[str], tags: Dict[str, Dict[str, str]], pending: Optional[Dict[str, int]] = None):
        self.workers = list(workers)
        self.tags = {n: dict(tags.get(n) or self.provider.node_tags(n)) for n in workers}
        self.pending = dict(pending or {})
        self.quorums = {}
        for n in self.workers:
            t = self.tags[n]
            nt, qid = t.get(T.CLOUDTIK_TAG_USER_NODE_TYPE), t.get(T.CLOUDTIK_TAG_QUORUM_ID)
            if nt in self.constraints and qid:
                self.quorums.setdefault(nt, {}).setdefault(qid, set()).add(n)
        self._collect_nodes_info()

    def _collect_nodes_info(self):
        self.nodes_info = {}
        for n in self.workers:
            t = self.tags[n]
            nt = t.get(T.CLOUDTIK_TAG_USER_NODE_TYPE)
            if not nt or (nt not in self.constraints and not self.strong_priority):
                continue
            info: Dict[str, Any] = {"node_ip": self.provider.internal_ip(n)}
            seq = t.get(T.CLOUDTIK_TAG_NODE_SEQ_ID)
            if seq and str(seq).isdigit():
                info["node_seq_id"] = int(seq)
            for key, tag in (("node_status", T.CLOUDTIK_TAG_NODE_STATUS), ("quorum_id", T.CLOUDTIK_TAG_QUORUM_ID),
                             ("quorum_join", T.CLOUDTIK_TAG_QUORUM_JOIN)):
                if tag in t:
                    info[key] = t[tag]
            self.nodes_info.setdefault(nt, {})[n] = info

    def remove_terminating(self, nodes: List[str]):
        for n in nodes:
            for q in self.quorums.values():
                for members in q.values():
                    members.discard(n)
            for infos in self.nodes_info.values():
                infos.pop(n, None)
        self.workers = [n for n in self.workers if n not in set(nodes)]

    # ------------------------------------------------------------------ quorum arithmetic
    def majority(self, node_type: str) -> int:
        return self.constraints[node_type].minimal // 2 + 1

    def running_quorum(self, node_type: str) -> Optional[str]:
        """A quorum id of this type that still has a majority of its minimal membership."""
        if node_type not in self.constraints:
            return None
        need = self.majority(node_type)
        for qid, members in sorted((self.quorums.get(node_type) or {}).items()):
            if len(members) >= need:
                return qid
        return None

    def join_in_progress(self, node_type: str) -> Optional[Tuple[str, Dict[str, Any]]]:
        for n, info in sorted((self.nodes_info.get(node_type) or {}).items()):
            if info.get("quorum_join") == T.QUORUM_JOIN_STATUS_INIT:
                return n, info
        return None

    def terminate_for_quorum(self, node_type: str, node_id: str) -> bool:
        c = self.constraints.get(node_type)
        if c is None or not c.quorum:
            return False
        for members in (self.quorums.get(node_type) or {}).values():
            if node_id in members:
                return len(members) < self.majority(node_type)
        return False

    # ------------------------------------------------------------------ launches
    def is_launch_allowed(self, node_type: str) -> Tuple[bool, Optional[str]]:
        c = self.constraints.get(node_type)
        if c is not None and c.quorum:
            qid = self.running_quorum(node_type)
            if qid is None:
                return True, None
            if not c.scalable:
                return False, None
            if self.pending.get(node_type, 0) > 0 or self.join_in_progress(node_type) is not None:
                logger.info("quorum join of %s in progress: pausing its launches", node_type)
                return False, None
            return True, qid
        if self.strong_priority:
            mine = self.launch_priority.get(node_type, 0)
            for other, p in self.launch_priority.items():
                if p < mine and not self._all_up_to_date(other):
                    logger.info("launch of %s waits for %s (lower launch_priority value) to be up to date",
                                node_type, other)
                    return False, None
        return True, None

    def _all_up_to_date(self, node_type: str) -> bool:
        if self.pending.get(node_type, 0) > 0:
            return False
        return all(info.get("node_status") == T.STATUS_UP_TO_DATE
                   for info in (self.nodes_info.get(node_type) or {}).values())

    def launch_tags(self, quorum_id: Optional[str]) -> Dict[str, str]:
        return {T.CLOUDTIK_TAG_QUORUM_ID: quorum_id, T.CLOUDTIK_TAG_QUORUM_JOIN: T.QUORUM_JOIN_STATUS_INIT} \
            if quorum_id else {}

    # ------------------------------------------------------------------ updates
    def wait_for_update(self) -> bool:
        """True: hold back node updates this round (a constrained type is not complete)."""
        for nt, c in sorted(self.constraints.items()):
            infos = self.nodes_info.get(nt) or {}
            if c.quorum:
                qid = self.running_quorum(nt)
                if qid is not None:
                    if not c.scalable:
                        continue
                    joining = self.join_in_progress(nt)
                    if joining is None:
                        continue
                    if joining[1].get("node_ip") is None:
                        logger.info("waiting for the IP of joining node %s", joining[0])
                        return True
                    members = {n: infos[n] for n in self.quorums[nt][qid] if n in infos}
                    self._publish(nt, members, c, qid)
                    continue
            if len(infos) < c.minimal:
                logger.info("waiting for the minimal %d nodes of %s (have %d) required by %s", c.minimal, nt,
                            len(infos), c.runtimes)
                return True
            if any(i.get("node_ip") is None for i in infos.values()):
                logger.info("waiting for the IPs of the %s nodes", nt)
                return True
            self._publish(nt, infos, c, None)
        return False

    def _publish(self, node_type: str, infos: Dict[str, Dict[str, Any]], c: NodeConstraints,
                 quorum_id: Optional[str]):
        members = infos
        if quorum_id is None and c.quorum:
            fresh = {n: i for n, i in infos.items() if not i.get("quorum_id")}
            if len(fresh) < self.majority(node_type):
                logger.warning("cannot form a new quorum of %s: %d nodes outside a quorum, %d needed", node_type,
                               len(fresh), self.majority(node_type))
                return False
            members = fresh
            quorum_id = _hash(json.dumps(sorted(fresh), sort_keys=True))
            for n in fresh:
                self.provider.set_node_tags(n, {T.CLOUDTIK_TAG_QUORUM_ID: quorum_id})
                fresh[n]["quorum_id"] = quorum_id
                self.tags.setdefault(n, {})[T.CLOUDTIK_TAG_QUORUM_ID] = quorum_id
                self.quorums.setdefault(node_type, {}).setdefault(quorum_id, set()).add(n)
            logger.info("committed quorum %s of %s with %d nodes", quorum_id, node_type, len(fresh))
        data = json.dumps(members, sort_keys=True)
        h = _hash(data)
        if self.published_hashes.get(node_type) == h:
            return False
        self.published_hashes[node_type] = h
        if self.state is not None:
            try:
                self.state.kv_put(NODES_INFO_KEY.format(node_type), data, namespace=NODES_INFO_NAMESPACE)
            except Exception as e:  # noqa: BLE001 - the notification below still happens
                logger.warning("could not publish nodes info of %s: %s", node_type, e)
        self._notify(node_type, members, c, quorum_id)
        return True

    def _notify(self, node_type, members, c: NodeConstraints, quorum_id):
        from cloudtik_amd.core import runtime_factory as rf
        from cloudtik_amd.core.cluster_utils import get_head_node
        head = get_head_node(self.provider, self.config["cluster_name"])
        head_info = {"node_id": head, "node_ip": self.provider.internal_ip(head) if head else None,
                     "node_seq_id": T.CLOUDTIK_TAG_HEAD_NODE_SEQ_ID}
        rc = node_type_runtime_config(self.config, node_type)
        self.notifications.append({"node_type": node_type, "quorum_id": quorum_id, "members": sorted(members),
                                   "runtimes": list(c.runtimes)})
        for t in c.runtimes:
            try:
                rf.get_runtime(t, rc.get(t, {}) or {}).node_constraints_reached(
                    self.config, node_type, head_info, members, quorum_id=quorum_id)
            except Exception:  # noqa: BLE001 - one runtime's hook never stops the scaler
                logger.exception("runtime %s: node_constraints_reached failed", t)

    def on_update_done(self, node_id: str, success: bool):
        t = self.provider.node_tags(node_id)
        if t.get(T.CLOUDTIK_TAG_QUORUM_JOIN) == T.QUORUM_JOIN_STATUS_INIT:
            self.provider.set_node_tags(node_id, {T.CLOUDTIK_TAG_QUORUM_JOIN: T.QUORUM_JOIN_STATUS_SUCCESS
                                                  if success else T.QUORUM_JOIN_STATUS_FAILED})
