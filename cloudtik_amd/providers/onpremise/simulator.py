"""Cloud simulator for on-premise pools (reference providers/onpremise/service/
cloudtik_cloud_simulator.py + _private/onpremise/cloud_simulator_scheduler.py; console
entry ``cloudtik-simulator``).

One service owns the pool of physical hosts (e.g. a rack of 8 x MI355X nodes) and hands them
out to the clusters of many users, like a tiny cloud: clusters "launch" nodes of an instance
type and get free hosts of that type, with tags kept per node.  State (which host belongs
to which cluster, tags) is a locked JSON file, so the service can restart.

Pool file (YAML)::

    instance_types:
        mi355x-8gpu: {CPU: 128, GPU: 8, "accelerator_type:MI355X": 8, memory: 1500000000000}
    nodes:
        - {ip: 10.0.0.11, instance_type: mi355x-8gpu}
        - {ip: 10.0.0.12, instance_type: mi355x-8gpu}

API: ``POST /api`` with ``{"method": name, "params": {...}}`` -> ``{"result": ...}`` or
``{"error": ...}``; methods mirror the NodeProvider interface.

    python -m cloudtik_amd.providers.onpremise.simulator --pool pool.yaml --port 8282
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List

import yaml

from cloudtik_amd.core.state.file_state_store import FileStateStore

logger = logging.getLogger(__name__)


class PoolScheduler:
    def __init__(self, pool: Dict[str, Any], state_file: str):
        self.instance_types = pool.get("instance_types", {}) or {}
        self.store = FileStateStore(state_file)
        self.lock = threading.RLock()
        with self.store.transaction() as st:
            nodes = st.setdefault("nodes", {})
            for n in pool.get("nodes", []):
                ip = n["ip"]
                cur = nodes.setdefault(ip, {"ip": ip, "state": "free", "cluster": None, "tags": {}})
                cur["instance_type"] = n.get("instance_type", "default")
                cur["external_ip"] = n.get("external_ip", ip)

    # every method takes/returns JSON-able values
    def get_instance_types(self):
        return self.instance_types

    def non_terminated_nodes(self, cluster_name: str, tag_filters: Dict[str, str]) -> List[str]:
        out = []
        for ip, n in self.store.get_nodes().items():
            # cluster_name None: every cluster of the pool (workspace-wide head listing)
            if n["state"] == "allocated" and (cluster_name is None or n["cluster"] == cluster_name) and \
                    all(n["tags"].get(k) == v for k, v in (tag_filters or {}).items()):
                out.append(ip)
        return sorted(out)

    def _node(self, node_id):
        n = self.store.get_node(node_id)
        if n is None:
            raise KeyError(f"unknown node {node_id}")
        return n

    def is_running(self, node_id: str) -> bool:
        return self._node(node_id)["state"] == "allocated"

    def is_terminated(self, node_id: str) -> bool:
        return self._node(node_id)["state"] != "allocated"

    def node_tags(self, node_id: str) -> Dict[str, str]:
        return dict(self._node(node_id).get("tags", {}))

    def internal_ip(self, node_id: str) -> str:
        return self._node(node_id)["ip"]

    def external_ip(self, node_id: str) -> str:
        return self._node(node_id).get("external_ip", node_id)

    def node_info(self, node_id: str) -> Dict[str, Any]:
        n = self._node(node_id)
        return {"node_id": node_id, "instance_type": n["instance_type"], "private_ip": n["ip"],
                "public_ip": n.get("external_ip"), "instance_status": n["state"],
                "resources": self.instance_types.get(n["instance_type"], {})}

    def create_node(self, cluster_name: str, node_config: Dict[str, Any], tags: Dict[str, str], count: int):
        itype = node_config.get("instance_type")
        with self.lock, self.store.transaction() as st:
            free = [ip for ip, n in sorted(st["nodes"].items())
                    if n["state"] == "free" and (itype is None or n["instance_type"] == itype)]
            if len(free) < count:
                raise RuntimeError(f"NoAvailableHost: requested {count} x {itype}, {len(free)} free")
            for ip in free[:count]:
                st["nodes"][ip].update(state="allocated", cluster=cluster_name, tags=dict(tags))
            return free[:count]

    def set_node_tags(self, node_id: str, tags: Dict[str, str]):
        with self.store.transaction() as st:
            st["nodes"][node_id]["tags"].update(tags)

    def terminate_node(self, node_id: str):
        with self.store.transaction() as st:
            n = st["nodes"].get(node_id)
            if n:
                n.update(state="free", cluster=None, tags={})

    def terminate_nodes(self, node_ids: List[str]):
        for n in node_ids:
            self.terminate_node(n)

    def pool_status(self):
        nodes = self.store.get_nodes()
        return {"total": len(nodes), "free": sum(n["state"] == "free" for n in nodes.values()),
                "clusters": sorted({n["cluster"] for n in nodes.values() if n["cluster"]})}


def make_handler(sched: PoolScheduler):
    class Handler(BaseHTTPRequestHandler):
        def log_message(self, fmt, *args):
            logger.debug(fmt, *args)

        def do_POST(self):
            if self.path != "/api":
                self.send_error(404)
                return
            try:
                req = json.loads(self.rfile.read(int(self.headers.get("Content-Length", 0))) or b"{}")
                method = req.get("method", "")
                if method.startswith("_") or not hasattr(sched, method):
                    raise AttributeError(f"unknown method {method!r}")
                res = {"result": getattr(sched, method)(**(req.get("params") or {}))}
                code = 200
            except Exception as e:  # noqa: BLE001 -- returned to the client
                res, code = {"error": f"{type(e).__name__}: {e}"}, 400
            body = json.dumps(res).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

    return Handler


def serve(pool_file: str, host: str = "0.0.0.0", port: int = 8282, state_file: str = None):
    with open(pool_file) as f:
        pool = yaml.safe_load(f)
    state_file = state_file or os.path.expanduser("~/.cloudtik/onpremise/simulator-state.json")
    srv = ThreadingHTTPServer((host, port), make_handler(PoolScheduler(pool, state_file)))
    return srv


def main(argv=None):
    ap = argparse.ArgumentParser(prog="cloudtik-simulator")
    ap.add_argument("--pool", required=True, help="pool YAML (instance_types + nodes)")
    ap.add_argument("--bind", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8282)
    ap.add_argument("--state-file", default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    srv = serve(a.pool, a.bind, a.port, a.state_file)
    logger.info("cloud simulator on %s:%d", a.bind, a.port)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass


if __name__ == "__main__":
    main()
