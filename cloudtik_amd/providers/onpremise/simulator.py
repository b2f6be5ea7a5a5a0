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
``{"error": ...}``; methods mirror the NodeProvider interface, plus pool management
(reference cloudtik_cloud_simulator.py:196-227, cloud_simulator_scheduler.py:146-158):
``reload`` re-reads the pool file (new hosts become free, removed free hosts leave, removed
allocated hosts drain -- they leave the pool when their cluster releases them), ``shutdown``
stops the service, and ``create_workspace`` / ``delete_workspace`` / ``get_workspace`` /
``list_workspaces`` keep the workspaces of the pool (the on-premise workspace provider).

The running service records its address in a process file (``~/.cloudtik/onpremise/
cloud-simulator.json``); providers and ``cloudtik-simulator --reload/--shutdown`` without an
explicit address discover it there (reference onpremise/config.py:20-50).

    cloudtik-simulator pool.yaml [--bind-address A] [--port 8282]   # serve
    cloudtik-simulator pool.yaml --reload | --shutdown               # control a running one
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import socket
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional

import yaml

from cloudtik_amd.core.state.file_state_store import FileStateStore

logger = logging.getLogger(__name__)


DEFAULT_PORT = 8282


def process_file() -> str:
    return os.path.expanduser(os.environ.get("CLOUDTIK_SIMULATOR_PROCESS_FILE",
                                             "~/.cloudtik/onpremise/cloud-simulator.json"))


def discover_simulator() -> Optional[str]:
    """host:port of the simulator running on this machine (from its process file)."""
    try:
        with open(process_file()) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    host, port = rec.get("bind_address"), rec.get("port")
    if not host or not port:
        return None
    if host in ("0.0.0.0", "::", ""):
        try:
            host = socket.gethostbyname(socket.gethostname())
        except OSError:
            host = "127.0.0.1"
    return f"{host}:{port}"


def simulator_address(configured: Optional[str]) -> str:
    addr = configured or discover_simulator()
    if not addr:
        raise ValueError("no cloud simulator address: set provider.cloud_simulator_address or start "
                         "cloudtik-simulator on this machine")
    return addr if ":" in addr.rsplit("]", 1)[-1] else f"{addr}:{DEFAULT_PORT}"


def load_pool(pool_file: str) -> Dict[str, Any]:
    """The pool file: ``instance_types`` + ``nodes``, or the reference's on-premise provider
    section format (``provider: {instance_types: ..., nodes: ...}``)."""
    with open(pool_file) as f:
        pool = yaml.safe_load(f) or {}
    return pool.get("provider", pool)


class PoolScheduler:
    def __init__(self, pool: Dict[str, Any], state_file: str, pool_file: Optional[str] = None):
        self.store = FileStateStore(state_file)
        self.lock = threading.RLock()
        self.pool_file = pool_file
        self._apply_pool(pool)

    def _apply_pool(self, pool: Dict[str, Any]) -> Dict[str, List[str]]:
        self.instance_types = pool.get("instance_types", {}) or {}
        want = {n["ip"]: n for n in pool.get("nodes", []) or []}
        added, removed, draining = [], [], []
        with self.lock, self.store.transaction() as st:
            nodes = st.setdefault("nodes", {})
            st.setdefault("workspaces", {})
            for ip, n in want.items():
                if ip not in nodes:
                    added.append(ip)
                cur = nodes.setdefault(ip, {"ip": ip, "state": "free", "cluster": None, "tags": {}})
                cur["instance_type"] = n.get("instance_type", "default")
                cur["external_ip"] = n.get("external_ip", ip)
                cur.pop("draining", None)
            for ip in [ip for ip in nodes if ip not in want]:
                if nodes[ip]["state"] == "free":
                    del nodes[ip]
                    removed.append(ip)
                else:
                    nodes[ip]["draining"] = True     # leaves the pool once its cluster releases it
                    draining.append(ip)
        return {"added": sorted(added), "removed": sorted(removed), "draining": sorted(draining)}

    def reload(self, pool_file: Optional[str] = None, pool: Optional[Dict[str, Any]] = None):
        """Apply a changed pool without restarting the service."""
        if pool is None:
            pool_file = pool_file or self.pool_file
            if not pool_file:
                raise ValueError("no pool file to reload")
            pool = load_pool(pool_file)
            self.pool_file = pool_file
        out = self._apply_pool(pool)
        logger.info("pool reloaded: %s", out)
        return out

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
                    if n["state"] == "free" and not n.get("draining")
                    and (itype is None or n["instance_type"] == itype)]
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
                if n.get("draining"):
                    del st["nodes"][node_id]        # removed from the pool by a reload
                else:
                    n.update(state="free", cluster=None, tags={})

    def terminate_nodes(self, node_ids: List[str]):
        for n in node_ids:
            self.terminate_node(n)

    def pool_status(self):
        nodes = self.store.get_nodes()
        return {"total": len(nodes), "free": sum(n["state"] == "free" and not n.get("draining")
                                                 for n in nodes.values()),
                "draining": sorted(ip for ip, n in nodes.items() if n.get("draining")),
                "clusters": sorted({n["cluster"] for n in nodes.values() if n["cluster"]}),
                "workspaces": sorted(self.store.get().get("workspaces", {}))}

    # ------------------------------------------------------------------ workspaces
    def create_workspace(self, workspace_name: str):
        with self.lock, self.store.transaction() as st:
            ws = st.setdefault("workspaces", {})
            if workspace_name in ws:
                raise RuntimeError(f"workspace {workspace_name} already exists")
            ws[workspace_name] = {"name": workspace_name}
        return {"name": workspace_name}

    def delete_workspace(self, workspace_name: str):
        from cloudtik_amd.core import tags as T
        with self.lock, self.store.transaction() as st:
            ws = st.setdefault("workspaces", {})
            if workspace_name not in ws:
                raise RuntimeError(f"workspace {workspace_name} does not exist")
            busy = sorted({n["cluster"] for n in st["nodes"].values() if n["state"] == "allocated"
                           and n["tags"].get(T.CLOUDTIK_TAG_WORKSPACE_NAME) == workspace_name})
            if busy:
                raise RuntimeError(f"workspace {workspace_name} still has running clusters: {busy}")
            del ws[workspace_name]
        return {"name": workspace_name}

    def get_workspace(self, workspace_name: str):
        return self.store.get().get("workspaces", {}).get(workspace_name)

    def list_workspaces(self):
        return sorted(self.store.get().get("workspaces", {}))


def make_handler(sched: PoolScheduler, server_ref: Optional[Dict[str, Any]] = None):
    server_ref = server_ref if server_ref is not None else {}

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
                if method == "shutdown":
                    srv = server_ref.get("server")
                    if srv is None:
                        raise RuntimeError("shutdown is not available")
                    logger.info("cloud simulator shutting down on request")
                    threading.Thread(target=shutdown_server, args=(srv,), daemon=True).start()
                    res, code = {"result": "shutting down"}, 200
                else:
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


def shutdown_server(srv):
    srv.shutdown()
    srv.server_close()
    try:
        with open(process_file()) as f:
            rec = json.load(f)
        if rec.get("pid") == os.getpid():
            os.remove(process_file())
    except (OSError, ValueError):
        pass


def serve(pool_file: str, host: str = "0.0.0.0", port: int = DEFAULT_PORT, state_file: str = None,
          record: bool = True):
    pool = load_pool(pool_file)
    state_file = state_file or os.path.expanduser("~/.cloudtik/onpremise/simulator-state.json")
    ref: Dict[str, Any] = {}
    srv = ThreadingHTTPServer((host, port), make_handler(PoolScheduler(pool, state_file, pool_file), ref))
    ref["server"] = srv
    if record:
        path = process_file()
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump({"pid": os.getpid(), "bind_address": srv.server_address[0], "port": srv.server_address[1],
                       "pool_file": os.path.abspath(pool_file)}, f)
    return srv


def request(address: Optional[str], method: str, **params):
    from cloudtik_amd.providers.onpremise.node_provider import SimulatorClient
    return SimulatorClient(simulator_address(address)).call(method, **params)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="cloudtik-simulator")
    ap.add_argument("config", nargs="?", help="pool YAML (instance_types + nodes)")
    ap.add_argument("--pool", default=None, help="pool YAML (alias of the positional argument)")
    ap.add_argument("--bind-address", "--bind", dest="bind", default=None)
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--state-file", default=None)
    ap.add_argument("--reload", action="store_true", help="ask the running simulator to re-read its pool")
    ap.add_argument("--shutdown", action="store_true", help="ask the running simulator to stop")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    pool_file = a.config or a.pool
    if a.reload and a.shutdown:
        ap.error("only one of --reload / --shutdown")
    if a.reload or a.shutdown:
        addr = f"{a.bind}:{a.port or DEFAULT_PORT}" if a.bind else None
        if a.reload:
            print(json.dumps(request(addr, "reload", pool_file=os.path.abspath(pool_file) if pool_file else None)))
        else:
            print(request(addr, "shutdown"))
        return
    if not pool_file:
        ap.error("a pool file is required to start the simulator")
    srv = serve(pool_file, a.bind or "0.0.0.0", a.port or DEFAULT_PORT, a.state_file)
    logger.info("cloud simulator on %s:%d", *srv.server_address[:2])
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass


if __name__ == "__main__":
    main()
