"""Control state on top of the native state server.

Parity map (reference core/_private/state/):
* ``StateClient`` namespaced KV -- control_state.py:17-151 (``@namespace_<ns>:`` key prefix)
* ``kv_*`` module functions      -- kv_store.py:10-112
* ``StateTable`` / ``NodeStateTable`` / ``StateTableStore`` -- state_table_store.py:9-52;
  tables are stored as one server-side HASH per table (one HGETALL lists a table instead of
  the reference's per-shard key scans)
* ``StateNodeManager``           -- state_node_manager.py:9-25
* ``ScalingStateClient``         -- scaling_state.py:21-119 (heartbeats from the node table,
  resource state from the node-metrics table, the scaling state written back as one key)
* ``StateServer``                -- start/stop the ``cloudtik-state-server`` process
  (what services.py does for redis-server in the reference)
"""
from __future__ import annotations

import json
import logging
import os
import subprocess
import time
from typing import Any, Dict, List, Optional

from cloudtik_amd.core.state.resp import RespConnection, RespError

logger = logging.getLogger(__name__)

NS_PREFIX = b"@namespace_"
NODE_TABLE = "node_table"
NODE_PROCESSES_TABLE = "node_processes_table"
NODE_METRICS_TABLE = "node_metrics_table"
SCALING_STATE_KEY = b"scaling_state"
TABLE_PREFIX = "table:"

# pub/sub channels (reference: LOG_FILE_CHANNEL / ERROR_INFO channels of services)
LOG_CHANNEL = "cloudtik:logs"
ERROR_CHANNEL = "cloudtik:errors"
EVENT_CHANNEL = "cloudtik:events"


def _b(x) -> bytes:
    return x if isinstance(x, bytes) else str(x).encode()


def make_key(namespace: Optional[str], key) -> bytes:
    key = _b(key)
    if namespace is None:
        if key.startswith(NS_PREFIX):
            raise ValueError(f"key must not start with {NS_PREFIX!r}")
        return key
    return NS_PREFIX + namespace.encode() + b":" + key


def strip_key(key: bytes) -> bytes:
    return key.split(b":", 1)[1] if key.startswith(NS_PREFIX) else key


class StateClient:
    def __init__(self, conn: RespConnection):
        self.conn = conn

    @classmethod
    def create(cls, address: str, password: Optional[str] = None, timeout: float = 10.0,
               client_name: Optional[str] = None) -> "StateClient":
        host, port = address.rsplit(":", 1)
        return cls(RespConnection(host, int(port), password, timeout=timeout,
                                  client_name=client_name).connect())

    # ------------------------------------------------------------------ KV
    def kv_get(self, key, namespace: Optional[str] = None) -> Optional[bytes]:
        return self.conn.get(make_key(namespace, key))

    def kv_multi_get(self, keys, namespace: Optional[str] = None) -> Dict[bytes, Optional[bytes]]:
        keys = list(keys)
        vals = self.conn.execute("MGET", *[make_key(namespace, k) for k in keys]) if keys else []
        return {_b(k): v for k, v in zip(keys, vals)}

    def kv_put(self, key, value, overwrite: bool = True, namespace: Optional[str] = None) -> int:
        """Returns 1 if the key already existed (and was not overwritten when
        ``overwrite`` is False), 0 otherwise (same contract as the reference)."""
        k = make_key(namespace, key)
        if overwrite:
            existed = self.conn.exists(k)
            self.conn.set(k, _b(value))
            return int(bool(existed))
        return 0 if self.conn.set(k, _b(value), nx=True) else 1

    def kv_del(self, key, namespace: Optional[str] = None, del_by_prefix: bool = False) -> int:
        if del_by_prefix:
            ks = self.conn.keys(make_key(namespace, key) + b"*")
            return self.conn.delete(*ks) if ks else 0
        return self.conn.delete(make_key(namespace, key))

    def kv_exists(self, key, namespace: Optional[str] = None) -> bool:
        return bool(self.conn.exists(make_key(namespace, key)))

    def kv_keys(self, prefix, namespace: Optional[str] = None) -> List[bytes]:
        pat = make_key(namespace, prefix) + b"*"
        return [strip_key(k) for k in self.conn.keys(pat)]

    # ------------------------------------------------------------------ tables
    def table_put(self, table: str, key, value: Any):
        self.conn.hset(TABLE_PREFIX + table, _b(key), json.dumps(value))

    def table_get(self, table: str, key) -> Optional[Any]:
        v = self.conn.hget(TABLE_PREFIX + table, _b(key))
        return None if v is None else json.loads(v)

    def table_get_all(self, table: str) -> Dict[str, Any]:
        return {k.decode(): json.loads(v) for k, v in self.conn.hgetall(TABLE_PREFIX + table).items()}

    def table_delete(self, table: str, key) -> int:
        return self.conn.hdel(TABLE_PREFIX + table, _b(key))

    # ------------------------------------------------------------------ pub/sub + misc
    def publish(self, channel: str, message) -> int:
        return self.conn.publish(channel, message if isinstance(message, (bytes, str)) else json.dumps(message))

    def subscribe(self, *channels):
        ps = self.conn.pubsub()
        ps.subscribe(*channels)
        return ps

    def save(self):
        return self.conn.save()

    def ping(self) -> bool:
        try:
            return self.conn.ping()
        except (ConnectionError, OSError, RespError):
            return False


# ---------------------------------------------------------------------- module-level KV
_kv_client: Optional[StateClient] = None


def kv_initialize(client: StateClient):
    global _kv_client
    _kv_client = client


def kv_initialize_with_address(address: str, password: Optional[str] = None):
    kv_initialize(StateClient.create(address, password))


def kv_reset():
    global _kv_client
    _kv_client = None


def kv_initialized() -> bool:
    return _kv_client is not None


def _kv() -> StateClient:
    if _kv_client is None:
        raise RuntimeError("kv store is not initialized (call kv_initialize first)")
    return _kv_client


def kv_get(key, namespace=None):
    return _kv().kv_get(key, namespace)


def kv_exists(key, namespace=None):
    return _kv().kv_exists(key, namespace)


def kv_put(key, value, overwrite=True, namespace=None):
    return _kv().kv_put(key, value, overwrite, namespace)


def kv_del(key, del_by_prefix=False, namespace=None):
    return _kv().kv_del(key, namespace, del_by_prefix)


def kv_list(prefix, namespace=None):
    return _kv().kv_keys(prefix, namespace)


def kv_save():
    return _kv().save()


# ---------------------------------------------------------------------- tables
class StateTable:
    def __init__(self, client: StateClient, name: str):
        self.client, self.name = client, name

    def put(self, key, value):
        self.client.table_put(self.name, key, value)

    def get(self, key):
        return self.client.table_get(self.name, key)

    def get_all(self) -> Dict[str, Any]:
        return self.client.table_get_all(self.name)

    def delete(self, key):
        return self.client.table_delete(self.name, key)


class NodeStateTable(StateTable):
    def __init__(self, client: StateClient):
        super().__init__(client, NODE_TABLE)


class StateTableStore:
    def __init__(self, client: StateClient):
        self.client = client
        self._node_table = NodeStateTable(client)
        self._user: Dict[str, StateTable] = {}

    def get_node_table(self) -> NodeStateTable:
        return self._node_table

    def get_user_state_table(self, name: str) -> StateTable:
        if name not in self._user:
            self._user[name] = StateTable(self.client, name)
        return self._user[name]


class StateNodeManager:
    """Node registration in the node table (reference state_node_manager.py)."""

    def __init__(self, store: StateTableStore):
        self.table = store.get_node_table()

    def register_node(self, node_id: str, node_info: Dict[str, Any]):
        info = dict(node_info)
        info.setdefault("node_id", node_id)
        info["last_heartbeat_time"] = time.time()
        self.table.put(node_id, info)

    def heartbeat(self, node_id: str, node_info: Optional[Dict[str, Any]] = None):
        cur = self.table.get(node_id) or {"node_id": node_id}
        if node_info:
            cur.update(node_info)
        cur["last_heartbeat_time"] = time.time()
        self.table.put(node_id, cur)

    def drain_node(self, node_id: str):
        self.table.delete(node_id)

    def get_node_table(self) -> Dict[str, Any]:
        return self.table.get_all()


class ControlState:
    """Facade owned by head services: one connection, the table store, and helpers."""

    def __init__(self, address: Optional[str] = None, password: Optional[str] = None,
                 client: Optional[StateClient] = None):
        self.address = address
        self.client = client or StateClient.create(address, password, client_name="control-state")
        self.tables = StateTableStore(self.client)

    def get_node_table(self) -> StateTable:
        return self.tables.get_node_table()

    def get_user_state_table(self, name: str) -> StateTable:
        return self.tables.get_user_state_table(name)

    def get_node_processes_table(self) -> StateTable:
        return self.tables.get_user_state_table(NODE_PROCESSES_TABLE)

    def get_node_metrics_table(self) -> StateTable:
        return self.tables.get_user_state_table(NODE_METRICS_TABLE)


class ScalingStateClient:
    """Reads heartbeats / node resources and writes the cluster scaling state."""

    def __init__(self, control_state: ControlState):
        self.cs = control_state

    @staticmethod
    def create_from(control_state: ControlState) -> "ScalingStateClient":
        return ScalingStateClient(control_state)

    def get_cluster_heartbeat_state(self) -> Dict[str, Dict[str, Any]]:
        out = {}
        for node_id, info in self.cs.get_node_table().get_all().items():
            out[node_id] = {"node_id": node_id, "node_ip": info.get("node_ip"),
                            "last_heartbeat_time": info.get("last_heartbeat_time", 0.0)}
        return out

    def get_node_resource_states(self) -> Dict[str, Dict[str, Any]]:
        return self.cs.get_node_metrics_table().get_all()

    def get_scaling_state(self) -> Optional[Dict[str, Any]]:
        v = self.cs.client.kv_get(SCALING_STATE_KEY, namespace="scaling")
        return None if v is None else json.loads(v)

    def update_scaling_state(self, scaling_state: Dict[str, Any]):
        self.cs.client.kv_put(SCALING_STATE_KEY, json.dumps(scaling_state), namespace="scaling")


# ---------------------------------------------------------------------- server process
class StateServer:
    """Launches the native ``cloudtik-state-server`` as a child process."""

    def __init__(self, port: int = 6789, bind: str = "127.0.0.1", password: Optional[str] = None,
                 data_dir: Optional[str] = None, save_interval: int = 0,
                 log_file: Optional[str] = None, sanitize: Optional[bool] = None):
        self.port, self.bind, self.password = int(port), bind, password
        # ASan/UBSan build of the server: sanitize=True or
        # CLOUDTIK_STATE_SERVER_SANITIZE=1
        self.sanitize = os.environ.get("CLOUDTIK_STATE_SERVER_SANITIZE", "0") == "1" if sanitize is None else sanitize
        self.data_dir = data_dir or os.getcwd()
        self.save_interval = save_interval
        self.log_file = log_file
        self.proc: Optional[subprocess.Popen] = None

    @property
    def address(self) -> str:
        host = "127.0.0.1" if self.bind in ("0.0.0.0", "") else self.bind
        return f"{host}:{self.port}"

    def start(self, wait: float = 10.0) -> "StateServer":
        from cloudtik_amd.native.build import state_server_path
        os.makedirs(self.data_dir, exist_ok=True)
        cmd = [state_server_path(sanitize=self.sanitize), "--port", str(self.port), "--bind", self.bind,
               "--dir", self.data_dir, "--save-interval", str(self.save_interval)]
        if self.password:
            cmd += ["--requirepass", self.password]
        out = open(self.log_file, "ab") if self.log_file else subprocess.DEVNULL
        self.proc = subprocess.Popen(cmd, stdout=out, stderr=out, start_new_session=True)
        deadline = time.time() + wait
        while time.time() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError(f"state server exited with code {self.proc.returncode}")
            try:
                c = StateClient.create(self.address, self.password, timeout=1.0)
                if c.ping():
                    c.conn.close()
                    return self
            except ConnectionError:
                pass
            time.sleep(0.05)
        self.stop()
        raise TimeoutError("state server did not come up")

    def stop(self, save: bool = False):
        if self.proc is None:
            return
        if self.proc.poll() is None:
            try:
                c = StateClient.create(self.address, self.password, timeout=2.0)
                c.conn.execute("SHUTDOWN", *([] if save else ["NOSAVE"]))
            except (ConnectionError, OSError, RespError):
                pass
            try:
                self.proc.wait(timeout=5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        self.proc = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
