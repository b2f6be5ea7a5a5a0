"""Postgres connection poolers whose backends follow service discovery
(``backend.config_mode: dynamic``).

Reference behaviour (what, not how): runtime/pgbouncer/discovery.py:12-52 +
pgbouncer/scripting.py:311-344 + pgbouncer/utils.py:119-205 and runtime/pgpool/discovery.py:
12-64 + pgpool/scripting.py:108-160.

* config modes: ``static`` (databases / servers given in the config), ``local`` (the Postgres
  of this cluster), ``dynamic`` (Postgres services discovered through Consul); the default is
  static when databases are configured, else local when the cluster runs Postgres, else
  dynamic when it runs Consul.
* PgBouncer: one ``[databases]`` entry per discovered Postgres service (name with ``-`` ->
  ``_``), host list = the service's live servers; the file is rewritten and PgBouncer
  reloaded (SIGHUP / ``RELOAD``) only when the discovered set changed.
* pgpool-II: discovered servers that are not yet backends are appended as
  ``backend_hostnameN / backend_portN`` (existing numbering is kept: pgpool addresses nodes by
  index, and a vanished server is handled by its health check, not by renumbering), then
  ``pgpool reload``.

Jobs take an injected ``query`` (service instances: name, host, port, meta) and ``runner``;
the change hash is recorded only after the reload succeeded, so a failed reload is retried.
"""
from __future__ import annotations

import json
import logging
import os
import re
import subprocess
from typing import Any, Dict, List, Optional, Tuple

from cloudtik_amd.core.load_balancer import json_hash
from cloudtik_amd.core.service_daemon import PullJob

logger = logging.getLogger(__name__)

CONFIG_MODES = ("static", "local", "dynamic")


def resolve_config_mode(backend: Dict[str, Any], runtimes: List[str], static_key: str = "databases") -> str:
    mode = backend.get("config_mode")
    if mode:
        if mode not in CONFIG_MODES:
            raise ValueError(f"backend.config_mode must be one of {CONFIG_MODES}, not {mode!r}")
        if mode == "dynamic" and "consul" not in runtimes and not backend.get("consul_address"):
            raise ValueError("backend.config_mode 'dynamic' needs a service discovery runtime (consul)")
        return mode
    if backend.get(static_key):
        return "static"
    if "postgres" in runtimes:
        return "local"
    if "consul" in runtimes:
        return "dynamic"
    return "local"                    # the head's Postgres (single-node clusters)


def _consul_query(selector, consul_address):
    from cloudtik_amd.runtime.common.consul import ConsulClient
    client = ConsulClient(consul_address or "127.0.0.1:8500")
    return lambda: client.select_services(selector)


def _selector(sel: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    s = dict(sel or {})
    if not s.get("services") and not s.get("runtimes"):
        s["runtimes"] = ["postgres"]          # every Postgres service by default
    return s


def group_servers(instances: List[Dict[str, Any]]) -> Dict[str, List[Tuple[str, int]]]:
    out: Dict[str, List[Tuple[str, int]]] = {}
    for i in instances:
        out.setdefault(i["name"], []).append((i["host"], int(i["port"])))
    return {k: sorted(set(v)) for k, v in sorted(out.items())}


# =============================================================================== PgBouncer
def database_line(cfg: Dict[str, Any]) -> str:
    """One ``[databases]`` value from {host(s), port, dbname, user, auth_user, pool_size}."""
    hosts = cfg["host"] if isinstance(cfg["host"], str) else ",".join(cfg["host"])
    parts = [f"host={hosts}", f"port={int(cfg.get('port', 5432))}"]
    for k in ("dbname", "user", "auth_user", "pool_size", "pool_mode"):
        if cfg.get(k) is not None:
            parts.append(f"{k}={cfg[k]}")
    return " ".join(parts)


def databases_from_services(servers: Dict[str, List[Tuple[str, int]]], db: Dict[str, Any]) -> Dict[str, Dict]:
    """{database name: config} of the discovered services (``db``: user / dbname / auth_user
    for every entry; ``bind_user`` keeps the client's user name instead)."""
    out = {}
    for name, addrs in servers.items():
        if not addrs:
            continue
        cfg = {"host": [h for h, _ in addrs], "port": addrs[0][1]}
        if len({p for _, p in addrs}) > 1:
            logger.warning("pgbouncer: service %s serves on several ports %s; using %d", name, addrs, addrs[0][1])
        cfg["dbname"] = db.get("dbname")
        if not db.get("bind_user"):
            cfg["user"] = db.get("user")
        cfg["auth_user"] = db.get("auth_user")
        out[name.replace("-", "_")] = cfg
    return out


def pgbouncer_ini(databases: Dict[str, Any], settings: Dict[str, Any]) -> str:
    lines = ["[databases]"]
    for name, v in sorted(databases.items()):
        lines.append(f"{name} = {v if isinstance(v, str) else database_line(v)}")
    lines.append("[pgbouncer]")
    lines += [f"{k} = {v}" for k, v in settings.items()]
    return "\n".join(lines) + "\n"


def replace_databases(ini_text: str, databases: Dict[str, Any]) -> str:
    """The ini with its ``[databases]`` section replaced (everything else kept)."""
    body = "".join(f"{n} = {v if isinstance(v, str) else database_line(v)}\n" for n, v in sorted(databases.items()))
    m = re.search(r"^\[databases\][^\n]*\n(.*?)(?=^\[|\Z)", ini_text, flags=re.M | re.S)
    if not m:
        return "[databases]\n" + body + ini_text
    return ini_text[:m.start(1)] + body + ini_text[m.end(1):]


def _run(cmd: str):
    return subprocess.run(["bash", "-c", cmd], check=False)


class _PoolerJob(PullJob):
    def __init__(self, interval, config_file, query, runner, reload_cmd, default_reload):
        fc = {}
        if config_file:
            with open(config_file) as f:
                fc = json.load(f)
        self.cfg = fc
        super().__init__(float(interval or fc.get("interval") or 15.0))
        self.query = query or _consul_query(_selector(fc.get("service_selector")), fc.get("consul_address"))
        self.runner = runner or _run
        self.reload_cmd = reload_cmd or fc.get("reload_cmd") or default_reload
        self.last_hash: Optional[str] = None
        self.reloads = 0
        self._dirty = False           # the file changed and the pooler has not reloaded it yet

    def _write(self, path: str, text: str):
        tmp = path + ".cloudtik-new"
        with open(tmp, "w") as f:
            f.write(text)
        os.replace(tmp, path)
        self._dirty = True

    def _reload_if_dirty(self):
        if not self._dirty:
            return
        r = self.runner(self.reload_cmd)
        if getattr(r, "returncode", 0) not in (0, None):
            raise RuntimeError(f"pooler reload failed (rc {r.returncode}): {self.reload_cmd}")
        self._dirty = False
        self.reloads += 1


class DiscoverPgBouncerBackends(_PoolerJob):
    """Rewrites ``[databases]`` of pgbouncer.ini from the discovered Postgres services."""

    def __init__(self, interval=None, config_file=None, conf_path=None, database=None, query=None, runner=None,
                 reload_cmd=None):
        super().__init__(interval, config_file, query, runner, reload_cmd,
                         "sudo systemctl reload pgbouncer 2>/dev/null || "
                         "sudo pkill -HUP -x pgbouncer")
        self.conf_path = conf_path or self.cfg["conf_path"]
        self.database = database if database is not None else (self.cfg.get("database") or {})
        self.static = self.cfg.get("static_databases") or {}

    def pull(self):
        servers = group_servers(self.query())
        dbs = dict(self.static)
        dbs.update(databases_from_services(servers, self.database))
        h = json_hash(dbs)
        if h == self.last_hash:
            return
        if not servers:
            logger.warning("pgbouncer discovery: no live Postgres service for the selector")
        with open(self.conf_path) as f:
            text = f.read()
        new = replace_databases(text, dbs)
        if new != text:
            self._write(self.conf_path, new)
        self._reload_if_dirty()           # raises on failure: the hash stays unrecorded
        self.last_hash = h


# =============================================================================== pgpool-II
_BACKEND = re.compile(r"^\s*backend_(hostname|port)(\d+)\s*=\s*'?([^'\n#]*)'?", re.M)


def pgpool_backends(conf_text: str) -> List[Tuple[str, int]]:
    """(host, port) of backend 0, 1, ... in index order (port default 5432)."""
    hosts: Dict[int, str] = {}
    ports: Dict[int, int] = {}
    for kind, idx, val in _BACKEND.findall(conf_text):
        if kind == "hostname":
            hosts[int(idx)] = val.strip()
        else:
            ports[int(idx)] = int(val.strip() or 5432)
    return [(hosts[i], ports.get(i, 5432)) for i in sorted(hosts)]


def pgpool_backend_lines(i: int, host: str, port: int, weight: int = 1, flag: str = "ALLOW_TO_FAILOVER") -> List[str]:
    return [f"backend_hostname{i} = '{host}'", f"backend_port{i} = {int(port)}", f"backend_weight{i} = {weight}",
            f"backend_flag{i} = '{flag}'"]


def add_pgpool_backends(conf_text: str, servers: List[Tuple[str, int]]) -> Tuple[str, List[Tuple[str, int]]]:
    """Append the servers that are not backends yet; returns (text, added)."""
    have = pgpool_backends(conf_text)
    added = [s for s in sorted(set(servers)) if s not in have]
    if not added:
        return conf_text, []
    lines = []
    for k, (h, p) in enumerate(added):
        lines += pgpool_backend_lines(len(have) + k, h, p)
    sep = "" if conf_text.endswith("\n") or not conf_text else "\n"
    return conf_text + sep + "\n".join(lines) + "\n", added


class DiscoverPgpoolBackends(_PoolerJob):
    """Appends newly discovered Postgres servers to pgpool.conf's backends and reloads."""

    def __init__(self, interval=None, config_file=None, conf_path=None, query=None, runner=None, reload_cmd=None):
        super().__init__(interval, config_file, query, runner, reload_cmd, "sudo pgpool reload")
        self.conf_path = conf_path or self.cfg["conf_path"]

    def pull(self):
        servers = [a for addrs in group_servers(self.query()).values() for a in addrs]
        h = json_hash(sorted(servers))
        if h == self.last_hash:
            return
        if not servers:
            logger.warning("pgpool discovery: no live Postgres server for the selector")
        with open(self.conf_path) as f:
            text = f.read()
        new, added = add_pgpool_backends(text, servers)
        if added:
            self._write(self.conf_path, new)
            logger.info("pgpool: backends added %s", added)
        self._reload_if_dirty()
        self.last_hash = h
