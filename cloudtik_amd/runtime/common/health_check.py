"""Role-aware health checks for replicated runtimes (reference runtime/common/health_check.py +
runtime/xinetd/scripting.py + the mysql / postgres / redis / hdfs health-check hooks).

A load balancer in front of a replicated database must send writes to the primary only and
reads anywhere: it probes ``http://<node>:<health_check_port>/<role>`` and the node answers
200 when it is alive and (if a role is given) currently holds that role, 503 otherwise.  The
responder is an xinetd service (one process per probe, request on stdin, response on
stdout) running ``python -m cloudtik_amd.runtime.common.health_check <runtime>``.

Roles, from the runtime's own view of itself:

* mysql    -- ``SELECT @@global.read_only``: primary / secondary;
* postgres -- ``SELECT pg_is_in_recovery()``: primary / secondary;
* redis    -- ``ROLE``: master / slave;
* hdfs     -- ``hdfs haadmin -getServiceState <nn>`` (HA) or the NameNode being up: active /
  standby.

``XinetdRuntime`` renders one service per runtime of the cluster that declares a
``health_check_port`` (configured_more.py), so enabling ``xinetd`` next to ``mysql`` with
``mysql.health_check_port: 9201`` is all HAProxy needs.
"""
from __future__ import annotations

import subprocess
import sys
from typing import Callable, Dict, List, Optional, Tuple

ROLE_PRIMARY, ROLE_SECONDARY = "primary", "secondary"
ROLE_MASTER, ROLE_SLAVE = "master", "slave"
ROLE_ACTIVE, ROLE_STANDBY = "active", "standby"

Runner = Callable[[List[str]], Tuple[int, str]]


def _run(cmd: List[str]) -> Tuple[int, str]:
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=10)
        return r.returncode, r.stdout
    except (OSError, subprocess.TimeoutExpired):
        return 1, ""


def _mysql(cfg, run) -> Optional[str]:
    rc, out = run(["mysql", "-N", "-B", "-h", "127.0.0.1", "-P", str(cfg.get("port", 3306)), "-u",
                   cfg.get("health_check_user", "root"), "-e", "SELECT @@global.read_only"])
    if rc != 0:
        return None
    return ROLE_SECONDARY if out.strip() == "1" else ROLE_PRIMARY


def _postgres(cfg, run) -> Optional[str]:
    rc, out = run(["psql", "-h", "127.0.0.1", "-p", str(cfg.get("port", 5432)), "-U",
                   cfg.get("health_check_user", "postgres"), "-tAc", "SELECT pg_is_in_recovery()"])
    if rc != 0:
        return None
    return ROLE_SECONDARY if out.strip() == "t" else ROLE_PRIMARY


def _redis(cfg, run) -> Optional[str]:
    cmd = ["redis-cli", "-h", "127.0.0.1", "-p", str(cfg.get("port", 6379))]
    if cfg.get("password"):
        cmd += ["-a", cfg["password"], "--no-auth-warning"]
    rc, out = run(cmd + ["ROLE"])
    if rc != 0 or not out.strip():
        return None
    return ROLE_MASTER if out.split()[0] == "master" else ROLE_SLAVE


def _hdfs(cfg, run) -> Optional[str]:
    nn = cfg.get("namenode_id")
    if nn:
        rc, out = run(["hdfs", "haadmin", "-getServiceState", nn])
        return out.strip() if rc == 0 and out.strip() in (ROLE_ACTIVE, ROLE_STANDBY) else None
    rc, _ = run(["hdfs", "dfsadmin", "-safemode", "get"])
    return ROLE_ACTIVE if rc == 0 else None


CHECKS: Dict[str, Callable[[dict, Runner], Optional[str]]] = {
    "mysql": _mysql, "postgres": _postgres, "redis": _redis, "hdfs": _hdfs}


def check(runtime: str, path: str, cfg: Optional[dict] = None, run: Runner = _run) -> Tuple[int, str]:
    """(HTTP status, body) for a probe of ``path`` (``/`` = alive, ``/<role>`` = holds role)."""
    role = CHECKS[runtime](cfg or {}, run)
    if role is None:
        return 503, f"{runtime} down\n"
    want = path.strip("/").split("/")[0] if path.strip("/") else ""
    if want and want != role:
        return 503, f"{runtime} is {role}, not {want}\n"
    return 200, f"{runtime} {role}\n"


def respond(runtime: str, stdin=sys.stdin, stdout=sys.stdout, cfg: Optional[dict] = None, run: Runner = _run):
    """xinetd entry: read the request line, answer one HTTP response, exit."""
    line = stdin.readline().strip()
    parts = line.split()
    path = parts[1] if len(parts) >= 2 else "/"
    status, body = check(runtime, path, cfg, run)
    reason = "OK" if status == 200 else "Service Unavailable"
    stdout.write(f"HTTP/1.1 {status} {reason}\r\nContent-Type: text/plain\r\nConnection: close\r\n"
                 f"Content-Length: {len(body)}\r\n\r\n{body}")
    stdout.flush()


def xinetd_services(runtime_configs: Dict[str, dict], python: str = sys.executable) -> Dict[str, dict]:
    """xinetd service definitions for every runtime with a ``health_check_port``."""
    out = {}
    for rt, rc in runtime_configs.items():
        if rt in CHECKS and (rc or {}).get("health_check_port"):
            args = f"-m cloudtik_amd.runtime.common.health_check {rt}"
            if rc.get("port"):
                args += f" --port {int(rc['port'])}"
            out[f"{rt}-health-check"] = {"port": int(rc["health_check_port"]), "server": python,
                                         "server_args": args, "user": rc.get("health_check_os_user", "root")}
    return out


def main(argv=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(prog="cloudtik-health-check")
    ap.add_argument("runtime", choices=sorted(CHECKS))
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--namenode-id", default=None)
    a = ap.parse_args(argv)
    cfg = {k: v for k, v in (("port", a.port), ("namenode_id", a.namenode_id)) if v is not None}
    respond(a.runtime, cfg=cfg)
    return 0


if __name__ == "__main__":
    sys.exit(main())


__all__ = ["check", "respond", "xinetd_services", "CHECKS"]
