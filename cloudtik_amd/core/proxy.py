"""SOCKS proxy into a cluster's network (reference cluster_operator.start_ssh_proxy:2520):
``ssh -D PORT -N`` to the head, its pid recorded so stop_proxy ends exactly that process.
Clusters on the local / virtual providers are reachable directly and need no proxy."""
from __future__ import annotations

import json
import os
import signal
import subprocess

from cloudtik_amd.core import constants as C


def _pid_path(config) -> str:
    d = os.path.join(os.path.expanduser("~"), ".cloudtik", "proxy")
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, f"{config['cluster_name']}.json")


def start_proxy(config, port: int = C.DEFAULT_PROXY_PORT) -> str:
    if config["provider"].get("type") in ("local", "virtual"):
        return "cluster network is directly reachable: no proxy needed"
    from cloudtik_amd.core.cluster_operator import get_head_node_ip
    auth = config.get("auth", {})
    ip = get_head_node_ip(config)
    cmd = ["ssh", "-o", "StrictHostKeyChecking=no", "-o", "UserKnownHostsFile=/dev/null", "-N", "-D", str(port)]
    if auth.get("ssh_private_key"):
        cmd += ["-i", os.path.expanduser(auth["ssh_private_key"])]
    cmd.append(f"{auth.get('ssh_user', 'ubuntu')}@{ip}")
    p = subprocess.Popen(cmd, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                         start_new_session=True)
    with open(_pid_path(config), "w") as f:
        json.dump({"pid": p.pid, "port": port, "head": ip}, f)
    return f"SOCKS5 proxy on localhost:{port} via {ip} (pid {p.pid})"


def stop_proxy(config) -> str:
    path = _pid_path(config)
    if not os.path.exists(path):
        return "no proxy running"
    with open(path) as f:
        info = json.load(f)
    try:
        os.kill(int(info["pid"]), signal.SIGTERM)
    except ProcessLookupError:
        pass
    os.remove(path)
    return f"stopped proxy pid {info['pid']}"
