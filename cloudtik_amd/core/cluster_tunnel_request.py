"""REST requests to services on the head node (reference
core/_private/cluster/cluster_tunnel_request.py:18-114).

On the head, or when the cluster uses internal IPs, the request goes straight to
``http://<head>:<port>/<endpoint>``.  From outside, an OpenSSH local forward
(``ssh -N -L <local>:<head-internal-ip>:<port>``, honouring the cluster's ssh user, key,
port and ``ssh_proxy_command``) carries it; the ssh process is started for the request and
stopped by its exact pid afterwards.
"""
from __future__ import annotations

import os
import shlex
import signal
import socket
import subprocess
import time
import urllib.error
import urllib.request
from contextlib import contextmanager
from typing import Any, Dict, Iterator, Optional

REST_ENDPOINT_URL_FORMAT = "http://{}:{}/{}"
REST_REQUEST_TIMEOUT = 60


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def request_rest_direct(rest_api_ip: str, rest_api_port: int, endpoint: str,
                        timeout: float = REST_REQUEST_TIMEOUT, data: Optional[bytes] = None) -> bytes:
    url = REST_ENDPOINT_URL_FORMAT.format(rest_api_ip, rest_api_port, endpoint.lstrip("/"))
    req = urllib.request.Request(url, data=data, headers={"Content-Type": "application/json"} if data else {})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.read()


def ssh_tunnel_command(auth: Dict[str, Any], server_ip: str, local_port: int,
                       remote_ip: str, remote_port: int):
    user = auth.get("ssh_user", "root")
    port = int(auth.get("ssh_port", 22))
    cmd = ["ssh", "-N", "-o", "StrictHostKeyChecking=no", "-o", "UserKnownHostsFile=/dev/null",
           "-o", "ExitOnForwardFailure=yes", "-o", "BatchMode=yes", "-p", str(port),
           "-L", f"127.0.0.1:{local_port}:{remote_ip}:{remote_port}"]
    if auth.get("ssh_private_key"):
        cmd += ["-i", os.path.expanduser(auth["ssh_private_key"])]
    proxy = auth.get("ssh_proxy_command")
    if proxy:
        proxy = proxy.replace("%h", server_ip).replace("%p", str(port)).replace("%r", str(user))
        cmd += ["-o", f"ProxyCommand={proxy}"]
    return cmd + [f"{user}@{server_ip}"]


@contextmanager
def open_tunnel(auth: Dict[str, Any], server_ip: str, remote_ip: str, remote_port: int,
                timeout: float = 30.0) -> Iterator[int]:
    """Yield a local port forwarded to remote_ip:remote_port through server_ip."""
    local = _free_port()
    proc = subprocess.Popen(ssh_tunnel_command(auth, server_ip, local, remote_ip, remote_port),
                            stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                            start_new_session=True)
    try:
        end = time.time() + timeout
        while True:
            if proc.poll() is not None:
                raise ConnectionError(f"ssh tunnel to {server_ip} failed: "
                                      f"{proc.stderr.read().decode(errors='replace').strip()}")
            try:
                socket.create_connection(("127.0.0.1", local), timeout=0.5).close()
                break
            except OSError:
                if time.time() > end:
                    raise TimeoutError(f"ssh tunnel to {server_ip} not ready after {timeout}s")
                time.sleep(0.1)
        yield local
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGTERM)
            try:
                proc.wait(timeout=5)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                proc.wait()


def request_rest_to_server(config: Dict[str, Any], server_ip: str, rest_api_ip: str, rest_api_port: int,
                           endpoint: str, data: Optional[bytes] = None) -> bytes:
    with open_tunnel(config.get("auth", {}) or {}, server_ip, rest_api_ip, rest_api_port) as local:
        return request_rest_direct("127.0.0.1", local, endpoint, data=data)


def _request_rest_to_head(config: Dict[str, Any], endpoint: str, rest_api_port: int, on_head: bool = False,
                          data: Optional[bytes] = None) -> bytes:
    from cloudtik_amd.core.cluster_operator import _provider
    from cloudtik_amd.core.cluster_utils import get_head_node
    provider = _provider(config)
    head = get_head_node(provider, config["cluster_name"])
    if head is None:
        raise RuntimeError(f"cluster {config['cluster_name']!r} has no head node")
    internal = provider.internal_ip(head)
    if on_head or config["provider"].get("use_internal_ips"):
        return request_rest_direct(internal, rest_api_port, endpoint, data=data)
    public = provider.external_ip(head) or internal
    return request_rest_to_server(config, public, internal, rest_api_port, endpoint, data=data)


def request_rest_to_head(cluster_config_file: str, endpoint: str, rest_api_port: int,
                         override_cluster_name: Optional[str] = None, on_head: bool = False,
                         data: Optional[bytes] = None) -> bytes:
    from cloudtik_amd.core.cluster_operator import _config
    return _request_rest_to_head(_config(cluster_config_file, override_cluster_name), endpoint,
                                 rest_api_port, on_head, data)


def tunnel_command_string(config: Dict[str, Any], server_ip: str, local_port: int, remote_ip: str,
                          remote_port: int) -> str:
    """The ssh command a user can run to open the same tunnel by hand."""
    return " ".join(shlex.quote(c) for c in ssh_tunnel_command(config.get("auth", {}) or {}, server_ip,
                                                               local_port, remote_ip, remote_port))
