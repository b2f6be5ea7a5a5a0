"""SSH key-pair bootstrap for the cloud providers: make sure every launched VM carries a public
key whose private half the node updater holds (``auth.ssh_private_key``), so the first
``wait_ready`` over SSH can reach it.

Two modes, as the reference (aws/config.py:3868 ``_configure_key_pair``, gcp/config.py:2678,
_azure/config.py:4068, aliyun/config.py:2153, huaweicloud/config.py:1876):

* **explicit** -- ``auth.ssh_private_key`` is configured: the config must also name the cloud
  key pair on every node type (``KeyName`` / ``KeyPairName`` / ``key_name``) unless the node
  type injects keys itself (``UserData``); GCP and Azure take the public key file
  (``auth.ssh_public_key``, or ``<private>.pub``) and install it through instance metadata /
  the VM's osProfile.
* **implicit** -- no private key configured: a key pair named
  ``cloudtik_<cloud>_<region>[_i]`` is looked up in the cloud; if it exists AND its private key
  file ``~/.ssh/<name>.pem`` is on this machine it is reused; if neither exists it is created
  (AWS / Aliyun / Huawei Cloud return the private key material once, written 0600); a name
  with only one of the two halves is skipped (another machine owns it) and the next index is
  tried.  GCP / Azure have no cloud-side key pairs: the pair is generated locally with
  ``ssh-keygen`` and the public half goes into the node configs.

The cloud calls go through the provider's own client (the boto3 EC2 client, the signed
Aliyun ECS / Huawei Cloud KPS calls), so fake clients in the tests see exactly the requests.
"""
from __future__ import annotations

import os
import subprocess
from typing import Any, Callable, Dict, Optional, Tuple

MAX_KEY_INDEX = 30

# cloud kind -> the node_config key naming the cloud key pair
KEY_FIELD = {"aws": "KeyName", "aliyun": "KeyPairName", "huaweicloud": "key_name"}


def key_pair_name(cloud: str, region: str, i: int, key_name: Optional[str] = None) -> Tuple[str, str]:
    """(cloud key-pair name, local private key path) for attempt ``i``."""
    base = key_name or f"cloudtik_{cloud}_{region}"
    name = base if i == 0 else (f"{base}_{i}" if key_name is None else f"{key_name}_key-{i}")
    return name, os.path.expanduser(f"~/.ssh/{name}.pem")


def write_private_key(path: str, material: str):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
    with os.fdopen(fd, "w") as f:
        f.write(material if material.endswith("\n") else material + "\n")


def _node_types(config) -> Dict[str, Any]:
    return config.get("available_node_types") or {}


def _check_explicit(config, cloud: str):
    field = KEY_FIELD[cloud]
    for name, nt in _node_types(config).items():
        nc = nt.get("node_config") or {}
        if field not in nc and "UserData" not in nc:
            raise ValueError(f"auth.ssh_private_key is set, so node type {name!r} needs `{field}` in its "
                             f"node_config (the cloud key pair of that private key)")


def configure_cloud_key_pair(config: Dict[str, Any], cloud: str, region: str,
                             describe: Callable[[str], bool], create: Callable[[str], str]) -> Dict[str, Any]:
    """AWS / Aliyun / Huawei Cloud: ``describe(name)`` -> does the key pair exist in the cloud;
    ``create(name)`` -> creates it and returns the private key material."""
    auth = config.setdefault("auth", {})
    if auth.get("ssh_private_key"):
        _check_explicit(config, cloud)
        return config
    wanted = (config.get("provider", {}).get("key_pair") or {}).get("key_name")
    chosen = None
    for i in range(MAX_KEY_INDEX):
        name, path = key_pair_name(cloud, region, i, wanted)
        exists, local = describe(name), os.path.exists(path)
        if exists and local:
            chosen = (name, path)
            break
        if not exists and not local:
            write_private_key(path, create(name))
            chosen = (name, path)
            break
    if chosen is None:
        raise RuntimeError(f"no usable {cloud} key pair among {MAX_KEY_INDEX} names: each one exists only in "
                           f"the cloud or only in ~/.ssh; delete unused key pairs or set auth.ssh_private_key")
    name, path = chosen
    auth["ssh_private_key"] = path
    for nt in _node_types(config).values():
        nt.setdefault("node_config", {})[KEY_FIELD[cloud]] = name
    return config


def local_key_pair(config: Dict[str, Any], cloud: str, scope: str) -> Tuple[str, str]:
    """GCP / Azure: (private key path, public key text).  The configured pair, or one
    generated with ssh-keygen under ~/.ssh/cloudtik_<cloud>_<scope>.pem (reused if present)."""
    auth = config.setdefault("auth", {})
    priv = auth.get("ssh_private_key")
    if priv:
        pub_path = os.path.expanduser(auth.get("ssh_public_key") or priv + ".pub")
        priv = os.path.expanduser(priv)
    else:
        priv = os.path.expanduser(f"~/.ssh/cloudtik_{cloud}_{scope}.pem")
        pub_path = priv + ".pub"
        if not os.path.exists(priv):
            os.makedirs(os.path.dirname(priv), exist_ok=True)
            subprocess.run(["ssh-keygen", "-q", "-t", "rsa", "-b", "4096", "-m", "PEM", "-N", "", "-C",
                            f"cloudtik_{cloud}", "-f", priv], check=True, stdin=subprocess.DEVNULL)
        elif not os.path.exists(pub_path):
            out = subprocess.run(["ssh-keygen", "-y", "-f", priv], check=True, capture_output=True, text=True)
            with open(pub_path, "w") as f:
                f.write(out.stdout)
        auth["ssh_private_key"] = priv
    if not os.path.exists(pub_path):
        raise ValueError(f"public key {pub_path} not found (set auth.ssh_public_key)")
    with open(pub_path) as f:
        return priv, f.read().strip()


def configure_gcp_key_pair(config: Dict[str, Any]) -> Dict[str, Any]:
    """Public key as ``ssh-keys`` instance metadata (``user:ssh-rsa AAA.. user``) on every
    node type; the reference adds it to the project's common metadata instead -- per instance
    it touches nothing outside the cluster."""
    user = config.setdefault("auth", {}).setdefault("ssh_user", "ubuntu")
    project = config.get("provider", {}).get("project_id", "default")
    _, pub = local_key_pair(config, "gcp", f"{project}_{user}")
    parts = pub.split()
    line = f"{user}:{parts[0]} {parts[1]} {user}"
    for nt in _node_types(config).values():
        items = nt.setdefault("node_config", {}).setdefault("metadata", {}).setdefault("items", [])
        cur = next((it for it in items if it.get("key") == "ssh-keys"), None)
        if cur is None:
            items.append({"key": "ssh-keys", "value": line})
        elif line not in cur["value"].split("\n"):
            cur["value"] = cur["value"].rstrip("\n") + "\n" + line
    return config


def configure_azure_key_pair(config: Dict[str, Any]) -> Dict[str, Any]:
    """adminUsername + the public key in every VM's osProfile, password login off."""
    user = config.setdefault("auth", {}).setdefault("ssh_user", "ubuntu")
    scope = config.get("provider", {}).get("resource_group") or config.get("provider", {}).get("location", "default")
    _, pub = local_key_pair(config, "azure", f"{scope}_{user}")
    for nt in _node_types(config).values():
        nc = nt.setdefault("node_config", {})
        osp = nc.setdefault("properties", {}).setdefault("osProfile", {})
        osp["adminUsername"] = user
        lc = osp.setdefault("linuxConfiguration", {})
        lc["disablePasswordAuthentication"] = True
        lc["ssh"] = {"publicKeys": [{"path": f"/home/{user}/.ssh/authorized_keys", "keyData": pub}]}
        arm = nc.get("azure_arm_parameters")
        if isinstance(arm, dict):            # reference-style ARM template parameters
            arm["adminUsername"], arm["publicKey"] = user, pub
    return config
