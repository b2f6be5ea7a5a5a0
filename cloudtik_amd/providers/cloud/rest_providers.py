"""GCP (Compute Engine) and Azure (ARM) node providers over the clouds' REST APIs
(reference providers/_private/gcp/node_provider.py and providers/_private/_azure/
node_provider.py).

The reference drives both clouds through their Python SDKs (googleapiclient discovery,
azure-mgmt-compute).  Neither SDK ships in this image, and a node provider needs only a
handful of calls -- list / insert / delete / label instances -- so these providers speak
the documented REST endpoints directly through ``requests`` and a bearer token:

* token: ``provider.access_token`` in the cluster config, else the ``GOOGLE_OAUTH_ACCESS_TOKEN``
  / ``AZURE_ACCESS_TOKEN`` environment variable, else the cloud's instance metadata
  service (the identity of the VM the head runs on).
* the HTTP layer is one ``transport(method, url, params, body) -> dict`` callable, injectable
  for tests (``tests/test_cloud_providers.py`` runs both providers against an in-memory
  fake of each API).

Cluster membership and node state live in instance labels (GCP) / tags (Azure), exactly as
the other providers keep them in core.tags.
"""
from __future__ import annotations

import json
import os
import re
import time
import uuid
from typing import Any, Callable, Dict, List, Optional

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.node_provider import NodeLaunchException, NodeProvider

Transport = Callable[[str, str, Optional[Dict[str, Any]], Optional[Dict[str, Any]]], Dict[str, Any]]


class CloudAPIError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"HTTP {status}: {message}")
        self.status = status


def requests_transport(token_fn: Callable[[], str], timeout_s: float = 60.0) -> Transport:
    import requests
    session = requests.Session()

    def call(method, url, params=None, body=None):
        r = session.request(method, url, params=params, json=body, timeout=timeout_s,
                            headers={"Authorization": f"Bearer {token_fn()}"})
        if r.status_code >= 400:
            raise CloudAPIError(r.status_code, r.text[:500])
        return r.json() if r.content else {}
    return call


def _metadata_token(url: str, headers: Dict[str, str]) -> str:
    import requests
    r = requests.get(url, headers=headers, timeout=5)
    r.raise_for_status()
    return r.json()["access_token"]


# ---------------------------------------------------------------------------------- GCP
_GCE = "https://compute.googleapis.com/compute/v1"
_LABEL_BAD = re.compile(r"[^a-z0-9_-]")
_TAGS_KEY = "cloudtik-tags"


def gcp_label(v: str) -> str:
    """GCE label keys / values: lowercase letters, digits, '_' and '-', at most 63 chars."""
    return _LABEL_BAD.sub("-", str(v).lower())[:63]


class GCPNodeProvider(NodeProvider):
    """Compute Engine instances as nodes; node id = instance name; tags = labels."""

    @staticmethod
    def bootstrap_config(cluster_config):
        """SSH public key into the instances' metadata (reference gcp/config.py:2678,3478)."""
        from cloudtik_amd.providers.cloud import keypairs
        return keypairs.configure_gcp_key_pair(cluster_config)

    def __init__(self, provider_config, cluster_name, transport: Optional[Transport] = None):
        super().__init__(provider_config, cluster_name)
        self.project = provider_config["project_id"]
        self.zone = provider_config.get("availability_zone") or provider_config["zone"]
        self._call = transport or provider_config.get("_transport") or requests_transport(self._token)
        self._cache: Dict[str, Dict[str, Any]] = {}

    def _token(self) -> str:
        tok = self.provider_config.get("access_token") or os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN")
        if tok:
            return tok
        return _metadata_token("http://metadata.google.internal/computeMetadata/v1/instance/service-accounts/"
                               "default/token", {"Metadata-Flavor": "Google"})

    @property
    def _base(self) -> str:
        return f"{_GCE}/projects/{self.project}/zones/{self.zone}/instances"

    def _wait(self, op: Dict[str, Any], timeout_s: float = 300.0):
        """Zone operations complete asynchronously; poll until DONE (or fail)."""
        deadline = time.time() + timeout_s
        while op.get("status") != "DONE":
            if time.time() > deadline:
                raise CloudAPIError(504, f"operation {op.get('name')} timed out")
            time.sleep(float(self.provider_config.get("poll_interval_s", 2.0)))
            op = self._call("GET", f"{_GCE}/projects/{self.project}/zones/{self.zone}/operations/{op['name']}",
                            None, None)
        if op.get("error"):
            raise CloudAPIError(400, json.dumps(op["error"])[:500])
        return op

    def non_terminated_nodes(self, tag_filters):
        flt = [f'labels.{gcp_label(k)} = "{gcp_label(v)}"'
               for k, v in dict(self.cluster_filter(), **tag_filters).items()]
        items, token = [], None
        while True:
            params = {"filter": " AND ".join(f"({f})" for f in flt)}
            if token:
                params["pageToken"] = token
            page = self._call("GET", self._base, params, None)
            items += page.get("items", [])
            token = page.get("nextPageToken")
            if not token:
                break
        live = [i for i in items if i.get("status") not in ("STOPPING", "TERMINATED", "SUSPENDED")]
        self._cache.update({i["name"]: i for i in live})
        # labels are a lossy (lowercased, sanitised) copy of the tags: confirm on the exact ones
        return [i["name"] for i in live
                if all(self.node_tags(i["name"]).get(k) == v for k, v in tag_filters.items())]

    def _node(self, node_id, refresh=False):
        if refresh or node_id not in self._cache:
            self._cache[node_id] = self._call("GET", f"{self._base}/{node_id}", None, None)
        return self._cache[node_id]

    def is_running(self, node_id):
        return self._node(node_id).get("status") == "RUNNING"

    def is_terminated(self, node_id):
        return self._node(node_id).get("status") in ("STOPPING", "TERMINATED", "SUSPENDED")

    def node_tags(self, node_id):
        """Exact tags from the ``cloudtik-tags`` metadata item (labels only allow a sanitised
        lowercase alphabet, e.g. a node type ``worker.default`` becomes ``worker-default``)."""
        inst = self._node(node_id)
        for item in inst.get("metadata", {}).get("items", []):
            if item.get("key") == _TAGS_KEY:
                return json.loads(item.get("value") or "{}")
        return dict(inst.get("labels", {}))

    def external_ip(self, node_id):
        for nic in self._node(node_id).get("networkInterfaces", []):
            for ac in nic.get("accessConfigs", []):
                if ac.get("natIP"):
                    return ac["natIP"]
        return None

    def internal_ip(self, node_id):
        nics = self._node(node_id).get("networkInterfaces", [])
        return nics[0].get("networkIP") if nics else None

    def create_node(self, node_config, tags, count):
        labels = {gcp_label(k): gcp_label(v) for k, v in dict(tags, **{
            T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name}).items()}
        created = {}
        for _ in range(count):
            body = json.loads(json.dumps(node_config))           # deep copy, JSON-clean
            name = gcp_label(f"{self.cluster_name}-{tags.get(T.CLOUDTIK_TAG_NODE_KIND, 'node')}-"
                             f"{uuid.uuid4().hex[:8]}")
            body["name"] = name
            mt = body.get("machineType", "n2-standard-8")
            if "/" not in mt:
                body["machineType"] = f"zones/{self.zone}/machineTypes/{mt}"
            body["labels"] = dict(body.get("labels", {}), **labels)
            exact = dict(tags, **{T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name})
            md = body.setdefault("metadata", {}).setdefault("items", [])
            md.append({"key": _TAGS_KEY, "value": json.dumps(exact, sort_keys=True)})
            try:
                self._wait(self._call("POST", self._base, None, body))
            except CloudAPIError as e:
                raise NodeLaunchException("GCPInsertFailed", str(e))
            created[name] = self._node(name, refresh=True)
        return created

    def set_node_tags(self, node_id, tags):
        inst = self._node(node_id, refresh=True)
        exact = dict(self.node_tags(node_id), **tags)
        items = [i for i in inst.get("metadata", {}).get("items", []) if i.get("key") != _TAGS_KEY]
        items.append({"key": _TAGS_KEY, "value": json.dumps(exact, sort_keys=True)})
        self._wait(self._call("POST", f"{self._base}/{node_id}/setMetadata", None,
                              {"items": items, "fingerprint": inst.get("metadata", {}).get("fingerprint", "")}))
        labels = dict(inst.get("labels", {}), **{gcp_label(k): gcp_label(v) for k, v in tags.items()})
        self._wait(self._call("POST", f"{self._base}/{node_id}/setLabels", None,
                              {"labels": labels, "labelFingerprint": inst.get("labelFingerprint", "")}))
        self._cache.pop(node_id, None)

    def terminate_node(self, node_id):
        self._wait(self._call("DELETE", f"{self._base}/{node_id}", None, None))
        self._cache.pop(node_id, None)


# -------------------------------------------------------------------------------- Azure
_ARM = "https://management.azure.com"
_VM_API = "2023-03-01"
_NET_API = "2023-05-01"


class AzureNodeProvider(NodeProvider):
    """ARM virtual machines as nodes; node id = VM name; tags = VM tags.  Each VM gets its
    own NIC (``<vm>-nic``) on ``provider.subnet_id`` and, with ``use_public_ip``, a public IP."""

    @staticmethod
    def bootstrap_config(cluster_config):
        """adminUsername + SSH public key in the VMs' osProfile (reference _azure/config.py:4068)."""
        from cloudtik_amd.providers.cloud import keypairs
        return keypairs.configure_azure_key_pair(cluster_config)

    def __init__(self, provider_config, cluster_name, transport: Optional[Transport] = None):
        super().__init__(provider_config, cluster_name)
        self.sub = provider_config["subscription_id"]
        self.rg = provider_config["resource_group"]
        self.location = provider_config.get("location", "eastus")
        self._call = transport or provider_config.get("_transport") or requests_transport(self._token)
        self._cache: Dict[str, Dict[str, Any]] = {}

    def _token(self) -> str:
        tok = self.provider_config.get("access_token") or os.environ.get("AZURE_ACCESS_TOKEN")
        if tok:
            return tok
        return _metadata_token("http://169.254.169.254/metadata/identity/oauth2/token?api-version=2018-02-01"
                               "&resource=https://management.azure.com/", {"Metadata": "true"})

    def _rg(self, provider: str, kind: str, name: str = "") -> str:
        url = f"{_ARM}/subscriptions/{self.sub}/resourceGroups/{self.rg}/providers/{provider}/{kind}"
        return f"{url}/{name}" if name else url

    def _vm_url(self, name=""):
        return self._rg("Microsoft.Compute", "virtualMachines", name)

    def non_terminated_nodes(self, tag_filters):
        want = dict(tag_filters, **self.cluster_filter())
        vms, url, params = [], self._vm_url(), {"api-version": _VM_API}
        while url:
            page = self._call("GET", url, params, None)
            vms += page.get("value", [])
            url, params = page.get("nextLink"), None
        out = []
        for vm in vms:
            tags = vm.get("tags") or {}
            state = vm.get("properties", {}).get("provisioningState", "")
            if all(tags.get(k) == v for k, v in want.items()) and state not in ("Deleting", "Failed"):
                self._cache[vm["name"]] = vm
                out.append(vm["name"])
        return out

    def _vm(self, node_id, refresh=False):
        if refresh or node_id not in self._cache:
            self._cache[node_id] = self._call("GET", self._vm_url(node_id), {"api-version": _VM_API}, None)
        return self._cache[node_id]

    def _power(self, node_id) -> str:
        iv = self._call("GET", self._vm_url(node_id) + "/instanceView", {"api-version": _VM_API}, None)
        for st in iv.get("statuses", []):
            if st.get("code", "").startswith("PowerState/"):
                return st["code"].split("/", 1)[1]
        return "unknown"

    def is_running(self, node_id):
        return self._power(node_id) == "running"

    def is_terminated(self, node_id):
        return self._power(node_id) in ("stopped", "deallocated", "deallocating", "stopping")

    def node_tags(self, node_id):
        return dict(self._vm(node_id).get("tags") or {})

    def _nic(self, node_id):
        return self._call("GET", self._rg("Microsoft.Network", "networkInterfaces", f"{node_id}-nic"),
                          {"api-version": _NET_API}, None)

    def internal_ip(self, node_id):
        cfgs = self._nic(node_id).get("properties", {}).get("ipConfigurations", [])
        return cfgs[0].get("properties", {}).get("privateIPAddress") if cfgs else None

    def external_ip(self, node_id):
        if not self.provider_config.get("use_public_ip", False):
            return None
        pip = self._call("GET", self._rg("Microsoft.Network", "publicIPAddresses", f"{node_id}-ip"),
                         {"api-version": _NET_API}, None)
        return pip.get("properties", {}).get("ipAddress")

    def create_node(self, node_config, tags, count):
        tags = dict(tags, **{T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name})
        created = {}
        for _ in range(count):
            name = re.sub(r"[^a-zA-Z0-9-]", "-", f"{self.cluster_name}-{tags.get(T.CLOUDTIK_TAG_NODE_KIND, 'node')}-"
                                                  f"{uuid.uuid4().hex[:8]}")[:64]
            try:
                ipcfg: Dict[str, Any] = {"subnet": {"id": self.provider_config["subnet_id"]},
                                         "privateIPAllocationMethod": "Dynamic"}
                if self.provider_config.get("use_public_ip", False):
                    pip = self._call("PUT", self._rg("Microsoft.Network", "publicIPAddresses", f"{name}-ip"),
                                     {"api-version": _NET_API},
                                     {"location": self.location, "sku": {"name": "Standard"},
                                      "properties": {"publicIPAllocationMethod": "Static"}, "tags": tags})
                    ipcfg["publicIPAddress"] = {"id": pip["id"]}
                nic = self._call("PUT", self._rg("Microsoft.Network", "networkInterfaces", f"{name}-nic"),
                                 {"api-version": _NET_API},
                                 {"location": self.location, "tags": tags,
                                  "properties": {"ipConfigurations": [{"name": "ipconfig1", "properties": ipcfg}]}})
                props = json.loads(json.dumps(node_config.get("properties", {})))
                if "vm_size" in node_config:
                    props.setdefault("hardwareProfile", {})["vmSize"] = node_config["vm_size"]
                props["networkProfile"] = {"networkInterfaces": [{"id": nic["id"], "properties": {"primary": True}}]}
                vm = self._call("PUT", self._vm_url(name), {"api-version": _VM_API},
                                {"location": self.location, "tags": tags, "properties": props})
            except CloudAPIError as e:
                raise NodeLaunchException("AzureCreateFailed", str(e))
            self._cache[name] = vm
            created[name] = vm
        return created

    def set_node_tags(self, node_id, tags):
        merged = dict(self._vm(node_id, refresh=True).get("tags") or {}, **tags)
        self._cache[node_id] = self._call("PATCH", self._vm_url(node_id), {"api-version": _VM_API},
                                          {"tags": merged})

    def terminate_node(self, node_id):
        self._call("DELETE", self._vm_url(node_id), {"api-version": _VM_API, "forceDeletion": "true"}, None)
        # VM deletion is asynchronous (202) and its NIC stays "in use" until it completes
        deadline = time.time() + float(self.provider_config.get("delete_timeout_s", 600))
        while True:
            try:
                self._call("GET", self._vm_url(node_id), {"api-version": _VM_API}, None)
            except CloudAPIError as e:
                if e.status == 404:
                    break
                raise
            if time.time() > deadline:
                raise CloudAPIError(504, f"VM {node_id} still exists after delete")
            time.sleep(float(self.provider_config.get("poll_interval_s", 5.0)))
        for kind, suffix in (("networkInterfaces", "-nic"), ("publicIPAddresses", "-ip")):
            try:
                self._call("DELETE", self._rg("Microsoft.Network", kind, node_id + suffix), {"api-version": _NET_API},
                           None)
            except CloudAPIError as e:
                if e.status != 404:
                    raise
        self._cache.pop(node_id, None)

    def terminate_nodes(self, node_ids: List[str]):
        for nid in node_ids:
            self.terminate_node(nid)
