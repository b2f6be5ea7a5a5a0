"""Aliyun (ECS) and Huawei Cloud (ECS) node providers over the clouds' signed HTTP APIs
(reference providers/_private/aliyun/node_provider.py and
providers/_private/huaweicloud/node_provider.py).

The reference drives both clouds through their Python SDKs (aliyunsdkcore / alibabacloud
tea clients, huaweicloudsdkecs).  Neither SDK ships in this image; a node provider needs a
handful of calls, and both APIs accept plain HTTPS requests signed with the account's
AccessKey pair, so the signing is implemented here (standard library ``hmac`` / ``hashlib``)
and the requests go out through ``requests``:

* Aliyun: RPC-style API, signature version 1.0 -- the sorted, RFC 3986-encoded query string
  signed with HMAC-SHA1 under ``secret + "&"`` (``aliyun_sign``).
* Huawei Cloud: REST API, ``SDK-HMAC-SHA256`` -- canonical request (method, path with a
  trailing ``/``, sorted query, signed headers, SHA-256 of the body) signed with HMAC-SHA256
  (``huawei_sign``).

Credentials: ``provider.access_key_id`` / ``provider.access_key_secret`` in the cluster
config, else ``ALIBABA_CLOUD_ACCESS_KEY_ID`` / ``ALIBABA_CLOUD_ACCESS_KEY_SECRET`` (Aliyun),
``HUAWEICLOUD_SDK_AK`` / ``HUAWEICLOUD_SDK_SK`` (Huawei Cloud).  The transport is injectable
(``provider._transport``) so ``tests/test_cloud_providers.py`` runs both providers against
in-memory fakes of the APIs.  Cluster membership and node state live in instance tags.
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import hmac
import json
import os
import time
import uuid
from typing import Any, Callable, Dict, List, Optional
from urllib.parse import quote, urlsplit

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.node_provider import NodeLaunchException, NodeProvider
from cloudtik_amd.providers.cloud.rest_providers import CloudAPIError


def _pct(s: str) -> str:
    """RFC 3986 percent-encoding (unreserved: A-Z a-z 0-9 - _ . ~)."""
    return quote(str(s), safe="-_.~")


def _creds(cfg: Dict[str, Any], env_id: str, env_secret: str):
    ak = cfg.get("access_key_id") or os.environ.get(env_id)
    sk = cfg.get("access_key_secret") or os.environ.get(env_secret)
    if not ak or not sk:
        raise RuntimeError(f"no access key pair: set provider.access_key_id/access_key_secret or {env_id}/{env_secret}")
    return ak, sk


# ------------------------------------------------------------------------------- Aliyun
_ECS_VERSION = "2014-05-26"


def aliyun_sign(params: Dict[str, str], secret: str, method: str = "GET") -> str:
    """Signature v1.0 of an RPC request's parameters (everything but ``Signature``)."""
    canon = "&".join(f"{_pct(k)}={_pct(v)}" for k, v in sorted(params.items()))
    to_sign = f"{method}&{_pct('/')}&{_pct(canon)}"
    mac = hmac.new((secret + "&").encode(), to_sign.encode(), hashlib.sha1).digest()
    return base64.b64encode(mac).decode()


def aliyun_transport(endpoint: str, ak: str, sk: str, timeout_s: float = 60.0,
                     version: str = _ECS_VERSION) -> Callable[[str, Dict], Dict]:
    """RPC caller of one product (``endpoint`` + API ``version``: ECS 2014-05-26, VPC
    2016-04-28, RAM 2015-05-01)."""
    import requests
    session = requests.Session()

    def call(action: str, params: Dict[str, Any]) -> Dict[str, Any]:
        q = {k: str(v) for k, v in params.items()}
        q.update(Action=action, Format="JSON", Version=version, AccessKeyId=ak, SignatureMethod="HMAC-SHA1",
                 SignatureVersion="1.0", SignatureNonce=uuid.uuid4().hex,
                 Timestamp=_dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"))
        q["Signature"] = aliyun_sign(q, sk)
        r = session.get(f"https://{endpoint}/", params=q, timeout=timeout_s)
        if r.status_code >= 400:
            raise CloudAPIError(r.status_code, r.text[:500])
        return r.json()
    return call


def _indexed(prefix: str, items: List[Any]) -> Dict[str, Any]:
    """RPC list parameters: ``InstanceId.1=a&InstanceId.2=b``."""
    return {f"{prefix}.{i + 1}": v for i, v in enumerate(items)}


def _tag_params(tags: Dict[str, str]) -> Dict[str, str]:
    out = {}
    for i, (k, v) in enumerate(sorted(tags.items())):
        out[f"Tag.{i + 1}.Key"], out[f"Tag.{i + 1}.Value"] = k, v
    return out


class AliyunNodeProvider(NodeProvider):
    """ECS instances as nodes; node id = instance id; tags = ECS tags (at most 20 per
    DescribeInstances filter, so the cluster-name tag filters server-side and the rest are
    checked on the returned tags).

    Stopped-node caching (``cache_stopped_nodes``, default true as in the reference
    aliyun node_provider.py:50,213,357): terminating STOPS pay-as-you-go instances
    (``StopInstances`` in StopCharging mode) and deletes spot ones; a launch first restarts
    (``StartInstances``) stopped instances of the same cluster, node kind, node type and
    launch hash, re-tagged with the new launch's tags, and runs only the remainder."""

    def __init__(self, provider_config, cluster_name, transport=None):
        super().__init__(provider_config, cluster_name)
        self.region = provider_config["region"]
        if transport is None and provider_config.get("_transport") is None:
            ak, sk = _creds(provider_config, "ALIBABA_CLOUD_ACCESS_KEY_ID", "ALIBABA_CLOUD_ACCESS_KEY_SECRET")
            transport = aliyun_transport(provider_config.get("endpoint", f"ecs.{self.region}.aliyuncs.com"), ak, sk)
        self._call = transport or provider_config["_transport"]
        self._cache: Dict[str, Dict[str, Any]] = {}
        self.cache_stopped_nodes = bool(provider_config.get("cache_stopped_nodes", True))

    @staticmethod
    def _tags_of(inst) -> Dict[str, str]:
        return {t["TagKey"]: t.get("TagValue", "") for t in (inst.get("Tags") or {}).get("Tag", [])}

    def key_pair_exists(self, name: str) -> bool:
        r = self._call("DescribeKeyPairs", {"RegionId": self.region, "KeyPairName": name})
        return any(k.get("KeyPairName") == name for k in (r.get("KeyPairs") or {}).get("KeyPair", []))

    def create_key_pair(self, name: str) -> str:
        return self._call("CreateKeyPair", {"RegionId": self.region, "KeyPairName": name})["PrivateKeyBody"]

    @staticmethod
    def bootstrap_config(cluster_config):
        """ECS key pair for the updater's SSH (reference aliyun/config.py:2153)."""
        from cloudtik_amd.providers.cloud import keypairs
        p = AliyunNodeProvider(cluster_config["provider"], cluster_config.get("cluster_name", "default"))
        return keypairs.configure_cloud_key_pair(cluster_config, "aliyun", p.region, p.key_pair_exists,
                                                 p.create_key_pair)

    def _describe(self, extra: Dict[str, Any]) -> List[Dict[str, Any]]:
        out, page = [], 1
        while True:
            r = self._call("DescribeInstances", dict(extra, RegionId=self.region, PageNumber=page, PageSize=100))
            got = (r.get("Instances") or {}).get("Instance", [])
            out += got
            if len(got) < 100 or len(out) >= int(r.get("TotalCount", 0)):
                return out
            page += 1

    def non_terminated_nodes(self, tag_filters):
        scope = self.cluster_filter() or {k: v for k, v in tag_filters.items()
                                          if k == T.CLOUDTIK_TAG_WORKSPACE_NAME}
        insts = self._describe(_tag_params(scope))
        live = [i for i in insts if i.get("Status") in ("Pending", "Starting", "Running")]
        self._cache.update({i["InstanceId"]: i for i in live})
        return [i["InstanceId"] for i in live
                if all(self._tags_of(i).get(k) == v for k, v in tag_filters.items())]

    def _node(self, node_id, refresh=False):
        if refresh or node_id not in self._cache:
            got = self._describe({"InstanceIds": json.dumps([node_id])})
            if not got:
                return {"InstanceId": node_id, "Status": "Deleted"}
            self._cache[node_id] = got[0]
        return self._cache[node_id]

    def is_running(self, node_id):
        return self._node(node_id).get("Status") == "Running"

    def is_terminated(self, node_id):
        return self._node(node_id).get("Status") not in ("Pending", "Starting", "Running")

    def node_tags(self, node_id):
        return self._tags_of(self._node(node_id))

    def internal_ip(self, node_id):
        ips = (((self._node(node_id).get("VpcAttributes") or {}).get("PrivateIpAddress") or {})
               .get("IpAddress") or [])
        return ips[0] if ips else None

    def external_ip(self, node_id):
        n = self._node(node_id)
        eip = (n.get("EipAddress") or {}).get("IpAddress")
        if eip:
            return eip
        ips = (n.get("PublicIpAddress") or {}).get("IpAddress") or []
        return ips[0] if ips else None

    def _reuse_stopped(self, tags, count) -> Dict[str, Any]:
        """Restart up to ``count`` stopped instances launched from the same configuration."""
        keys = (T.CLOUDTIK_TAG_CLUSTER_NAME, T.CLOUDTIK_TAG_NODE_KIND, T.CLOUDTIK_TAG_LAUNCH_CONFIG,
                T.CLOUDTIK_TAG_USER_NODE_TYPE)
        want = {k: tags[k] for k in keys if k in tags}
        insts = self._describe(dict(_tag_params(want), Status="Stopped"))
        found = sorted((i for i in insts if i.get("Status") == "Stopped"
                        and all(self._tags_of(i).get(k) == v for k, v in want.items())),
                       key=lambda i: i["InstanceId"])[:count]
        if not found:
            return {}
        ids = [i["InstanceId"] for i in found]
        self._call("StartInstances", dict(_indexed("InstanceId", ids), RegionId=self.region))
        self._call("TagResources", dict(_tag_params({k: str(v) for k, v in tags.items()}),
                                        RegionId=self.region, ResourceType="instance",
                                        **_indexed("ResourceId", ids)))
        out = {}
        for inst in found:
            cur = self._tags_of(inst)
            cur.update({k: str(v) for k, v in tags.items()})
            inst = dict(inst, Status="Starting",
                        Tags={"Tag": [{"TagKey": k, "TagValue": v} for k, v in cur.items()]})
            self._cache[inst["InstanceId"]] = inst
            out[inst["InstanceId"]] = inst
        return out

    def create_node(self, node_config, tags, count):
        tags = dict(tags, **{T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name})
        reused: Dict[str, Any] = {}
        if self.cache_stopped_nodes:
            reused = self._reuse_stopped(tags, count)
            count -= len(reused)
            if count <= 0:
                return reused
        out = self._run(node_config, tags, count)
        out.update(reused)
        return out

    def _run(self, node_config, tags, count):
        params: Dict[str, Any] = {"RegionId": self.region, "Amount": count,
                                  "InstanceName": f"{self.cluster_name}-{tags.get(T.CLOUDTIK_TAG_NODE_KIND, 'node')}"}
        for key in ("InstanceType", "ImageId", "SecurityGroupId", "VSwitchId", "ZoneId", "KeyPairName",
                    "InternetMaxBandwidthOut", "InstanceChargeType", "SystemDisk.Category", "SystemDisk.Size"):
            if key in node_config:
                params[key] = node_config[key]
        params.update(_tag_params(tags))
        try:
            r = self._call("RunInstances", params)
        except CloudAPIError as e:
            raise NodeLaunchException("AliyunRunInstancesFailed", str(e))
        ids = (r.get("InstanceIdSets") or {}).get("InstanceIdSet", [])
        return {i: {"InstanceId": i} for i in ids}

    def set_node_tags(self, node_id, tags):
        self._call("TagResources", dict(_tag_params(tags), RegionId=self.region, ResourceType="instance",
                                        **{"ResourceId.1": node_id}))
        self._node(node_id, refresh=True)

    def terminate_node(self, node_id):
        self.terminate_nodes([node_id])

    def terminate_nodes(self, node_ids: List[str]):
        if not node_ids:
            return
        delete, stop = list(node_ids), []
        if self.cache_stopped_nodes:
            # spot instances are reclaimed by the cloud when stopped: those are deleted
            spot = {n for n in node_ids
                    if self._node(n).get("SpotStrategy", "NoSpot") not in ("NoSpot", "")}
            stop = [n for n in node_ids if n not in spot]
            delete = [n for n in node_ids if n in spot]
        for i in range(0, len(stop), 100):     # StopInstances / DeleteInstances take at most 100 ids
            self._call("StopInstances", dict(_indexed("InstanceId", stop[i:i + 100]), RegionId=self.region,
                                             StoppedMode="StopCharging"))
        for i in range(0, len(delete), 100):
            self._call("DeleteInstances", dict(_indexed("InstanceId", delete[i:i + 100]), RegionId=self.region,
                                               Force="true"))
        for nid in node_ids:
            self._cache.pop(nid, None)


# -------------------------------------------------------------------------- Huawei Cloud
def huawei_sign(method: str, url: str, params: Optional[Dict[str, Any]], headers: Dict[str, str], body: bytes,
                ak: str, sk: str) -> str:
    """``Authorization`` header value of an SDK-HMAC-SHA256 signed request.  ``headers`` must
    hold ``Host`` and ``X-Sdk-Date`` (``%Y%m%dT%H%M%SZ``); all given headers are signed."""
    path = urlsplit(url).path or "/"
    canon_uri = "/".join(_pct(seg) for seg in path.split("/"))
    if not canon_uri.endswith("/"):
        canon_uri += "/"
    canon_q = "&".join(f"{_pct(k)}={_pct(v)}" for k, v in sorted((params or {}).items()))
    hs = sorted((k.lower(), v.strip()) for k, v in headers.items())
    canon_h = "".join(f"{k}:{v}\n" for k, v in hs)
    signed = ";".join(k for k, _ in hs)
    creq = "\n".join([method.upper(), canon_uri, canon_q, canon_h, signed, hashlib.sha256(body).hexdigest()])
    date = next(v for k, v in hs if k == "x-sdk-date")
    to_sign = f"SDK-HMAC-SHA256\n{date}\n{hashlib.sha256(creq.encode()).hexdigest()}"
    sig = hmac.new(sk.encode(), to_sign.encode(), hashlib.sha256).hexdigest()
    return f"SDK-HMAC-SHA256 Access={ak}, SignedHeaders={signed}, Signature={sig}"


def huawei_transport(ak: str, sk: str, timeout_s: float = 60.0):
    import requests
    session = requests.Session()

    def call(method, url, params=None, body=None):
        data = json.dumps(body).encode() if body is not None else b""
        headers = {"Host": urlsplit(url).netloc, "Content-Type": "application/json",
                   "X-Sdk-Date": _dt.datetime.now(_dt.timezone.utc).strftime("%Y%m%dT%H%M%SZ")}
        headers["Authorization"] = huawei_sign(method, url, params, headers, data, ak, sk)
        r = session.request(method, url, params=params, data=data or None, headers=headers, timeout=timeout_s)
        if r.status_code >= 400:
            raise CloudAPIError(r.status_code, r.text[:500])
        return r.json() if r.content else {}
    return call


class HuaweiCloudNodeProvider(NodeProvider):
    """ECS servers as nodes; node id = server id; tags = server tags (``key=value`` strings
    in the server detail, ``{key, value}`` objects on the tag actions)."""

    def __init__(self, provider_config, cluster_name, transport=None):
        super().__init__(provider_config, cluster_name)
        self.region = provider_config["region"]
        self.project = provider_config["project_id"]
        if transport is None and provider_config.get("_transport") is None:
            ak, sk = _creds(provider_config, "HUAWEICLOUD_SDK_AK", "HUAWEICLOUD_SDK_SK")
            transport = huawei_transport(ak, sk)
        self._call = transport or provider_config["_transport"]
        self._cache: Dict[str, Dict[str, Any]] = {}
        self.cache_stopped_nodes = bool(provider_config.get("cache_stopped_nodes", True))

    def _url(self, path: str, version: str = "v1") -> str:
        host = self.provider_config.get("endpoint", f"ecs.{self.region}.myhuaweicloud.com")
        return f"https://{host}/{version}/{self.project}/cloudservers{path}"

    def _kps_url(self, name: str = "") -> str:
        host = self.provider_config.get("kps_endpoint", f"kps.{self.region}.myhuaweicloud.com")
        return f"https://{host}/v3/{self.project}/keypairs" + (f"/{name}" if name else "")

    def key_pair_exists(self, name: str) -> bool:
        try:
            return bool(self._call("GET", self._kps_url(name), None, None).get("keypair"))
        except CloudAPIError as e:
            if e.status == 404:
                return False
            raise

    def create_key_pair(self, name: str) -> str:
        return self._call("POST", self._kps_url(), None, {"keypair": {"name": name}})["keypair"]["private_key"]

    @staticmethod
    def bootstrap_config(cluster_config):
        """KPS key pair for the updater's SSH (reference huaweicloud/config.py:1876)."""
        from cloudtik_amd.providers.cloud import keypairs
        p = HuaweiCloudNodeProvider(cluster_config["provider"], cluster_config.get("cluster_name", "default"))
        return keypairs.configure_cloud_key_pair(cluster_config, "huaweicloud", p.region, p.key_pair_exists,
                                                 p.create_key_pair)

    @staticmethod
    def _tags_of(srv) -> Dict[str, str]:
        out = {}
        for t in srv.get("tags") or []:
            k, _, v = t.partition("=")
            out[k] = v
        return out

    def non_terminated_nodes(self, tag_filters):
        want = dict(tag_filters, **self.cluster_filter())
        servers, offset = [], 1
        while True:
            page = self._call("GET", self._url("/detail"), {"limit": 100, "offset": offset}, None)
            got = page.get("servers", [])
            servers += got
            if len(got) < 100:
                break
            offset += 1
        out = []
        for s in servers:
            if s.get("status") in ("BUILD", "ACTIVE", "REBOOT", "HARD_REBOOT", "RESIZE", "VERIFY_RESIZE") and \
                    all(self._tags_of(s).get(k) == v for k, v in want.items()):
                self._cache[s["id"]] = s
                out.append(s["id"])
        return out

    def _node(self, node_id, refresh=False):
        if refresh or node_id not in self._cache:
            try:
                self._cache[node_id] = self._call("GET", self._url(f"/{node_id}"), None, None)["server"]
            except CloudAPIError as e:
                if e.status != 404:
                    raise
                return {"id": node_id, "status": "DELETED"}
        return self._cache[node_id]

    def is_running(self, node_id):
        return self._node(node_id).get("status") == "ACTIVE"

    def is_terminated(self, node_id):
        return self._node(node_id).get("status") in ("SHUTOFF", "DELETED", "SOFT_DELETED", "ERROR")

    def node_tags(self, node_id):
        return self._tags_of(self._node(node_id))

    def _addr(self, node_id, kind):
        for addrs in (self._node(node_id).get("addresses") or {}).values():
            for a in addrs:
                if a.get("OS-EXT-IPS:type") == kind:
                    return a.get("addr")
        return None

    def internal_ip(self, node_id):
        return self._addr(node_id, "fixed")

    def external_ip(self, node_id):
        return self._addr(node_id, "floating")

    def create_node(self, node_config, tags, count):
        tags = dict(tags, **{T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name})
        server = json.loads(json.dumps(node_config.get("server", {})))
        for key, dst in (("flavor", "flavorRef"), ("image_id", "imageRef"), ("vpc_id", "vpcid"),
                         ("key_name", "key_name")):
            if key in node_config:
                server[dst] = node_config[key]
        if "subnet_id" in node_config:
            server["nics"] = [{"subnet_id": node_config["subnet_id"]}]
        server.setdefault("root_volume", {"volumetype": node_config.get("root_volume_type", "SSD")})
        server["name"] = f"{self.cluster_name}-{tags.get(T.CLOUDTIK_TAG_NODE_KIND, 'node')}-{uuid.uuid4().hex[:6]}"
        server["count"] = count
        server["server_tags"] = [{"key": k, "value": v} for k, v in sorted(tags.items())]
        try:
            r = self._call("POST", self._url("", "v1.1"), None, {"server": server})
        except CloudAPIError as e:
            raise NodeLaunchException("HuaweiCreateServersFailed", str(e))
        return {i: {"id": i} for i in r.get("serverIds", [])}

    def set_node_tags(self, node_id, tags):
        self._call("POST", self._url(f"/{node_id}/tags/action"), None,
                   {"action": "create", "tags": [{"key": k, "value": v} for k, v in sorted(tags.items())]})
        self._node(node_id, refresh=True)

    def terminate_node(self, node_id):
        self.terminate_nodes([node_id])

    def terminate_nodes(self, node_ids: List[str]):
        if not node_ids:
            return
        r = self._call("POST", self._url("/delete"), None,
                       {"servers": [{"id": i} for i in node_ids], "delete_publicip": True, "delete_volume": True})
        job = r.get("job_id")
        if job and self.provider_config.get("wait_for_delete", False):
            deadline = time.time() + float(self.provider_config.get("delete_timeout_s", 600))
            host = self.provider_config.get("endpoint", f"ecs.{self.region}.myhuaweicloud.com")
            while time.time() < deadline:
                st = self._call("GET", f"https://{host}/v1/{self.project}/jobs/{job}", None, None).get("status")
                if st in ("SUCCESS", "FAIL"):
                    break
                time.sleep(float(self.provider_config.get("poll_interval_s", 5.0)))
        for nid in node_ids:
            self._cache.pop(nid, None)
