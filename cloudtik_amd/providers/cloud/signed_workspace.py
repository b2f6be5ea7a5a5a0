"""Aliyun and Huawei Cloud workspaces: network, identity and managed object storage as step
plans (reference providers/_private/aliyun/config.py:211-1420 -- VPC, VSwitches, NAT gateway
+ EIP + SNAT entries, security group, RAM instance roles, OSS bucket -- and
providers/_private/huaweicloud/config.py:131-1000 -- VPC, subnet, NAT gateway + EIP + SNAT
rule, security group, IAM agencies, OBS bucket).

Same contract as providers/cloud/workspace.py: each resource is a ``Step`` with exists /
create / delete, found by its workspace-derived name, so ``WorkspaceBuilder`` creates the
missing ones in order (a failed create resumes where it stopped), deletes in reverse order
and keeps the managed bucket unless asked.

Neither cloud's SDK ships in this image, so the calls are the clouds' signed HTTP APIs
(signing in providers/cloud/signed_providers.py):

* Aliyun: RPC APIs of ECS (security group), VPC (VPC, VSwitch, NAT, EIP, SNAT) and RAM
  (roles, policies) -- ``rpc(product, action, params)``; OSS over its REST API with the
  ``OSS <ak>:<signature>`` header (``oss_sign``) -- ``oss(method, bucket, sub, body, headers)``.
* Huawei Cloud: REST APIs of VPC (VPC, subnet, security group + rules, EIP), NAT (gateway,
  SNAT rule) and IAM (agencies, role grants) with SDK-HMAC-SHA256 -- ``call(method, url,
  params, body)``; OBS with the ``OBS <ak>:<signature>`` header (same string-to-sign layout).

Both transports are injectable (``provider._transport`` / ``provider._object_transport``),
which is how tests/test_signed_workspace.py runs the plans against in-memory fakes of the
APIs that enforce the clouds' dependency rules (no VPC delete while a subnet exists, no
bucket delete while objects remain, ...)."""
from __future__ import annotations

import base64
import email.utils
import hashlib
import hmac
import json
import time
import xml.etree.ElementTree as ET
from typing import Any, Callable, Dict, List, Optional

from cloudtik_amd.providers.cloud.rest_providers import CloudAPIError
from cloudtik_amd.providers.cloud.workspace import Step

WORKSPACE_TAG = "cloudtik-workspace"


def _subnets_of(vpc_cidr: str, n: int) -> List[str]:
    """The first ``n`` /20 (or /24 inside a /20-or-smaller VPC) blocks of the VPC CIDR."""
    import ipaddress
    net = ipaddress.ip_network(vpc_cidr)
    prefix = 20 if net.prefixlen <= 18 else min(28, net.prefixlen + 2)
    return [str(s) for _, s in zip(range(n), net.subnets(new_prefix=prefix))]


def _wait(check: Callable[[], bool], what: str, timeout_s: float, poll_s: float):
    deadline = time.time() + timeout_s
    while not check():
        if time.time() > deadline:
            raise TimeoutError(f"timed out waiting for {what}")
        time.sleep(poll_s)


def object_store_sign(prefix: str, method: str, resource: str, headers: Dict[str, str], sk: str) -> str:
    """``<prefix> <ak>:``-style header signature shared by OSS (``x-oss-``) and OBS
    (``x-obs-``): HMAC-SHA1 over VERB, Content-MD5, Content-Type, Date, the sorted vendor
    headers and the canonical resource ``/bucket/key?subresource``."""
    low = {k.lower(): v.strip() for k, v in headers.items()}
    vendor = f"x-{prefix.lower()}-"
    canon_h = "".join(f"{k}:{low[k]}\n" for k in sorted(low) if k.startswith(vendor))
    to_sign = "\n".join([method.upper(), low.get("content-md5", ""), low.get("content-type", ""),
                         low.get("date", "")]) + "\n" + canon_h + resource
    return base64.b64encode(hmac.new(sk.encode(), to_sign.encode(), hashlib.sha1).digest()).decode()


# query parameters that are part of the signed resource (plain listing parameters are not)
_SUBRESOURCES = {"acl", "bucketInfo", "cors", "delete", "lifecycle", "location", "logging", "policy",
                 "tagging", "uploads", "versioning", "website"}


def canonical_resource(bucket: str, key: str, sub: str) -> str:
    subs = sorted(p for p in (sub or "").split("&") if p and p.split("=")[0] in _SUBRESOURCES)
    return f"/{bucket}/{key}" + ("?" + "&".join(subs) if subs else "")


def _object_transport(prefix: str, host_fmt: str, ak: str, sk: str, timeout_s: float = 60.0):
    """``call(method, bucket, sub='', body=b'', key='')`` -> (status, text) over the bucket's
    virtual-host endpoint; raises ``CloudAPIError`` for >= 400."""
    import requests
    session = requests.Session()

    def call(method, bucket, sub="", body=b"", key=""):
        headers = {"Date": email.utils.formatdate(usegmt=True)}
        if body:
            headers["Content-Type"] = "application/xml"
            headers["Content-MD5"] = base64.b64encode(hashlib.md5(body).digest()).decode()
        resource = canonical_resource(bucket, key, sub)
        headers["Authorization"] = f"{prefix} {ak}:{object_store_sign(prefix, method, resource, headers, sk)}"
        url = f"https://{host_fmt.format(bucket=bucket)}/{key}" + (f"?{sub}" if sub else "")
        r = session.request(method, url, data=body or None, headers=headers, timeout=timeout_s)
        if r.status_code >= 400:
            raise CloudAPIError(r.status_code, r.text[:500])
        return r.status_code, r.text
    return call


def _xml_keys(text: str) -> List[str]:
    """Object keys of a ListObjects response (namespace-agnostic)."""
    if not text:
        return []
    root = ET.fromstring(text)
    return [e.text for e in root.iter() if e.tag.split("}")[-1] == "Key" and e.text]


def _tagging_xml(tags: Dict[str, str]) -> bytes:
    body = "".join(f"<Tag><Key>{k}</Key><Value>{v}</Value></Tag>" for k, v in sorted(tags.items()))
    return f"<Tagging><TagSet>{body}</TagSet></Tagging>".encode()


def _bucket_missing(obj, bucket: str, sub: str) -> bool:
    try:
        obj("GET" if sub else "HEAD", bucket, sub)
        return False
    except CloudAPIError as e:
        if e.status == 404:
            return True
        raise


def _empty_and_delete_bucket(obj, bucket: str, list_sub: str):
    """Objects first (a non-empty bucket refuses DELETE), then the bucket."""
    while True:
        _, text = obj("GET", bucket, list_sub)
        keys = _xml_keys(text)
        if not keys:
            break
        for k in keys:
            obj("DELETE", bucket, "", b"", k)
    obj("DELETE", bucket)


# ============================================================================== Aliyun
ALIYUN_PRODUCTS = {"ecs": ("ecs.{region}.aliyuncs.com", "2014-05-26"),
                   "vpc": ("vpc.{region}.aliyuncs.com", "2016-04-28"),
                   "ram": ("ram.aliyuncs.com", "2015-05-01")}


def aliyun_rpc(provider_config: Dict[str, Any]):
    from cloudtik_amd.providers.cloud.signed_providers import _creds, aliyun_transport
    ak, sk = _creds(provider_config, "ALIBABA_CLOUD_ACCESS_KEY_ID", "ALIBABA_CLOUD_ACCESS_KEY_SECRET")
    region = provider_config["region"]
    calls = {p: aliyun_transport(h.format(region=region), ak, sk, version=v) for p, (h, v) in ALIYUN_PRODUCTS.items()}
    return lambda product, action, params: calls[product](action, params)


def aliyun_oss(provider_config: Dict[str, Any]):
    from cloudtik_amd.providers.cloud.signed_providers import _creds
    ak, sk = _creds(provider_config, "ALIBABA_CLOUD_ACCESS_KEY_ID", "ALIBABA_CLOUD_ACCESS_KEY_SECRET")
    return _object_transport("OSS", "{bucket}.oss-" + provider_config["region"] + ".aliyuncs.com", ak, sk)


class AliyunWorkspace:
    """Steps: VPC -> instance VSwitch -> NAT VSwitch -> NAT gateway -> EIP (bound to the
    NAT) -> SNAT entry (instance VSwitch -> EIP) -> security group -> head / worker RAM roles
    -> [OSS bucket].  Names: ``cloudtik-<workspace>-<kind>``."""

    HEAD_POLICIES = ("AliyunECSFullAccess", "AliyunOSSFullAccess", "AliyunRAMReadOnlyAccess")
    WORKER_POLICIES = ("AliyunOSSFullAccess",)

    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, rpc=None, oss=None,
                 poll_s: float = 3.0, timeout_s: float = 900.0):
        self.cfg = provider_config
        self.ws = workspace_name
        self.region = provider_config["region"]
        self.rpc = rpc or provider_config.get("_transport") or aliyun_rpc(provider_config)
        self.oss = oss or provider_config.get("_object_transport")
        self.poll_s = float(provider_config.get("poll_interval_s", poll_s))
        self.timeout_s = timeout_s
        self.vpc_cidr = provider_config.get("vpc_cidr", "10.0.0.0/16")
        self.bucket = provider_config.get("managed_bucket_name") or f"cloudtik-{workspace_name}-{self.region}-default"
        self.roles = {"head": f"cloudtik-{workspace_name}-head-role", "worker": f"cloudtik-{workspace_name}-worker-role"}

    def _n(self, kind: str) -> str:
        return f"cloudtik-{self.ws}-{kind}"

    def _r(self, product: str, action: str, **params):
        return self.rpc(product, action, dict(params, RegionId=self.region) if product != "ram" else params)

    # -- lookups
    def _vpc(self) -> Optional[Dict[str, Any]]:
        v = (self._r("vpc", "DescribeVpcs", VpcName=self._n("vpc")).get("Vpcs") or {}).get("Vpc", [])
        return v[0] if v else None

    def _vpc_id(self) -> Optional[str]:
        v = self._vpc()
        return v["VpcId"] if v else None

    def _zone(self) -> str:
        z = self.cfg.get("zone_id")
        if z:
            return z
        zones = (self._r("ecs", "DescribeZones").get("Zones") or {}).get("Zone", [])
        if not zones:
            raise RuntimeError(f"no availability zone in {self.region}")
        return zones[0]["ZoneId"]

    def _vswitch(self, kind: str) -> Optional[Dict[str, Any]]:
        vpc = self._vpc_id()
        if vpc is None:
            return None
        v = (self._r("vpc", "DescribeVSwitches", VpcId=vpc, VSwitchName=self._n(kind)).get("VSwitches") or {}).get(
            "VSwitch", [])
        return v[0] if v else None

    def _nat(self) -> Optional[Dict[str, Any]]:
        vpc = self._vpc_id()
        if vpc is None:
            return None
        n = (self._r("vpc", "DescribeNatGateways", VpcId=vpc, Name=self._n("nat")).get("NatGateways") or {}).get(
            "NatGateway", [])
        return n[0] if n else None

    def _eip(self) -> Optional[Dict[str, Any]]:
        e = (self._r("vpc", "DescribeEipAddresses", EipName=self._n("eip")).get("EipAddresses") or {}).get(
            "EipAddress", [])
        return e[0] if e else None

    def _snat_table(self) -> Optional[str]:
        n = self._nat()
        ids = ((n or {}).get("SnatTableIds") or {}).get("SnatTableId", [])
        return ids[0] if ids else None

    def _snat(self) -> Optional[Dict[str, Any]]:
        t = self._snat_table()
        if t is None:
            return None
        s = (self._r("vpc", "DescribeSnatTableEntries", SnatTableId=t, SnatEntryName=self._n("snat"))
             .get("SnatTableEntries") or {}).get("SnatTableEntry", [])
        return s[0] if s else None

    def _sg(self) -> Optional[str]:
        vpc = self._vpc_id()
        if vpc is None:
            return None
        g = (self._r("ecs", "DescribeSecurityGroups", VpcId=vpc, SecurityGroupName=self._n("sg"))
             .get("SecurityGroups") or {}).get("SecurityGroup", [])
        return g[0]["SecurityGroupId"] if g else None

    def _role_exists(self, role: str) -> bool:
        try:
            self._r("ram", "GetRole", RoleName=self.roles[role])
            return True
        except CloudAPIError as e:
            if e.status == 404 or "EntityNotExist" in str(e):
                return False
            raise

    # -- actions
    def _create_vpc(self):
        self._r("vpc", "CreateVpc", CidrBlock=self.vpc_cidr, VpcName=self._n("vpc"),
                Description=f"CloudTik workspace {self.ws}")
        _wait(lambda: (self._vpc() or {}).get("Status") == "Available", "VPC", self.timeout_s, self.poll_s)

    def _create_vswitch(self, kind: str, cidr: str):
        self._r("vpc", "CreateVSwitch", VpcId=self._vpc_id(), ZoneId=self._zone(), CidrBlock=cidr,
                VSwitchName=self._n(kind))
        _wait(lambda: (self._vswitch(kind) or {}).get("Status") == "Available", kind, self.timeout_s, self.poll_s)

    def _create_nat(self):
        self._r("vpc", "CreateNatGateway", VpcId=self._vpc_id(), VSwitchId=self._vswitch("nat-vswitch")["VSwitchId"],
                Name=self._n("nat"), NatType="Enhanced", InternetChargeType="PayByLcu")
        _wait(lambda: (self._nat() or {}).get("Status") == "Available", "NAT gateway", self.timeout_s, self.poll_s)

    def _delete_nat(self):
        nid = self._nat()["NatGatewayId"]
        self._r("vpc", "DeleteNatGateway", NatGatewayId=nid, Force="true")
        _wait(lambda: self._nat() is None, "NAT gateway deletion", self.timeout_s, self.poll_s)

    def _create_eip(self):
        r = self._r("vpc", "AllocateEipAddress", Name=self._n("eip"), Bandwidth=str(self.cfg.get("eip_bandwidth", 100)),
                    InternetChargeType="PayByTraffic")
        self._r("vpc", "AssociateEipAddress", AllocationId=r["AllocationId"], InstanceId=self._nat()["NatGatewayId"],
                InstanceType="Nat")
        _wait(lambda: (self._eip() or {}).get("Status") == "InUse", "EIP association", self.timeout_s, self.poll_s)

    def _delete_eip(self):
        e = self._eip()
        if e.get("InstanceId"):
            self._r("vpc", "UnassociateEipAddress", AllocationId=e["AllocationId"], InstanceId=e["InstanceId"],
                    InstanceType="Nat")
            _wait(lambda: (self._eip() or {}).get("Status") == "Available", "EIP release", self.timeout_s,
                  self.poll_s)
        self._r("vpc", "ReleaseEipAddress", AllocationId=e["AllocationId"])

    def _create_snat(self):
        self._r("vpc", "CreateSnatEntry", SnatTableId=self._snat_table(),
                SourceVSwitchId=self._vswitch("vswitch")["VSwitchId"], SnatIp=self._eip()["IpAddress"],
                SnatEntryName=self._n("snat"))

    def _delete_snat(self):
        s = self._snat()
        self._r("vpc", "DeleteSnatEntry", SnatTableId=self._snat_table(), SnatEntryId=s["SnatEntryId"])

    def _create_sg(self, ssh_sources):
        gid = self._r("ecs", "CreateSecurityGroup", VpcId=self._vpc_id(), SecurityGroupName=self._n("sg"),
                      Description=f"CloudTik workspace {self.ws}")["SecurityGroupId"]
        for src in ssh_sources:
            self._r("ecs", "AuthorizeSecurityGroup", SecurityGroupId=gid, IpProtocol="tcp", PortRange="22/22",
                    SourceCidrIp=src)
        # every port between the workspace's nodes
        self._r("ecs", "AuthorizeSecurityGroup", SecurityGroupId=gid, IpProtocol="all", PortRange="-1/-1",
                SourceCidrIp=self.vpc_cidr)

    def _create_role(self, role: str, policies):
        trust = {"Statement": [{"Action": "sts:AssumeRole", "Effect": "Allow",
                                "Principal": {"Service": ["ecs.aliyuncs.com"]}}], "Version": "1"}
        self._r("ram", "CreateRole", RoleName=self.roles[role], AssumeRolePolicyDocument=json.dumps(trust),
                Description=f"CloudTik workspace {self.ws} {role}")
        for p in policies:
            self._r("ram", "AttachPolicyToRole", PolicyType="System", PolicyName=p, RoleName=self.roles[role])

    def _delete_role(self, role: str, policies):
        for p in policies:
            try:
                self._r("ram", "DetachPolicyFromRole", PolicyType="System", PolicyName=p, RoleName=self.roles[role])
            except CloudAPIError as e:
                if e.status != 404:
                    raise
        self._r("ram", "DeleteRole", RoleName=self.roles[role])

    def _oss(self):
        if self.oss is None:
            self.oss = aliyun_oss(self.cfg)
        return self.oss

    def _create_bucket(self):
        body = b"<CreateBucketConfiguration><StorageClass>Standard</StorageClass></CreateBucketConfiguration>"
        self._oss()("PUT", self.bucket, "", body)
        self._oss()("PUT", self.bucket, "tagging", _tagging_xml({WORKSPACE_TAG: self.ws}))

    def steps(self, config: Dict[str, Any]) -> List[Step]:
        ssh = config.get("allowed_ssh_sources") or self.cfg.get("allowed_ssh_sources") or ["0.0.0.0/0"]
        inst_cidr, nat_cidr = _subnets_of(self.vpc_cidr, 2)
        out = [
            Step("VPC", lambda: self._vpc_id() is not None, self._create_vpc,
                 lambda: self._r("vpc", "DeleteVpc", VpcId=self._vpc_id())),
            Step("instance VSwitch", lambda: self._vswitch("vswitch") is not None,
                 lambda: self._create_vswitch("vswitch", self.cfg.get("vswitch_cidr", inst_cidr)),
                 lambda: self._r("vpc", "DeleteVSwitch", VSwitchId=self._vswitch("vswitch")["VSwitchId"])),
            Step("NAT VSwitch", lambda: self._vswitch("nat-vswitch") is not None,
                 lambda: self._create_vswitch("nat-vswitch", self.cfg.get("nat_vswitch_cidr", nat_cidr)),
                 lambda: self._r("vpc", "DeleteVSwitch", VSwitchId=self._vswitch("nat-vswitch")["VSwitchId"])),
            Step("NAT gateway", lambda: self._nat() is not None, self._create_nat, self._delete_nat),
            Step("elastic IP", lambda: self._eip() is not None, self._create_eip, self._delete_eip),
            Step("SNAT entry", lambda: self._snat() is not None, self._create_snat, self._delete_snat),
            Step("security group", lambda: self._sg() is not None, lambda: self._create_sg(ssh),
                 lambda: self._r("ecs", "DeleteSecurityGroup", SecurityGroupId=self._sg())),
            Step("head role", lambda: self._role_exists("head"),
                 lambda: self._create_role("head", self.HEAD_POLICIES),
                 lambda: self._delete_role("head", self.HEAD_POLICIES)),
            Step("worker role", lambda: self._role_exists("worker"),
                 lambda: self._create_role("worker", self.WORKER_POLICIES),
                 lambda: self._delete_role("worker", self.WORKER_POLICIES)),
        ]
        if config.get("managed_cloud_storage"):
            out.append(Step("managed OSS bucket", lambda: not _bucket_missing(self._oss(), self.bucket, "bucketInfo"),
                            self._create_bucket,
                            lambda: _empty_and_delete_bucket(self._oss(), self.bucket, "list-type=2&max-keys=1000"),
                            managed="storage"))
        return out

    def info(self) -> Dict[str, Any]:
        vs = self._vswitch("vswitch") or {}
        return {"vpc": self._vpc_id(), "vswitch": vs.get("VSwitchId"), "zone": vs.get("ZoneId"),
                "security_group": self._sg(), "roles": dict(self.roles), "bucket": self.bucket}

    def node_config_defaults(self) -> Dict[str, Any]:
        """What a cluster in this workspace fills into its ECS node_config (reference
        aliyun/config.py ``bootstrap_aliyun_from_workspace``)."""
        i = self.info()
        return {"VSwitchId": i["vswitch"], "ZoneId": i["zone"], "SecurityGroupId": i["security_group"]}

    def head_node_config_defaults(self) -> Dict[str, Any]:
        return dict(self.node_config_defaults(), RamRoleName=self.roles["head"])

    def worker_node_config_defaults(self) -> Dict[str, Any]:
        return dict(self.node_config_defaults(), RamRoleName=self.roles["worker"])


# ======================================================================== Huawei Cloud
def huawei_obs(provider_config: Dict[str, Any]):
    from cloudtik_amd.providers.cloud.signed_providers import _creds
    ak, sk = _creds(provider_config, "HUAWEICLOUD_SDK_AK", "HUAWEICLOUD_SDK_SK")
    return _object_transport("OBS", "{bucket}.obs." + provider_config["region"] + ".myhuaweicloud.com", ak, sk)


class HuaweiCloudWorkspace:
    """Steps: VPC -> subnet -> NAT gateway -> EIP -> SNAT rule (subnet -> EIP) -> security
    group (+ rules) -> head / worker IAM agencies (ECS-trusted; OBS access, plus ECS for the
    head) -> [OBS bucket].  Names: ``cloudtik-<workspace>-<kind>``."""

    HEAD_ROLES = ("ECS FullAccess", "OBS OperateAccess")
    WORKER_ROLES = ("OBS OperateAccess",)

    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, call=None, obs=None,
                 poll_s: float = 3.0, timeout_s: float = 900.0):
        from cloudtik_amd.providers.cloud.signed_providers import _creds, huawei_transport
        self.cfg = provider_config
        self.ws = workspace_name
        self.region = provider_config["region"]
        self.project = provider_config["project_id"]
        call = call or provider_config.get("_transport")
        if call is None:
            call = huawei_transport(*_creds(provider_config, "HUAWEICLOUD_SDK_AK", "HUAWEICLOUD_SDK_SK"))
        self.call = call
        self.obs = obs or provider_config.get("_object_transport")
        self.poll_s = float(provider_config.get("poll_interval_s", poll_s))
        self.timeout_s = timeout_s
        self.vpc_cidr = provider_config.get("vpc_cidr", "10.0.0.0/16")
        self.bucket = provider_config.get("managed_bucket_name") or f"cloudtik-{workspace_name}-{self.region}-default"
        self.agencies = {"head": f"cloudtik-{workspace_name}-head-profile",
                         "worker": f"cloudtik-{workspace_name}-worker-profile"}
        self._domain: Optional[str] = provider_config.get("domain_id")

    def _n(self, kind: str) -> str:
        return f"cloudtik-{self.ws}-{kind}"

    def _vpc_url(self, path: str) -> str:
        return f"https://vpc.{self.region}.myhuaweicloud.com/v1/{self.project}{path}"

    def _nat_url(self, path: str) -> str:
        return f"https://nat.{self.region}.myhuaweicloud.com/v2/{self.project}{path}"

    @staticmethod
    def _iam_url(path: str) -> str:
        return f"https://iam.myhuaweicloud.com{path}"

    def _named(self, items: List[Dict[str, Any]], name: str, key: str = "name") -> Optional[Dict[str, Any]]:
        return next((i for i in items if i.get(key) == name), None)

    # -- lookups
    def _vpc(self):
        return self._named(self.call("GET", self._vpc_url("/vpcs"), {"limit": 1000}, None).get("vpcs", []),
                           self._n("vpc"))

    def _vpc_id(self):
        v = self._vpc()
        return v["id"] if v else None

    def _subnet(self):
        vpc = self._vpc_id()
        if vpc is None:
            return None
        return self._named(self.call("GET", self._vpc_url("/subnets"), {"vpc_id": vpc}, None).get("subnets", []),
                           self._n("subnet"))

    def _nat(self):
        g = self.call("GET", self._nat_url("/nat_gateways"), {"name": self._n("nat")}, None).get("nat_gateways", [])
        return g[0] if g else None

    def _eip(self):
        return self._named(self.call("GET", self._vpc_url("/publicips"), {"limit": 1000}, None).get("publicips", []),
                           self._n("bandwidth"), key="bandwidth_name")

    def _snat(self):
        nat = self._nat()
        if nat is None:
            return None
        rules = self.call("GET", self._nat_url("/snat_rules"), {"nat_gateway_id": nat["id"]}, None).get(
            "snat_rules", [])
        sub = self._subnet()
        return next((r for r in rules if sub and r.get("network_id") == sub["id"]), None)

    def _sg(self):
        vpc = self._vpc_id()
        if vpc is None:
            return None
        return self._named(self.call("GET", self._vpc_url("/security-groups"), {"vpc_id": vpc}, None).get(
            "security_groups", []), self._n("sg"))

    def _domain_id(self) -> str:
        if self._domain is None:
            self._domain = self.call("GET", self._iam_url("/v3/auth/domains"), None, None)["domains"][0]["id"]
        return self._domain

    def _agency(self, role: str):
        a = self.call("GET", self._iam_url("/v3.0/OS-AGENCY/agencies"),
                      {"domain_id": self._domain_id(), "name": self.agencies[role]}, None).get("agencies", [])
        return a[0] if a else None

    # -- actions
    def _create_vpc(self):
        self.call("POST", self._vpc_url("/vpcs"), None, {"vpc": {"name": self._n("vpc"), "cidr": self.vpc_cidr}})
        _wait(lambda: (self._vpc() or {}).get("status") == "OK", "VPC", self.timeout_s, self.poll_s)

    def _create_subnet(self):
        import ipaddress
        cidr = self.cfg.get("subnet_cidr") or _subnets_of(self.vpc_cidr, 1)[0]
        gw = str(next(ipaddress.ip_network(cidr).hosts()))
        self.call("POST", self._vpc_url("/subnets"), None,
                  {"subnet": {"name": self._n("subnet"), "cidr": cidr, "gateway_ip": gw, "vpc_id": self._vpc_id()}})
        _wait(lambda: (self._subnet() or {}).get("status") == "ACTIVE", "subnet", self.timeout_s, self.poll_s)

    def _create_nat(self):
        self.call("POST", self._nat_url("/nat_gateways"), None,
                  {"nat_gateway": {"name": self._n("nat"), "router_id": self._vpc_id(),
                                   "internal_network_id": self._subnet()["id"],
                                   "spec": str(self.cfg.get("nat_spec", "1"))}})
        _wait(lambda: (self._nat() or {}).get("status") == "ACTIVE", "NAT gateway", self.timeout_s, self.poll_s)

    def _create_eip(self):
        self.call("POST", self._vpc_url("/publicips"), None,
                  {"publicip": {"type": "5_bgp"},
                   "bandwidth": {"name": self._n("bandwidth"), "size": int(self.cfg.get("eip_bandwidth", 100)),
                                 "share_type": "PER", "charge_mode": "traffic"}})

    def _create_snat(self):
        self.call("POST", self._nat_url("/snat_rules"), None,
                  {"snat_rule": {"nat_gateway_id": self._nat()["id"], "network_id": self._subnet()["id"],
                                 "floating_ip_id": self._eip()["id"], "source_type": 0}})

    def _delete_snat(self):
        self.call("DELETE", self._nat_url(f"/nat_gateways/{self._nat()['id']}/snat_rules/{self._snat()['id']}"),
                  None, None)

    def _rule(self, sg: str, **kw):
        self.call("POST", self._vpc_url("/security-group-rules"), None,
                  {"security_group_rule": dict(security_group_id=sg, direction="ingress", ethertype="IPv4", **kw)})

    def _create_sg(self, ssh_sources):
        sg = self.call("POST", self._vpc_url("/security-groups"), None,
                       {"security_group": {"name": self._n("sg"), "vpc_id": self._vpc_id()}})["security_group"]["id"]
        for src in ssh_sources:
            self._rule(sg, protocol="tcp", port_range_min=22, port_range_max=22, remote_ip_prefix=src)
        self._rule(sg, remote_ip_prefix=self.vpc_cidr)            # every protocol / port inside the VPC

    def _role_id(self, display_name: str) -> str:
        roles = self.call("GET", self._iam_url("/v3/roles"), {"display_name": display_name}, None).get("roles", [])
        if not roles:
            raise RuntimeError(f"IAM role '{display_name}' not found")
        return roles[0]["id"]

    def _create_agency(self, role: str, grants):
        dom = self._domain_id()
        a = self.call("POST", self._iam_url("/v3.0/OS-AGENCY/agencies"), None,
                      {"agency": {"name": self.agencies[role], "domain_id": dom, "trust_domain_name": "op_svc_ecs",
                                  "duration": "FOREVER", "description": f"CloudTik workspace {self.ws} {role}"}})[
            "agency"]
        for g in grants:            # all-projects permission
            self.call("PUT", self._iam_url(f"/v3.0/OS-INHERIT/domains/{dom}/agencies/{a['id']}/roles/"
                                           f"{self._role_id(g)}/inherited_to_projects"), None, None)

    def _obs(self):
        if self.obs is None:
            self.obs = huawei_obs(self.cfg)
        return self.obs

    def _create_bucket(self):
        body = (f"<CreateBucketConfiguration><Location>{self.region}</Location>"
                f"</CreateBucketConfiguration>").encode()
        self._obs()("PUT", self.bucket, "", body)
        self._obs()("PUT", self.bucket, "tagging", _tagging_xml({WORKSPACE_TAG: self.ws}))

    def steps(self, config: Dict[str, Any]) -> List[Step]:
        ssh = config.get("allowed_ssh_sources") or self.cfg.get("allowed_ssh_sources") or ["0.0.0.0/0"]
        out = [
            Step("VPC", lambda: self._vpc_id() is not None, self._create_vpc,
                 lambda: self.call("DELETE", self._vpc_url(f"/vpcs/{self._vpc_id()}"), None, None)),
            Step("subnet", lambda: self._subnet() is not None, self._create_subnet,
                 lambda: self.call("DELETE", self._vpc_url(f"/vpcs/{self._vpc_id()}/subnets/{self._subnet()['id']}"),
                                   None, None)),
            Step("NAT gateway", lambda: self._nat() is not None, self._create_nat,
                 lambda: self.call("DELETE", self._nat_url(f"/nat_gateways/{self._nat()['id']}"), None, None)),
            Step("elastic IP", lambda: self._eip() is not None, self._create_eip,
                 lambda: self.call("DELETE", self._vpc_url(f"/publicips/{self._eip()['id']}"), None, None)),
            Step("SNAT rule", lambda: self._snat() is not None, self._create_snat, self._delete_snat),
            Step("security group", lambda: self._sg() is not None, lambda: self._create_sg(ssh),
                 lambda: self.call("DELETE", self._vpc_url(f"/security-groups/{self._sg()['id']}"), None, None)),
            Step("head agency", lambda: self._agency("head") is not None,
                 lambda: self._create_agency("head", self.HEAD_ROLES),
                 lambda: self.call("DELETE", self._iam_url(f"/v3.0/OS-AGENCY/agencies/{self._agency('head')['id']}"),
                                   None, None)),
            Step("worker agency", lambda: self._agency("worker") is not None,
                 lambda: self._create_agency("worker", self.WORKER_ROLES),
                 lambda: self.call("DELETE", self._iam_url(
                     f"/v3.0/OS-AGENCY/agencies/{self._agency('worker')['id']}"), None, None)),
        ]
        if config.get("managed_cloud_storage"):
            out.append(Step("managed OBS bucket", lambda: not _bucket_missing(self._obs(), self.bucket, ""),
                            self._create_bucket,
                            lambda: _empty_and_delete_bucket(self._obs(), self.bucket, "max-keys=1000"),
                            managed="storage"))
        return out

    def info(self) -> Dict[str, Any]:
        sub, sg = self._subnet() or {}, self._sg() or {}
        return {"vpc": self._vpc_id(), "subnet": sub.get("id"), "security_group": sg.get("id"),
                "agencies": dict(self.agencies), "bucket": self.bucket}

    def node_config_defaults(self) -> Dict[str, Any]:
        """ECS node_config fields of a cluster in this workspace (reference huaweicloud/
        config.py ``bootstrap_huaweicloud_from_workspace``)."""
        i = self.info()
        return {"vpc_id": i["vpc"], "subnet_id": i["subnet"],
                "server": {"security_groups": [{"id": i["security_group"]}]}}

    def head_node_config_defaults(self) -> Dict[str, Any]:
        d = self.node_config_defaults()
        d["server"]["metadata"] = {"agency_name": self.agencies["head"]}
        return d

    def worker_node_config_defaults(self) -> Dict[str, Any]:
        d = self.node_config_defaults()
        d["server"]["metadata"] = {"agency_name": self.agencies["worker"]}
        return d
