"""Aliyun and Huawei Cloud workspaces + managed object storage
(providers/cloud/signed_workspace.py) against in-memory fakes of the clouds' APIs.

The fakes enforce the dependency rules the real APIs enforce (a VPC with a VSwitch / subnet,
security group or NAT gateway refuses deletion, a bound EIP refuses release, a role with an
attached policy refuses deletion, a non-empty bucket refuses deletion) and report new
resources as pending first, so the plans' ordering and waits are exercised.  Checked: create
is complete and idempotent, resources are wired to each other (SNAT: instance subnet -> EIP
of the NAT; security-group rules; role / agency grants; bucket tag), a failed step leaves a
resumable IN_COMPLETED workspace, delete runs in reverse and keeps the managed bucket unless
asked, and the workspace / storage providers drive the same plans (reference
providers/_private/aliyun/config.py create/delete/check workspace, aliyun/storage_provider.py,
huaweicloud/config.py, huaweicloud/storage_provider.py).  Signing: the OSS / OBS header
signature over a fixed request."""
import itertools
import re
import xml.etree.ElementTree as ET

import pytest

from cloudtik_amd.core.workspace import Existence
from cloudtik_amd.providers.cloud.rest_providers import CloudAPIError
from cloudtik_amd.providers.cloud.signed_workspace import (AliyunWorkspace, HuaweiCloudWorkspace,
                                                            canonical_resource, object_store_sign)
from cloudtik_amd.providers.cloud.workspace import WorkspaceBuilder

_ids = itertools.count(1)


def _id(prefix):
    return f"{prefix}-{next(_ids):05d}"


class FakeBuckets:
    """OSS / OBS: (method, bucket, sub, body, key) -> (status, text)."""

    def __init__(self):
        self.buckets = {}

    def __call__(self, method, bucket, sub="", body=b"", key=""):
        b = self.buckets.get(bucket)
        if method == "PUT" and not sub and not key:
            if b is not None:
                raise CloudAPIError(409, "BucketAlreadyExists")
            self.buckets[bucket] = {"objects": set(), "tags": {}, "config": body.decode()}
            return 200, ""
        if b is None:
            raise CloudAPIError(404, "NoSuchBucket")
        if method == "PUT" and sub == "tagging":
            root = ET.fromstring(body)
            b["tags"] = {t.find("Key").text: t.find("Value").text for t in root.iter("Tag")}
            return 200, ""
        if method == "PUT" and key:
            b["objects"].add(key)
            return 200, ""
        if method in ("GET", "HEAD") and sub in ("", "bucketInfo"):
            return 200, "<BucketInfo/>"
        if method == "GET":
            keys = "".join(f"<Contents><Key>{k}</Key></Contents>" for k in sorted(b["objects"])[:2])
            return 200, f'<ListBucketResult xmlns="http://example">{keys}</ListBucketResult>'
        if method == "DELETE" and key:
            b["objects"].discard(key)
            return 204, ""
        if method == "DELETE":
            if b["objects"]:
                raise CloudAPIError(409, "BucketNotEmpty")
            del self.buckets[bucket]
            return 204, ""
        raise AssertionError((method, bucket, sub, key))


# ------------------------------------------------------------------------------ Aliyun
class FakeAliyun:
    def __init__(self):
        self.vpcs, self.vsw, self.nats, self.eips, self.snat, self.sgs = {}, {}, {}, {}, {}, {}
        self.roles = {}
        self.fail = None
        self.calls = []

    @staticmethod
    def _ready(d):
        """New resources are pending on the first describe, then available."""
        if d.get("_pending"):
            d["_pending"] -= 1
            return dict(d, Status="Pending")
        return {k: v for k, v in d.items() if not k.startswith("_")}

    def __call__(self, product, action, p):
        self.calls.append((product, action))
        if self.fail == action:
            raise CloudAPIError(400, f"{action} throttled")
        if product != "ram":
            assert p["RegionId"] == "cn-hangzhou"
        fn = getattr(self, action)
        return fn(p)

    # ECS
    def DescribeZones(self, p):
        return {"Zones": {"Zone": [{"ZoneId": "cn-hangzhou-h"}, {"ZoneId": "cn-hangzhou-i"}]}}

    def CreateSecurityGroup(self, p):
        gid = _id("sg")
        assert p["VpcId"] in self.vpcs
        self.sgs[gid] = {"SecurityGroupId": gid, "VpcId": p["VpcId"], "SecurityGroupName": p["SecurityGroupName"],
                         "rules": []}
        return {"SecurityGroupId": gid}

    def AuthorizeSecurityGroup(self, p):
        self.sgs[p["SecurityGroupId"]]["rules"].append((p["IpProtocol"], p["PortRange"], p["SourceCidrIp"]))
        return {}

    def DescribeSecurityGroups(self, p):
        g = [{"SecurityGroupId": s["SecurityGroupId"]} for s in self.sgs.values()
             if s["VpcId"] == p["VpcId"] and s["SecurityGroupName"] == p["SecurityGroupName"]]
        return {"SecurityGroups": {"SecurityGroup": g}}

    def DeleteSecurityGroup(self, p):
        del self.sgs[p["SecurityGroupId"]]
        return {}

    # VPC
    def CreateVpc(self, p):
        vid = _id("vpc")
        self.vpcs[vid] = {"VpcId": vid, "VpcName": p["VpcName"], "CidrBlock": p["CidrBlock"], "Status": "Available",
                          "_pending": 1}
        return {"VpcId": vid}

    def DescribeVpcs(self, p):
        return {"Vpcs": {"Vpc": [self._ready(v) for v in self.vpcs.values() if v["VpcName"] == p["VpcName"]]}}

    def DeleteVpc(self, p):
        vid = p["VpcId"]
        if any(v["VpcId"] == vid for v in self.vsw.values()) or any(s["VpcId"] == vid for s in self.sgs.values()) \
                or any(n["VpcId"] == vid for n in self.nats.values()):
            raise CloudAPIError(400, "DependencyViolation")
        del self.vpcs[vid]
        return {}

    def CreateVSwitch(self, p):
        vid = p["VpcId"]
        import ipaddress
        assert ipaddress.ip_network(p["CidrBlock"]).subnet_of(ipaddress.ip_network(self.vpcs[vid]["CidrBlock"]))
        sid = _id("vsw")
        self.vsw[sid] = {"VSwitchId": sid, "VpcId": vid, "VSwitchName": p["VSwitchName"], "ZoneId": p["ZoneId"],
                         "CidrBlock": p["CidrBlock"], "Status": "Available", "_pending": 1}
        return {"VSwitchId": sid}

    def DescribeVSwitches(self, p):
        return {"VSwitches": {"VSwitch": [self._ready(v) for v in self.vsw.values()
                                          if v["VpcId"] == p["VpcId"] and v["VSwitchName"] == p["VSwitchName"]]}}

    def DeleteVSwitch(self, p):
        sid = p["VSwitchId"]
        if any(n["VSwitchId"] == sid for n in self.nats.values()) or \
                any(s["SourceVSwitchId"] == sid for s in self.snat.values()):
            raise CloudAPIError(400, "DependencyViolation.VSwitch")
        del self.vsw[sid]
        return {}

    def CreateNatGateway(self, p):
        assert p["VSwitchId"] in self.vsw and p["NatType"] == "Enhanced"
        nid = _id("ngw")
        self.nats[nid] = {"NatGatewayId": nid, "VpcId": p["VpcId"], "VSwitchId": p["VSwitchId"], "Name": p["Name"],
                          "SnatTableIds": {"SnatTableId": [_id("stb")]}, "Status": "Available", "_pending": 2}
        return {"NatGatewayId": nid}

    def DescribeNatGateways(self, p):
        return {"NatGateways": {"NatGateway": [self._ready(n) for n in self.nats.values()
                                               if n["VpcId"] == p["VpcId"] and n["Name"] == p["Name"]]}}

    def DeleteNatGateway(self, p):
        nid = p["NatGatewayId"]
        if any(e.get("InstanceId") == nid for e in self.eips.values()) or \
                any(s["table"] in self.nats[nid]["SnatTableIds"]["SnatTableId"] for s in self.snat.values()):
            raise CloudAPIError(400, "DependencyViolation.NatGateway")
        del self.nats[nid]
        return {}

    def AllocateEipAddress(self, p):
        aid = _id("eip")
        self.eips[aid] = {"AllocationId": aid, "Name": p["Name"], "IpAddress": f"47.0.0.{len(self.eips) + 1}",
                          "Status": "Available", "InstanceId": ""}
        return {"AllocationId": aid, "EipAddress": self.eips[aid]["IpAddress"]}

    def AssociateEipAddress(self, p):
        assert p["InstanceType"] == "Nat" and p["InstanceId"] in self.nats
        self.eips[p["AllocationId"]].update(InstanceId=p["InstanceId"], Status="InUse")
        return {}

    def UnassociateEipAddress(self, p):
        self.eips[p["AllocationId"]].update(InstanceId="", Status="Available")
        return {}

    def DescribeEipAddresses(self, p):
        return {"EipAddresses": {"EipAddress": [dict(e) for e in self.eips.values() if e["Name"] == p["EipName"]]}}

    def ReleaseEipAddress(self, p):
        if self.eips[p["AllocationId"]]["Status"] != "Available":
            raise CloudAPIError(400, "IncorrectEipStatus")
        del self.eips[p["AllocationId"]]
        return {}

    def CreateSnatEntry(self, p):
        assert p["SourceVSwitchId"] in self.vsw
        assert any(e["IpAddress"] == p["SnatIp"] and e["Status"] == "InUse" for e in self.eips.values())
        sid = _id("snat")
        self.snat[sid] = {"SnatEntryId": sid, "table": p["SnatTableId"], "SourceVSwitchId": p["SourceVSwitchId"],
                          "SnatIp": p["SnatIp"], "SnatEntryName": p["SnatEntryName"]}
        return {"SnatEntryId": sid}

    def DescribeSnatTableEntries(self, p):
        return {"SnatTableEntries": {"SnatTableEntry": [
            dict(s) for s in self.snat.values() if s["table"] == p["SnatTableId"] and
            s["SnatEntryName"] == p["SnatEntryName"]]}}

    def DeleteSnatEntry(self, p):
        del self.snat[p["SnatEntryId"]]
        return {}

    # RAM
    def GetRole(self, p):
        if p["RoleName"] not in self.roles:
            raise CloudAPIError(404, "EntityNotExist.Role")
        return {"Role": {"RoleName": p["RoleName"]}}

    def CreateRole(self, p):
        import json
        doc = json.loads(p["AssumeRolePolicyDocument"])
        assert doc["Statement"][0]["Principal"]["Service"] == ["ecs.aliyuncs.com"]
        self.roles[p["RoleName"]] = set()
        return {}

    def AttachPolicyToRole(self, p):
        assert p["PolicyType"] == "System"
        self.roles[p["RoleName"]].add(p["PolicyName"])
        return {}

    def DetachPolicyFromRole(self, p):
        self.roles[p["RoleName"]].discard(p["PolicyName"])
        return {}

    def DeleteRole(self, p):
        if self.roles[p["RoleName"]]:
            raise CloudAPIError(409, "DeleteConflict.Role.Policy")
        del self.roles[p["RoleName"]]
        return {}


def _aliyun(fake, oss, **cfg):
    pc = dict(type="aliyun", region="cn-hangzhou", poll_interval_s=0, _transport=fake, _object_transport=oss, **cfg)
    return pc, AliyunWorkspace(pc, "ws1")


def test_aliyun_workspace_create_idempotent_delete_keeps_bucket():
    fake, oss = FakeAliyun(), FakeBuckets()
    _, plan = _aliyun(fake, oss)
    cfg = {"managed_cloud_storage": True, "allowed_ssh_sources": ["1.2.3.4/32"]}
    b = WorkspaceBuilder(plan.steps(cfg), log=lambda m: None)
    assert b.existence() == Existence.NOT_EXIST
    made = b.create()
    assert made[0] == "VPC" and made[-1] == "managed OSS bucket" and len(made) == len(b.steps)
    assert b.existence() == Existence.COMPLETED and all(b.status().values())
    assert WorkspaceBuilder(plan.steps(cfg), log=lambda m: None).create() == []           # idempotent
    # wiring: the SNAT entry sends the instance VSwitch out through the NAT's EIP
    (snat,) = fake.snat.values()
    (eip,) = fake.eips.values()
    (nat,) = fake.nats.values()
    inst = plan._vswitch("vswitch")
    assert snat["SourceVSwitchId"] == inst["VSwitchId"] and snat["SnatIp"] == eip["IpAddress"]
    assert eip["InstanceId"] == nat["NatGatewayId"] and nat["VSwitchId"] == plan._vswitch("nat-vswitch")["VSwitchId"]
    (sg,) = fake.sgs.values()
    assert ("tcp", "22/22", "1.2.3.4/32") in sg["rules"] and ("all", "-1/-1", "10.0.0.0/16") in sg["rules"]
    assert fake.roles[plan.roles["head"]] == set(AliyunWorkspace.HEAD_POLICIES)
    assert fake.roles[plan.roles["worker"]] == set(AliyunWorkspace.WORKER_POLICIES)
    assert oss.buckets[plan.bucket]["tags"] == {"cloudtik-workspace": "ws1"}
    nc = plan.head_node_config_defaults()
    assert nc == {"VSwitchId": inst["VSwitchId"], "ZoneId": "cn-hangzhou-h", "SecurityGroupId": sg["SecurityGroupId"],
                  "RamRoleName": plan.roles["head"]}
    # delete keeps the bucket unless asked; everything else is gone
    gone = b.delete()
    assert gone[-1] == "VPC" and "managed OSS bucket" not in gone
    assert b.existence() == Existence.NOT_EXIST and b.status()["managed OSS bucket"]
    assert not (fake.vpcs or fake.vsw or fake.nats or fake.eips or fake.snat or fake.sgs or fake.roles)
    oss.buckets[plan.bucket]["objects"].update({"a", "b", "c", "d", "e"})            # a non-empty bucket
    assert b.delete(delete_managed_storage=True) == ["managed OSS bucket"]
    assert not oss.buckets and not any(b.status().values())


def test_aliyun_failed_step_is_resumable():
    fake, oss = FakeAliyun(), FakeBuckets()
    _, plan = _aliyun(fake, oss, zone_id="cn-hangzhou-k")
    fake.fail = "CreateSnatEntry"
    b = WorkspaceBuilder(plan.steps({}), log=lambda m: None)
    with pytest.raises(RuntimeError, match=r"SNAT entry.*completed: \['VPC', 'instance VSwitch', 'NAT VSwitch', "
                                           r"'NAT gateway', 'elastic IP'\]"):
        b.create()
    assert b.existence() == Existence.IN_COMPLETED
    fake.fail = None
    assert b.create()[0] == "SNAT entry"
    assert b.existence() == Existence.COMPLETED
    assert {v["ZoneId"] for v in fake.vsw.values()} == {"cn-hangzhou-k"}
    assert "DescribeZones" not in {a for _, a in fake.calls}


# ------------------------------------------------------------------------ Huawei Cloud
class FakeHuawei:
    def __init__(self, project="p1"):
        self.p = project
        self.vpcs, self.subnets, self.sgs, self.rules, self.eips, self.nats, self.snat = {}, {}, {}, [], {}, {}, {}
        self.agencies, self.grants = {}, set()
        self.fail = None

    def __call__(self, method, url, params, body):
        params = params or {}
        if self.fail and self.fail in url and method in ("POST", "PUT"):
            raise CloudAPIError(403, f"quota at {url}")
        vpc = f"https://vpc.ap-southeast-1.myhuaweicloud.com/v1/{self.p}"
        nat = f"https://nat.ap-southeast-1.myhuaweicloud.com/v2/{self.p}"
        iam = "https://iam.myhuaweicloud.com"
        path_vpc = url[len(vpc):] if url.startswith(vpc) else None
        path_nat = url[len(nat):] if url.startswith(nat) else None
        path_iam = url[len(iam):] if url.startswith(iam) else None
        if path_vpc is not None:
            return self._vpc(method, path_vpc, params, body)
        if path_nat is not None:
            return self._nat(method, path_nat, params, body)
        if path_iam is not None:
            return self._iam(method, path_iam, params, body)
        raise AssertionError(url)

    def _vpc(self, method, path, params, body):
        if path == "/vpcs" and method == "POST":
            vid = _id("vpc")
            self.vpcs[vid] = dict(body["vpc"], id=vid, status="CREATING")
            return {"vpc": dict(self.vpcs[vid])}
        if path == "/vpcs":
            out = [dict(v) for v in self.vpcs.values()]
            for v in self.vpcs.values():
                v["status"] = "OK"
            return {"vpcs": out}
        if m := re.fullmatch(r"/vpcs/([^/]+)", path):
            vid = m.group(1)
            if any(s["vpc_id"] == vid for s in self.subnets.values()) or \
                    any(g["vpc_id"] == vid for g in self.sgs.values()):
                raise CloudAPIError(409, "VPC.0012 still has dependencies")
            del self.vpcs[vid]
            return {}
        if path == "/subnets" and method == "POST":
            sid = _id("subnet")
            assert body["subnet"]["vpc_id"] in self.vpcs
            self.subnets[sid] = dict(body["subnet"], id=sid, status="UNKNOWN")
            return {"subnet": dict(self.subnets[sid])}
        if path == "/subnets":
            out = [dict(s) for s in self.subnets.values() if s["vpc_id"] == params["vpc_id"]]
            for s in self.subnets.values():
                s["status"] = "ACTIVE"
            return {"subnets": out}
        if m := re.fullmatch(r"/vpcs/([^/]+)/subnets/([^/]+)", path):
            sid = m.group(2)
            if any(n["internal_network_id"] == sid for n in self.nats.values()):
                raise CloudAPIError(409, "subnet in use by a NAT gateway")
            del self.subnets[sid]
            return {}
        if path == "/security-groups" and method == "POST":
            gid = _id("sg")
            self.sgs[gid] = dict(body["security_group"], id=gid)
            return {"security_group": dict(self.sgs[gid])}
        if path == "/security-groups":
            return {"security_groups": [dict(g) for g in self.sgs.values() if g["vpc_id"] == params["vpc_id"]]}
        if path == "/security-group-rules":
            self.rules.append(body["security_group_rule"])
            return {"security_group_rule": body["security_group_rule"]}
        if m := re.fullmatch(r"/security-groups/([^/]+)", path):
            del self.sgs[m.group(1)]
            self.rules = [r for r in self.rules if r["security_group_id"] != m.group(1)]
            return {}
        if path == "/publicips" and method == "POST":
            eid = _id("eip")
            self.eips[eid] = {"id": eid, "bandwidth_name": body["bandwidth"]["name"], "type": body["publicip"]["type"],
                              "public_ip_address": f"119.0.0.{len(self.eips) + 1}"}
            return {"publicip": dict(self.eips[eid])}
        if path == "/publicips":
            return {"publicips": [dict(e) for e in self.eips.values()]}
        if m := re.fullmatch(r"/publicips/([^/]+)", path):
            if any(s["floating_ip_id"] == m.group(1) for s in self.snat.values()):
                raise CloudAPIError(409, "EIP bound to an SNAT rule")
            del self.eips[m.group(1)]
            return {}
        raise AssertionError((method, path))

    def _nat(self, method, path, params, body):
        if path == "/nat_gateways" and method == "POST":
            g = body["nat_gateway"]
            assert g["router_id"] in self.vpcs and g["internal_network_id"] in self.subnets
            nid = _id("nat")
            self.nats[nid] = dict(g, id=nid, status="PENDING_CREATE")
            return {"nat_gateway": dict(self.nats[nid])}
        if path == "/nat_gateways":
            out = [dict(n) for n in self.nats.values() if n["name"] == params["name"]]
            for n in self.nats.values():
                n["status"] = "ACTIVE"
            return {"nat_gateways": out}
        if m := re.fullmatch(r"/nat_gateways/([^/]+)", path):
            if any(s["nat_gateway_id"] == m.group(1) for s in self.snat.values()):
                raise CloudAPIError(409, "NAT gateway has SNAT rules")
            del self.nats[m.group(1)]
            return {}
        if path == "/snat_rules" and method == "POST":
            r = body["snat_rule"]
            assert r["nat_gateway_id"] in self.nats and r["floating_ip_id"] in self.eips
            sid = _id("snat")
            self.snat[sid] = dict(r, id=sid)
            return {"snat_rule": dict(self.snat[sid])}
        if path == "/snat_rules":
            return {"snat_rules": [dict(s) for s in self.snat.values()
                                   if s["nat_gateway_id"] == params["nat_gateway_id"]]}
        if m := re.fullmatch(r"/nat_gateways/([^/]+)/snat_rules/([^/]+)", path):
            del self.snat[m.group(2)]
            return {}
        raise AssertionError((method, path))

    def _iam(self, method, path, params, body):
        if path == "/v3/auth/domains":
            return {"domains": [{"id": "dom1", "name": "acct"}]}
        if path == "/v3/roles":
            return {"roles": [{"id": "role-" + params["display_name"].replace(" ", "_"),
                               "display_name": params["display_name"]}]}
        if path == "/v3.0/OS-AGENCY/agencies" and method == "POST":
            a = body["agency"]
            assert a["trust_domain_name"] == "op_svc_ecs" and a["domain_id"] == "dom1"
            aid = _id("agency")
            self.agencies[aid] = dict(a, id=aid)
            return {"agency": dict(self.agencies[aid])}
        if path == "/v3.0/OS-AGENCY/agencies":
            return {"agencies": [dict(a) for a in self.agencies.values() if a["name"] == params["name"]]}
        if m := re.fullmatch(r"/v3\.0/OS-INHERIT/domains/dom1/agencies/([^/]+)/roles/([^/]+)/inherited_to_projects",
                             path):
            assert method == "PUT" and m.group(1) in self.agencies
            self.grants.add((m.group(1), m.group(2)))
            return {}
        if m := re.fullmatch(r"/v3\.0/OS-AGENCY/agencies/([^/]+)", path):
            del self.agencies[m.group(1)]
            self.grants = {g for g in self.grants if g[0] != m.group(1)}
            return {}
        raise AssertionError((method, path))


def _huawei(fake, obs, **cfg):
    pc = dict(type="huaweicloud", region="ap-southeast-1", project_id="p1", poll_interval_s=0, _transport=fake,
              _object_transport=obs, **cfg)
    return pc, HuaweiCloudWorkspace(pc, "ws2")


def test_huawei_workspace_create_idempotent_delete_keeps_bucket():
    fake, obs = FakeHuawei(), FakeBuckets()
    _, plan = _huawei(fake, obs)
    cfg = {"managed_cloud_storage": True, "allowed_ssh_sources": ["5.6.7.0/24"]}
    b = WorkspaceBuilder(plan.steps(cfg), log=lambda m: None)
    assert b.existence() == Existence.NOT_EXIST
    made = b.create()
    assert made == ["VPC", "subnet", "NAT gateway", "elastic IP", "SNAT rule", "security group", "head agency",
                    "worker agency", "managed OBS bucket"]
    assert b.existence() == Existence.COMPLETED
    assert WorkspaceBuilder(plan.steps(cfg), log=lambda m: None).create() == []
    (sub,) = fake.subnets.values()
    (eip,) = fake.eips.values()
    (nat,) = fake.nats.values()
    (snat,) = fake.snat.values()
    assert sub["cidr"] == "10.0.0.0/20" and sub["gateway_ip"] == "10.0.0.1"
    assert snat["network_id"] == sub["id"] and snat["floating_ip_id"] == eip["id"] and snat["nat_gateway_id"] == nat["id"]
    ssh = [r for r in fake.rules if r.get("port_range_min") == 22]
    assert [r["remote_ip_prefix"] for r in ssh] == ["5.6.7.0/24"]
    assert any(r.get("remote_ip_prefix") == "10.0.0.0/16" and "protocol" not in r for r in fake.rules)
    head = plan._agency("head")["id"]
    worker = plan._agency("worker")["id"]
    assert {g for a, g in fake.grants if a == head} == {"role-ECS_FullAccess", "role-OBS_OperateAccess"}
    assert {g for a, g in fake.grants if a == worker} == {"role-OBS_OperateAccess"}
    assert "<Location>ap-southeast-1</Location>" in obs.buckets[plan.bucket]["config"]
    nc = plan.worker_node_config_defaults()
    assert nc["subnet_id"] == sub["id"] and nc["server"]["metadata"] == {"agency_name": plan.agencies["worker"]}
    gone = b.delete()
    assert gone[0] == "worker agency" and gone[-1] == "VPC"
    assert not (fake.vpcs or fake.subnets or fake.sgs or fake.eips or fake.nats or fake.snat or fake.agencies)
    assert b.status()["managed OBS bucket"]
    obs.buckets[plan.bucket]["objects"].add("x")
    b.delete(delete_managed_storage=True)
    assert not obs.buckets


def test_huawei_failed_step_is_resumable():
    fake, obs = FakeHuawei(), FakeBuckets()
    _, plan = _huawei(fake, obs, domain_id="dom1")
    fake.fail = "/nat_gateways"
    b = WorkspaceBuilder(plan.steps({}), log=lambda m: None)
    with pytest.raises(RuntimeError, match=r"NAT gateway.*completed: \['VPC', 'subnet'\]"):
        b.create()
    assert b.existence() == Existence.IN_COMPLETED
    fake.fail = None
    assert b.create()[:2] == ["NAT gateway", "elastic IP"]
    assert b.existence() == Existence.COMPLETED


# ------------------------------------------------------------------------ providers
@pytest.mark.parametrize("cloud", ["aliyun", "huaweicloud"])
def test_workspace_and_storage_providers_drive_the_plans(cloud, tmp_path, monkeypatch):
    import cloudtik_amd.providers.cloud.workspace_provider as cwp
    import cloudtik_amd.providers.local.workspace_provider as lwp
    from cloudtik_amd.providers.cloud.storage_provider import CloudDatabaseProvider, CloudStorageProvider
    monkeypatch.setattr(lwp, "STATE_DIR", str(tmp_path))
    store = FakeBuckets()
    pc, _ = _aliyun(FakeAliyun(), store) if cloud == "aliyun" else _huawei(FakeHuawei(), store)
    wp = cwp.CloudWorkspaceProvider(pc, "ws1" if cloud == "aliyun" else "ws2")
    config = {"workspace_name": wp.workspace_name, "provider": pc}
    assert wp.check_workspace_existence(config) == Existence.NOT_EXIST
    wp.create_workspace(config)
    assert wp.check_workspace_integrity(config)
    assert wp.get_workspace_info(config)["resources"]["vpc"].startswith("vpc-")
    sp = CloudStorageProvider(pc, wp.workspace_name, "bucket")
    assert not sp.get_info({"provider": pc})["exists"]
    sp.create({"provider": pc})
    info = sp.get_info({"provider": pc})
    assert info["exists"] and info["bucket"] in store.buckets
    with pytest.raises(NotImplementedError, match="mysql or postgres"):
        CloudDatabaseProvider(pc, wp.workspace_name, "db").create({"provider": pc})
    wp.delete_workspace(config)
    assert wp.check_workspace_existence(config) == Existence.NOT_EXIST and store.buckets
    sp.delete({"provider": pc})
    assert not store.buckets


def test_object_store_signature():
    """OSS / OBS header signature: HMAC-SHA1 over VERB, MD5, type, date, sorted vendor
    headers and the canonical resource (subresources only)."""
    import base64
    import hashlib
    import hmac
    assert canonical_resource("bk", "", "list-type=2&max-keys=1000") == "/bk/"
    assert canonical_resource("bk", "k/o", "tagging") == "/bk/k/o?tagging"
    h = {"Date": "Tue, 01 Oct 2024 00:00:00 GMT", "Content-Type": "application/xml", "x-oss-meta-b": "2",
         "X-OSS-Meta-A": " 1 "}
    want = "PUT\n\napplication/xml\nTue, 01 Oct 2024 00:00:00 GMT\nx-oss-meta-a:1\nx-oss-meta-b:2\n/bk/?tagging"
    ref = base64.b64encode(hmac.new(b"secret", want.encode(), hashlib.sha1).digest()).decode()
    assert object_store_sign("OSS", "PUT", "/bk/?tagging", h, "secret") == ref
    # OBS signs x-obs-* headers, not x-oss-*
    assert object_store_sign("OBS", "PUT", "/bk/?tagging", h, "secret") != ref
