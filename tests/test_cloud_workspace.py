"""Cloud workspaces (providers/cloud/workspace.py): GCP and Azure step plans against in-memory
fakes of their REST APIs, AWS against fake boto3 clients -- create is complete and idempotent,
a failed step leaves a resumable IN_COMPLETED workspace, delete runs in reverse and keeps the
managed bucket / database unless asked, IAM / role bindings follow the identities, and the
workspace / storage / database providers drive the same plans (reference
providers/_private/{gcp,_azure,aws}/config.py create/delete/check workspace)."""
import itertools
import re

import pytest

from cloudtik_amd.core.workspace import Existence
from cloudtik_amd.providers.cloud.rest_providers import CloudAPIError
from cloudtik_amd.providers.cloud.workspace import (AWSWorkspace, AzureWorkspace, GCPWorkspace,
                                                     WorkspaceBuilder)


# ------------------------------------------------------------------------------ GCP fake
class FakeGCP:
    def __init__(self, project="proj"):
        self.project = project
        self.items = {}
        self.ops = 0
        self.policy = {"bindings": []}
        self.connections = []
        self.fail = None
        self.calls = []

    def _op(self):
        self.ops += 1
        link = f"https://compute.googleapis.com/compute/v1/projects/{self.project}/global/operations/op{self.ops}"
        self.items[link] = {"status": "DONE", "selfLink": link}
        return {"status": "RUNNING", "selfLink": link, "name": f"op{self.ops}"}

    def __call__(self, method, url, params, body):
        self.calls.append((method, url))
        if self.fail and self.fail in url and method in ("POST", "PUT"):
            raise CloudAPIError(403, f"quota exceeded at {url}")
        if url.endswith(":getIamPolicy"):
            return {"bindings": [dict(b, members=list(b["members"])) for b in self.policy["bindings"]]}
        if url.endswith(":setIamPolicy"):
            self.policy = body["policy"]
            return self.policy
        if "servicenetworking" in url:
            if method == "GET":
                return {"connections": [dict(c) for c in self.connections]}
            if url.endswith(":deleteConnection"):
                self.connections = []
                return {}
            self.connections.append({"network": body["network"], "reservedPeeringRanges": body["reservedPeeringRanges"]})
            return {}
        if method == "GET":
            if url not in self.items:
                raise CloudAPIError(404, url)
            return self.items[url]
        if method == "DELETE":
            if url not in self.items:
                raise CloudAPIError(404, url)
            del self.items[url]
            return self._op()
        if method == "POST":
            if url.endswith("/serviceAccounts"):
                name = f"{body['accountId']}@{self.project}.iam.gserviceaccount.com"
            else:
                name = body["name"]
            self.items[f"{url}/{name}"] = dict(body)
            return self._op()
        raise AssertionError((method, url))


def _gcp(fake, **cfg):
    pc = dict(type="gcp", project_id="proj", region="us-central1", poll_interval_s=0, **cfg)
    return GCPWorkspace(pc, "ws1", fake)


def test_gcp_workspace_create_idempotent_delete_keeps_managed():
    fake = FakeGCP()
    plan = _gcp(fake, database={"engine_version": "MYSQL_8_0"})
    config = {"managed_cloud_storage": True, "managed_cloud_database": True, "allowed_ssh_sources": ["1.2.3.4/32"]}
    b = WorkspaceBuilder(plan.steps(config), log=lambda m: None)
    assert b.existence() == Existence.NOT_EXIST
    made = b.create()
    assert made[0] == "VPC network" and "managed database" in made and len(made) == len(b.steps)
    assert b.existence() == Existence.COMPLETED and all(b.status().values())
    assert WorkspaceBuilder(plan.steps(config), log=lambda m: None).create() == []       # idempotent
    fw = fake.items[f"https://compute.googleapis.com/compute/v1/projects/proj/global/firewalls/{plan.firewalls['ssh']}"]
    assert fw["sourceRanges"] == ["1.2.3.4/32"] and fw["allowed"][0]["ports"] == ["22"]
    router = fake.items[f"https://compute.googleapis.com/compute/v1/projects/proj/regions/us-central1/routers/"
                        f"{plan.router}"]
    assert router["nats"][0]["subnetworks"][0]["name"].endswith(plan.subnets["private"])
    head = "serviceAccount:" + plan._sa_email("head")
    roles = {b["role"] for b in fake.policy["bindings"] if head in b["members"]}
    assert roles == set(GCPWorkspace.HEAD_ROLES)
    sql = fake.items[f"https://sqladmin.googleapis.com/v1/projects/proj/instances/{plan.db}"]
    assert sql["settings"]["ipConfiguration"]["privateNetwork"].endswith(plan.vpc)
    # delete: managed bucket and database stay by default
    gone = b.delete()
    assert "VPC network" in gone and "managed bucket" not in gone and "managed database" not in gone
    assert b.existence() == Existence.NOT_EXIST
    st = b.status()
    assert st["managed bucket"] and st["managed database"] and not st["VPC network"]
    assert not any(head in bb["members"] for bb in fake.policy["bindings"])               # bindings removed
    b.delete(delete_managed_storage=True, delete_managed_database=True)
    assert not any(b.status().values())


def test_gcp_failed_step_is_resumable():
    fake = FakeGCP()
    fake.fail = "/routers"
    b = WorkspaceBuilder(_gcp(fake).steps({}), log=lambda m: None)
    with pytest.raises(RuntimeError, match=r"router \+ NAT.*completed: \['VPC network', 'private subnet', "
                                           r"'public subnet'\]"):
        b.create()
    assert b.existence() == Existence.IN_COMPLETED
    fake.fail = None
    assert b.create()[0] == "router + NAT"
    assert b.existence() == Existence.COMPLETED


# ------------------------------------------------------------------------------ Azure fake
class FakeARM:
    def __init__(self):
        self.items = {}
        self.polls = 0
        self.ids = itertools.count(1)

    def __call__(self, method, url, params, body):
        assert params and "api-version" in params
        if method == "GET":
            if url not in self.items:
                raise CloudAPIError(404, url)
            it = self.items[url]
            if it.get("properties", {}).get("provisioningState") == "Updating":
                self.polls += 1
                it["properties"]["provisioningState"] = "Succeeded"
            return it
        if method == "PUT":
            item = dict(body)
            props = dict(item.get("properties", {}))
            if "/resourcegroups/" not in url.lower() or "/providers/" in url:
                props["provisioningState"] = "Updating"
            if "userAssignedIdentities" in url:
                props["principalId"] = f"principal-{next(self.ids)}"
            item["properties"] = props
            self.items[url] = item
            return item
        if method == "DELETE":
            if url not in self.items:
                raise CloudAPIError(404, url)
            for k in [k for k in self.items if k == url or k.startswith(url + "/")]:
                del self.items[k]
            return {}
        raise AssertionError(method)


def test_azure_workspace_create_and_delete():
    fake = FakeARM()
    plan = AzureWorkspace({"type": "azure", "subscription_id": "sub", "location": "westus2", "poll_interval_s": 0},
                          "ws2", fake)
    b = WorkspaceBuilder(plan.steps({"managed_cloud_storage": True, "allowed_ssh_sources": ["10.9.0.0/16"]}),
                         log=lambda m: None)
    b.create()
    assert b.existence() == Existence.COMPLETED and fake.polls > 0
    sub = next(v for k, v in fake.items.items() if k.endswith(plan.subnets["private"]))
    assert sub["properties"]["natGateway"]["id"].endswith(f"natGateways/{plan.nat}")
    assert sub["properties"]["networkSecurityGroup"]["id"].endswith(f"networkSecurityGroups/{plan.nsg}")
    nsg = next(v for k, v in fake.items.items() if k.endswith(f"networkSecurityGroups/{plan.nsg}"))
    assert nsg["properties"]["securityRules"][0]["properties"]["sourceAddressPrefixes"] == ["10.9.0.0/16"]
    assigns = [v for k, v in fake.items.items() if "roleAssignments" in k]
    assert len(assigns) == 3 and {a["properties"]["principalId"] for a in assigns} == {"principal-1", "principal-2"}
    acct = next(v for k, v in fake.items.items() if k.endswith(f"storageAccounts/{plan.account}"))
    assert acct["properties"]["isHnsEnabled"] is True and re.fullmatch(r"[a-z0-9]{3,24}", plan.account)
    b.create()                                                     # idempotent: no duplicate assignments
    assert len([k for k in fake.items if "roleAssignments" in k]) == 3
    b.delete(delete_managed_storage=True)
    assert b.existence() == Existence.NOT_EXIST and not fake.items


# ------------------------------------------------------------------------------ AWS fakes
class NoSuchEntityException(Exception):
    pass


class DBInstanceNotFoundFault(Exception):
    pass


class FakeAWS:
    def __init__(self):
        self.n = itertools.count(1)
        self.res = {}          # id -> dict(kind, tags, ...)
        self.roles, self.profiles, self.buckets, self.dbs, self.subnet_groups = {}, {}, set(), {}, set()

    def client(self, svc):
        return self

    def _new(self, kind, tagspec=None, **kw):
        rid = f"{kind}-{next(self.n)}"
        tags = {t["Key"]: t["Value"] for t in (tagspec[0]["Tags"] if tagspec else [])}
        self.res[rid] = dict(kind=kind, tags=tags, **kw)
        return rid

    def _find(self, kind, Filters=None, **kw):
        out = []
        for rid, r in self.res.items():
            if r["kind"] != kind:
                continue
            ok = True
            for f in Filters or []:
                if f["Name"].startswith("tag:"):
                    ok &= r["tags"].get(f["Name"][4:]) in f["Values"]
                elif f["Name"] == "state":
                    ok &= r.get("state", "available") in f["Values"]
            if ok:
                out.append((rid, r))
        return out

    # ec2
    def create_vpc(self, CidrBlock, TagSpecifications):
        return {"Vpc": {"VpcId": self._new("vpc", TagSpecifications, cidr=CidrBlock)}}

    def describe_vpcs(self, Filters):
        return {"Vpcs": [{"VpcId": i} for i, _ in self._find("vpc", Filters)]}

    def delete_vpc(self, VpcId):
        assert not [r for r in self.res.values() if r.get("vpc") == VpcId], "VPC still has dependencies"
        del self.res[VpcId]

    def create_internet_gateway(self, TagSpecifications):
        return {"InternetGateway": {"InternetGatewayId": self._new("igw", TagSpecifications)}}

    def attach_internet_gateway(self, InternetGatewayId, VpcId):
        self.res[InternetGatewayId]["vpc"] = VpcId

    def describe_internet_gateways(self, Filters):
        return {"InternetGateways": [{"InternetGatewayId": i} for i, _ in self._find("igw", Filters)]}

    def detach_internet_gateway(self, InternetGatewayId, VpcId):
        self.res[InternetGatewayId].pop("vpc")

    def delete_internet_gateway(self, InternetGatewayId):
        del self.res[InternetGatewayId]

    def create_subnet(self, VpcId, CidrBlock, TagSpecifications):
        return {"Subnet": {"SubnetId": self._new("subnet", TagSpecifications, vpc=VpcId, cidr=CidrBlock)}}

    def modify_subnet_attribute(self, SubnetId, MapPublicIpOnLaunch):
        self.res[SubnetId]["public_ip"] = MapPublicIpOnLaunch["Value"]

    def describe_subnets(self, Filters):
        return {"Subnets": [{"SubnetId": i} for i, _ in self._find("subnet", Filters)]}

    def delete_subnet(self, SubnetId):
        del self.res[SubnetId]

    def allocate_address(self, Domain, TagSpecifications):
        return {"AllocationId": self._new("eip", TagSpecifications)}

    def release_address(self, AllocationId):
        del self.res[AllocationId]

    def create_nat_gateway(self, SubnetId, AllocationId, TagSpecifications):
        return {"NatGateway": {"NatGatewayId": self._new("nat", TagSpecifications, subnet=SubnetId,
                                                         alloc=AllocationId, state="available")}}

    def describe_nat_gateways(self, Filters):
        return {"NatGateways": [{"NatGatewayId": i, "NatGatewayAddresses": [{"AllocationId": r["alloc"]}]}
                                for i, r in self._find("nat", Filters)]}

    def delete_nat_gateway(self, NatGatewayId):
        del self.res[NatGatewayId]

    def create_route_table(self, VpcId, TagSpecifications):
        return {"RouteTable": {"RouteTableId": self._new("rtb", TagSpecifications, vpc=VpcId, routes=[],
                                                         assoc=[])}}

    def create_route(self, RouteTableId, DestinationCidrBlock, **target):
        self.res[RouteTableId]["routes"].append(dict(target, dst=DestinationCidrBlock))

    def associate_route_table(self, RouteTableId, SubnetId):
        self.res[RouteTableId]["assoc"].append(SubnetId)

    def describe_route_tables(self, Filters=None, RouteTableIds=None):
        rows = self._find("rtb", Filters) if Filters else [(i, self.res[i]) for i in RouteTableIds]
        return {"RouteTables": [{"RouteTableId": i, "Associations": [
            {"RouteTableAssociationId": f"{i}|{s}", "Main": False} for s in r["assoc"]]} for i, r in rows]}

    def disassociate_route_table(self, AssociationId):
        rtb, s = AssociationId.split("|")
        self.res[rtb]["assoc"].remove(s)

    def delete_route_table(self, RouteTableId):
        assert not self.res[RouteTableId]["assoc"]
        del self.res[RouteTableId]

    def create_security_group(self, GroupName, Description, VpcId, TagSpecifications):
        return {"GroupId": self._new("sg", TagSpecifications, vpc=VpcId, rules=[])}

    def authorize_security_group_ingress(self, GroupId, IpPermissions):
        self.res[GroupId]["rules"] += IpPermissions

    def describe_security_groups(self, Filters):
        return {"SecurityGroups": [{"GroupId": i} for i, _ in self._find("sg", Filters)]}

    def delete_security_group(self, GroupId):
        del self.res[GroupId]

    # iam
    def get_role(self, RoleName):
        if RoleName not in self.roles:
            raise NoSuchEntityException(RoleName)
        return {"Role": {"RoleName": RoleName}}

    def create_role(self, RoleName, AssumeRolePolicyDocument, Tags):
        self.roles[RoleName] = set()

    def attach_role_policy(self, RoleName, PolicyArn):
        self.roles[RoleName].add(PolicyArn)

    def detach_role_policy(self, RoleName, PolicyArn):
        self.roles[RoleName].remove(PolicyArn)

    def delete_role(self, RoleName):
        assert not self.roles[RoleName]
        del self.roles[RoleName]

    def create_instance_profile(self, InstanceProfileName):
        self.profiles[InstanceProfileName] = set()

    def add_role_to_instance_profile(self, InstanceProfileName, RoleName):
        self.profiles[InstanceProfileName].add(RoleName)

    def remove_role_from_instance_profile(self, InstanceProfileName, RoleName):
        self.profiles[InstanceProfileName].remove(RoleName)

    def delete_instance_profile(self, InstanceProfileName):
        del self.profiles[InstanceProfileName]

    # s3 / rds
    def head_bucket(self, Bucket):
        if Bucket not in self.buckets:
            raise Exception("An error occurred (404) when calling the HeadBucket operation: Not Found")

    def create_bucket(self, Bucket, **kw):
        self.buckets.add(Bucket)

    def delete_bucket(self, Bucket):
        self.buckets.remove(Bucket)

    def describe_db_instances(self, DBInstanceIdentifier):
        if DBInstanceIdentifier not in self.dbs:
            raise DBInstanceNotFoundFault(DBInstanceIdentifier)
        return {"DBInstances": [self.dbs[DBInstanceIdentifier]]}

    def create_db_subnet_group(self, DBSubnetGroupName, DBSubnetGroupDescription, SubnetIds):
        assert all(SubnetIds)
        self.subnet_groups.add(DBSubnetGroupName)

    def create_db_instance(self, **kw):
        self.dbs[kw["DBInstanceIdentifier"]] = kw

    def delete_db_instance(self, DBInstanceIdentifier, SkipFinalSnapshot):
        del self.dbs[DBInstanceIdentifier]

    def delete_db_subnet_group(self, DBSubnetGroupName):
        self.subnet_groups.remove(DBSubnetGroupName)


def test_aws_workspace_create_and_delete():
    fake = FakeAWS()
    plan = AWSWorkspace({"type": "aws", "region": "us-west-2"}, "ws3", fake.client)
    cfg = {"managed_cloud_storage": True, "managed_cloud_database": True}
    b = WorkspaceBuilder(plan.steps(cfg), log=lambda m: None)
    b.create()
    assert b.existence() == Existence.COMPLETED
    pub, priv = plan._rtb("public"), plan._rtb("private")
    assert fake.res[pub]["routes"][0]["GatewayId"] == plan._igw()
    assert fake.res[priv]["routes"][0]["NatGatewayId"] == plan._nat()["NatGatewayId"]
    assert fake.res[plan._subnet("public")]["public_ip"] is True
    assert fake.dbs[plan.db]["VpcSecurityGroupIds"] == [plan._sg()]
    assert fake.profiles[plan.roles["head"]] == {plan.roles["head"]}
    assert WorkspaceBuilder(plan.steps(cfg), log=lambda m: None).create() == []
    b.delete(delete_managed_storage=True, delete_managed_database=True)
    assert not fake.res and not fake.roles and not fake.profiles and not fake.buckets and not fake.dbs


# ------------------------------------------------------------------------------ providers
def test_workspace_and_storage_providers_drive_the_plans(tmp_path, monkeypatch):
    import cloudtik_amd.providers.local.workspace_provider as lwp
    import cloudtik_amd.providers.cloud.workspace_provider as cwp
    monkeypatch.setattr(lwp, "STATE_DIR", str(tmp_path))
    from cloudtik_amd.providers.cloud.storage_provider import CloudDatabaseProvider, CloudStorageProvider
    fake = FakeGCP()
    pc = {"type": "gcp", "project_id": "proj", "region": "us-central1", "poll_interval_s": 0, "_transport": fake}
    wp = cwp.CloudWorkspaceProvider(pc, "ws4")
    config = {"workspace_name": "ws4", "provider": pc}
    assert wp.check_workspace_existence(config) == Existence.NOT_EXIST
    wp.create_workspace(config)
    assert wp.check_workspace_integrity(config)
    info = wp.get_workspace_info(config)
    assert info["resources"]["vpc"] == "cloudtik-ws4-vpc"
    sp = CloudStorageProvider(pc, "ws4", "bucket")
    sp.create({"provider": pc})
    assert sp.get_info({"provider": pc})["exists"]
    assert [s for s in fake.items if "/storage/v1/b/" in s]
    dp = CloudDatabaseProvider(pc, "ws4", "db")
    assert not dp.get_info({"provider": pc})["exists"]
    wp.delete_workspace(config)
    assert wp.check_workspace_existence(config) == Existence.NOT_EXIST
    assert [s for s in fake.items if "/storage/v1/b/" in s]                # the managed bucket survives
    sp.delete({"provider": pc})
    assert not [s for s in fake.items if "/storage/v1/b/" in s]
    # existing-network workspaces only set up the registry
    pc2 = dict(pc, use_working_vpc=True)
    n_calls = len(fake.calls)
    cwp.CloudWorkspaceProvider(pc2, "ws5").create_workspace({"provider": pc2})
    assert len(fake.calls) == n_calls
