"""Cloud workspaces: the network, identity, storage and database resources a workspace's
clusters run in (reference providers/_private/gcp/config.py:254-2330,
providers/_private/_azure/config.py, providers/_private/aws/config.py -- create / delete /
check of VPC, subnets, router + NAT, firewalls, service accounts / managed identities / IAM
roles, the managed bucket and the managed database).

A workspace is an ordered list of ``Step``s.  Each step knows how to tell whether its
resource exists, how to create it and how to delete it; ``WorkspaceBuilder`` creates the
missing steps in order (idempotent: re-running ``cloudtik workspace create`` after a failure
continues where it stopped), deletes the existing ones in reverse order, and reports
existence as NOT_EXIST / IN_COMPLETED / COMPLETED -- the same contract as the reference's
``check_workspace_existence``.  Managed storage / database steps are part of the plan only
when ``managed_cloud_storage`` / ``managed_cloud_database`` are set, and deletion keeps them
unless asked.

Clouds:
* GCP over REST (Compute, IAM, Cloud Resource Manager, Cloud Storage, Cloud SQL admin,
  Service Networking) -- the same bearer-token transport as the GCP node provider;
* Azure over ARM REST (resource group, VNet, NSG, NAT gateway + public IP, subnets,
  user-assigned identities + role assignments, ADLS Gen2 storage account + container,
  MySQL flexible server);
* AWS over boto3 clients (VPC, subnets, internet gateway, NAT gateway, route tables,
  security group, IAM roles + instance profiles, S3 bucket, RDS instance);
* Aliyun and Huawei Cloud over their signed HTTP APIs (providers/cloud/signed_workspace.py:
  VPC, VSwitch / subnet, NAT gateway + EIP + SNAT, security group, RAM roles / IAM agencies,
  OSS / OBS bucket).
"""
from __future__ import annotations

import hashlib
import time
import uuid
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional

from cloudtik_amd.providers.cloud.rest_providers import CloudAPIError


@dataclass
class Step:
    name: str
    exists: Callable[[], bool]
    create: Callable[[], None]
    delete: Callable[[], None]
    managed: str = ""          # "" | "storage" | "database": optional, kept on delete by default


class WorkspaceBuilder:
    def __init__(self, steps: List[Step], log: Callable[[str], None] = print):
        self.steps = steps
        self.log = log

    def create(self) -> List[str]:
        made = []
        n = len(self.steps)
        for i, s in enumerate(self.steps, 1):
            if s.exists():
                self.log(f"[{i}/{n}] {s.name}: exists")
                continue
            self.log(f"[{i}/{n}] creating {s.name}")
            try:
                s.create()
            except Exception as e:
                raise RuntimeError(f"workspace step '{s.name}' failed ({e}); completed: {made}. "
                                   "Fix the cause and run the create again: finished steps are skipped") from e
            made.append(s.name)
        return made

    def delete(self, delete_managed_storage: bool = False, delete_managed_database: bool = False) -> List[str]:
        gone = []
        steps = list(reversed(self.steps))
        n = len(steps)
        for i, s in enumerate(steps, 1):
            if (s.managed == "storage" and not delete_managed_storage) or \
                    (s.managed == "database" and not delete_managed_database):
                self.log(f"[{i}/{n}] {s.name}: kept (managed {s.managed})")
                continue
            if not s.exists():
                continue
            self.log(f"[{i}/{n}] deleting {s.name}")
            s.delete()
            gone.append(s.name)
        return gone

    def status(self) -> Dict[str, bool]:
        return {s.name: bool(s.exists()) for s in self.steps}

    def existence(self):
        from cloudtik_amd.core.workspace import Existence
        core = [v for s, v in zip(self.steps, self.status().values()) if not s.managed]
        if core and all(core):
            return Existence.COMPLETED
        return Existence.IN_COMPLETED if any(core) else Existence.NOT_EXIST


def _missing(call: Callable[[], Any]) -> bool:
    """True when the GET raises a 404."""
    try:
        call()
        return False
    except CloudAPIError as e:
        if e.status == 404:
            return True
        raise


def _name(ws: str, suffix: str, limit: int = 63) -> str:
    n = f"cloudtik-{ws}-{suffix}".lower()
    return n[:limit]


def _cidr(cfg: Dict[str, Any], key: str, default: str) -> str:
    return cfg.get(key, default)


# =============================================================================== GCP
_GCE = "https://compute.googleapis.com/compute/v1"
_IAM = "https://iam.googleapis.com/v1"
_CRM = "https://cloudresourcemanager.googleapis.com/v1"
_GCS = "https://storage.googleapis.com/storage/v1"
_SQL = "https://sqladmin.googleapis.com/v1"
_SN = "https://servicenetworking.googleapis.com/v1"


class GCPWorkspace:
    """Steps: VPC -> private / public subnets -> router with NAT -> firewalls -> head / worker
    service accounts (+ project role bindings) -> [bucket] -> [private service connection +
    Cloud SQL instance]."""

    HEAD_ROLES = ("roles/storage.admin", "roles/compute.admin", "roles/iam.serviceAccountUser")
    WORKER_ROLES = ("roles/storage.admin",)

    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, call, poll_s: float = 2.0):
        self.cfg = provider_config
        self.ws = workspace_name
        self.project = provider_config["project_id"]
        self.region = provider_config["region"]
        self.call = call
        self.poll_s = float(provider_config.get("poll_interval_s", poll_s))
        self.vpc = _name(workspace_name, "vpc")
        self.subnets = {"private": _name(workspace_name, "private-subnet"),
                        "public": _name(workspace_name, "public-subnet")}
        self.router = _name(workspace_name, "router")
        self.nat = _name(workspace_name, "nat")
        self.firewalls = {"internal": _name(workspace_name, "allow-internal"),
                          "ssh": _name(workspace_name, "allow-ssh")}
        self.sa = {"head": f"cloudtik-{workspace_name}-head"[:30], "worker": f"cloudtik-{workspace_name}-worker"[:30]}
        self.bucket = _name(workspace_name, "bucket-" + hashlib.sha1(self.project.encode()).hexdigest()[:8])
        self.db = _name(workspace_name, "db")
        self.address = _name(workspace_name, "psa")

    # ---------------------------------------------------------------- helpers
    def _wait(self, op: Dict[str, Any], timeout_s: float = 1800.0):
        if not isinstance(op, dict) or "status" not in op or "selfLink" not in op:
            return op
        deadline = time.time() + timeout_s
        while op.get("status") != "DONE":
            if time.time() > deadline:
                raise CloudAPIError(504, f"operation {op.get('name')} timed out")
            time.sleep(self.poll_s)
            op = self.call("GET", op["selfLink"], None, None)
        if op.get("error"):
            raise CloudAPIError(400, str(op["error"])[:500])
        return op

    def _p(self, path: str) -> str:
        return f"{_GCE}/projects/{self.project}/{path}"

    def _vpc_link(self) -> str:
        return self._p(f"global/networks/{self.vpc}")

    def _sa_email(self, role: str) -> str:
        return f"{self.sa[role]}@{self.project}.iam.gserviceaccount.com"

    # ---------------------------------------------------------------- steps
    def _subnet_step(self, kind: str, cidr: str) -> Step:
        name = self.subnets[kind]
        url = self._p(f"regions/{self.region}/subnetworks/{name}")
        body = {"name": name, "network": self._vpc_link(), "ipCidrRange": cidr,
                "privateIpGoogleAccess": kind == "private"}
        return Step(f"{kind} subnet", lambda: not _missing(lambda: self.call("GET", url, None, None)),
                    lambda: self._wait(self.call("POST", self._p(f"regions/{self.region}/subnetworks"), None, body)),
                    lambda: self._wait(self.call("DELETE", url, None, None)))

    def _firewall_step(self, kind: str, body: Dict[str, Any]) -> Step:
        name = self.firewalls[kind]
        url = self._p(f"global/firewalls/{name}")
        body = dict(body, name=name, network=self._vpc_link())
        return Step(f"firewall {kind}", lambda: not _missing(lambda: self.call("GET", url, None, None)),
                    lambda: self._wait(self.call("POST", self._p("global/firewalls"), None, body)),
                    lambda: self._wait(self.call("DELETE", url, None, None)))

    def _router_exists(self) -> bool:
        return not _missing(lambda: self.call("GET", self._p(f"regions/{self.region}/routers/{self.router}"),
                                              None, None))

    def _create_router(self):
        body = {"name": self.router, "network": self._vpc_link(),
                "nats": [{"name": self.nat, "natIpAllocateOption": "AUTO_ONLY",
                          "sourceSubnetworkIpRangesToNat": "LIST_OF_SUBNETWORKS",
                          "subnetworks": [{"name": self._p(f"regions/{self.region}/subnetworks/"
                                                           f"{self.subnets['private']}"),
                                           "sourceIpRangesToNat": ["ALL_IP_RANGES"]}]}]}
        self._wait(self.call("POST", self._p(f"regions/{self.region}/routers"), None, body))

    def _sa_step(self, role: str) -> Step:
        url = f"{_IAM}/projects/{self.project}/serviceAccounts/{self._sa_email(role)}"

        def create():
            self.call("POST", f"{_IAM}/projects/{self.project}/serviceAccounts", None,
                      {"accountId": self.sa[role],
                       "serviceAccount": {"displayName": f"CloudTik {self.ws} {role}"}})
            roles = self.HEAD_ROLES if role == "head" else self.WORKER_ROLES
            self._bind(f"serviceAccount:{self._sa_email(role)}", roles, add=True)

        def delete():
            roles = self.HEAD_ROLES if role == "head" else self.WORKER_ROLES
            self._bind(f"serviceAccount:{self._sa_email(role)}", roles, add=False)
            self.call("DELETE", url, None, None)
        return Step(f"{role} service account", lambda: not _missing(lambda: self.call("GET", url, None, None)),
                    create, delete)

    def _bind(self, member: str, roles, add: bool):
        url = f"{_CRM}/projects/{self.project}"
        policy = self.call("POST", url + ":getIamPolicy", None, {})
        bindings = policy.setdefault("bindings", [])
        for role in roles:
            b = next((x for x in bindings if x["role"] == role), None)
            if add:
                if b is None:
                    bindings.append({"role": role, "members": [member]})
                elif member not in b["members"]:
                    b["members"].append(member)
            elif b is not None and member in b["members"]:
                b["members"].remove(member)
        policy["bindings"] = [b for b in bindings if b["members"]]
        self.call("POST", url + ":setIamPolicy", None, {"policy": policy})

    def _db_steps(self) -> List[Step]:
        addr_url = self._p(f"global/addresses/{self.address}")
        conn_url = f"{_SN}/services/servicenetworking.googleapis.com/connections"
        db_url = f"{_SQL}/projects/{self.project}/instances/{self.db}"
        dbc = self.cfg.get("database", {})

        def conn_exists():
            out = self.call("GET", conn_url, {"network": f"projects/{self.project}/global/networks/{self.vpc}"}, None)
            return any(self.address in c.get("reservedPeeringRanges", []) for c in out.get("connections", []))

        def create_db():
            body = {"name": self.db, "region": self.region,
                    "databaseVersion": dbc.get("engine_version", "MYSQL_8_0"),
                    "rootPassword": dbc.get("admin_password") or uuid.uuid4().hex,
                    "settings": {"tier": dbc.get("instance_type", "db-custom-4-15360"),
                                 "dataDiskSizeGb": str(dbc.get("storage_size", 50)),
                                 "availabilityType": "REGIONAL" if dbc.get("high_availability") else "ZONAL",
                                 "ipConfiguration": {"ipv4Enabled": False,
                                                     "privateNetwork": f"projects/{self.project}/global/"
                                                                       f"networks/{self.vpc}"}}}
            self._wait(self.call("POST", f"{_SQL}/projects/{self.project}/instances", None, body))
        return [
            Step("private service address", lambda: not _missing(lambda: self.call("GET", addr_url, None, None)),
                 lambda: self._wait(self.call("POST", self._p("global/addresses"), None,
                                              {"name": self.address, "purpose": "VPC_PEERING", "addressType":
                                               "INTERNAL", "prefixLength": 16, "network": self._vpc_link()})),
                 lambda: self._wait(self.call("DELETE", addr_url, None, None)), managed="database"),
            Step("private service connection", conn_exists,
                 lambda: self.call("POST", conn_url, None,
                                   {"network": f"projects/{self.project}/global/networks/{self.vpc}",
                                    "reservedPeeringRanges": [self.address]}),
                 lambda: self.call("POST", f"{_SN}/services/servicenetworking.googleapis.com/connections/"
                                           f"servicenetworking-googleapis-com:deleteConnection", None,
                                   {"consumerNetwork": f"projects/{self.project}/global/networks/{self.vpc}"}),
                 managed="database"),
            Step("managed database", lambda: not _missing(lambda: self.call("GET", db_url, None, None)),
                 create_db, lambda: self._wait(self.call("DELETE", db_url, None, None)), managed="database"),
        ]

    def steps(self, config: Dict[str, Any]) -> List[Step]:
        ssh_sources = config.get("allowed_ssh_sources") or self.cfg.get("allowed_ssh_sources") or ["0.0.0.0/0"]
        out = [
            Step("VPC network", lambda: not _missing(lambda: self.call("GET", self._vpc_link(), None, None)),
                 lambda: self._wait(self.call("POST", self._p("global/networks"), None,
                                              {"name": self.vpc, "autoCreateSubnetworks": False,
                                               "routingConfig": {"routingMode": "REGIONAL"}})),
                 lambda: self._wait(self.call("DELETE", self._vpc_link(), None, None))),
            self._subnet_step("private", _cidr(self.cfg, "private_subnet_cidr", "10.0.0.0/16")),
            self._subnet_step("public", _cidr(self.cfg, "public_subnet_cidr", "10.1.0.0/16")),
            Step("router + NAT", self._router_exists, self._create_router,
                 lambda: self._wait(self.call("DELETE", self._p(f"regions/{self.region}/routers/{self.router}"),
                                              None, None))),
            self._firewall_step("internal", {"sourceRanges": ["10.0.0.0/8"],
                                             "allowed": [{"IPProtocol": "tcp"}, {"IPProtocol": "udp"},
                                                         {"IPProtocol": "icmp"}]}),
            self._firewall_step("ssh", {"sourceRanges": list(ssh_sources),
                                        "allowed": [{"IPProtocol": "tcp", "ports": ["22"]}]}),
            self._sa_step("head"),
            self._sa_step("worker"),
        ]
        if config.get("managed_cloud_storage"):
            burl = f"{_GCS}/b/{self.bucket}"
            out.append(Step("managed bucket", lambda: not _missing(lambda: self.call("GET", burl, None, None)),
                            lambda: self.call("POST", f"{_GCS}/b", {"project": self.project},
                                              {"name": self.bucket, "location": self.region,
                                               "iamConfiguration": {"uniformBucketLevelAccess": {"enabled": True}}}),
                            lambda: self.call("DELETE", burl, None, None), managed="storage"))
        if config.get("managed_cloud_database"):
            out += self._db_steps()
        return out

    def info(self) -> Dict[str, Any]:
        return {"vpc": self.vpc, "subnets": dict(self.subnets), "router": self.router,
                "service_accounts": {k: self._sa_email(k) for k in self.sa}, "bucket": self.bucket,
                "database": self.db}


# =============================================================================== Azure
_ARM = "https://management.azure.com"
_API = {"resources": "2021-04-01", "network": "2023-04-01", "identity": "2023-01-31",
        "authorization": "2022-04-01", "storage": "2023-01-01", "mysql": "2023-06-30"}
ROLE_CONTRIBUTOR = "b24988ac-6180-42a0-ab88-20f7382dd24c"
ROLE_STORAGE_BLOB_OWNER = "b7e6dc6d-f1e8-4753-8033-0f276bb0955b"


class AzureWorkspace:
    """Steps: resource group -> VNet -> NSG -> NAT public IP -> NAT gateway -> private /
    public subnets -> head / worker user-assigned identities (+ role assignments) ->
    [ADLS Gen2 account + container] -> [MySQL flexible server]."""

    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, call, poll_s: float = 5.0):
        self.cfg = provider_config
        self.ws = workspace_name
        self.sub = provider_config["subscription_id"]
        self.rg = provider_config.get("resource_group") or f"cloudtik-{workspace_name}-rg"
        self.location = provider_config.get("location", "eastus")
        self.call = call
        self.poll_s = float(provider_config.get("poll_interval_s", poll_s))
        self.vnet = f"cloudtik-{workspace_name}-vnet"
        self.nsg = f"cloudtik-{workspace_name}-nsg"
        self.nat_ip = f"cloudtik-{workspace_name}-nat-ip"
        self.nat = f"cloudtik-{workspace_name}-nat"
        self.subnets = {"private": f"cloudtik-{workspace_name}-private-subnet",
                        "public": f"cloudtik-{workspace_name}-public-subnet"}
        self.identities = {"head": f"cloudtik-{workspace_name}-head-identity",
                           "worker": f"cloudtik-{workspace_name}-worker-identity"}
        h = hashlib.sha1(f"{self.sub}/{workspace_name}".encode()).hexdigest()[:10]
        self.account = ("cloudtik" + "".join(c for c in workspace_name.lower() if c.isalnum()))[:14] + h
        self.container = f"cloudtik-{workspace_name}"
        self.db = f"cloudtik-{workspace_name}-db"

    def _rg(self, path: str = "") -> str:
        return f"{_ARM}/subscriptions/{self.sub}/resourceGroups/{self.rg}{path}"

    def _res(self, provider: str, path: str) -> str:
        return self._rg(f"/providers/{provider}/{path}")

    def _get(self, url: str, api: str):
        return self.call("GET", url, {"api-version": _API[api]}, None)

    def _put(self, url: str, api: str, body: Dict[str, Any], wait: bool = True):
        out = self.call("PUT", url, {"api-version": _API[api]}, body)
        if wait:
            deadline = time.time() + 1800
            while (out or {}).get("properties", {}).get("provisioningState") not in (None, "Succeeded"):
                if out["properties"]["provisioningState"] in ("Failed", "Canceled"):
                    raise CloudAPIError(400, f"{url}: {out['properties']['provisioningState']}")
                if time.time() > deadline:
                    raise CloudAPIError(504, f"{url}: provisioning timed out")
                time.sleep(self.poll_s)
                out = self._get(url, api)
        return out

    def _del(self, url: str, api: str):
        try:
            self.call("DELETE", url, {"api-version": _API[api]}, None)
        except CloudAPIError as e:
            if e.status != 404:
                raise

    def _step(self, name: str, url: str, api: str, body_fn: Callable[[], Dict[str, Any]], managed: str = "",
              after_create: Optional[Callable[[], None]] = None, before_delete: Optional[Callable[[], None]] = None):
        def create():
            self._put(url, api, body_fn())
            if after_create:
                after_create()

        def delete():
            if before_delete:
                before_delete()
            self._del(url, api)
        return Step(name, lambda: not _missing(lambda: self._get(url, api)), create, delete, managed)

    def _id(self, provider: str, path: str) -> str:
        return f"/subscriptions/{self.sub}/resourceGroups/{self.rg}/providers/{provider}/{path}"

    def _assign(self, identity_url: str, roles, scope: str):
        principal = self._get(identity_url, "identity")["properties"]["principalId"]
        for role in roles:
            # deterministic assignment name: re-running create does not duplicate it
            aid = str(uuid.uuid5(uuid.NAMESPACE_URL, f"{scope}|{principal}|{role}"))
            self.call("PUT", f"{_ARM}{scope}/providers/Microsoft.Authorization/roleAssignments/{aid}",
                      {"api-version": _API["authorization"]},
                      {"properties": {"roleDefinitionId": f"/subscriptions/{self.sub}/providers/"
                                                          f"Microsoft.Authorization/roleDefinitions/{role}",
                                      "principalId": principal, "principalType": "ServicePrincipal"}})

    def steps(self, config: Dict[str, Any]) -> List[Step]:
        ssh_sources = config.get("allowed_ssh_sources") or self.cfg.get("allowed_ssh_sources") or ["*"]
        loc = self.location
        scope = f"/subscriptions/{self.sub}/resourceGroups/{self.rg}"
        net = "Microsoft.Network"
        out = [
            Step("resource group", lambda: not _missing(lambda: self._get(self._rg(), "resources")),
                 lambda: self._put(self._rg(), "resources", {"location": loc}, wait=False),
                 lambda: self._del(self._rg(), "resources")),
            self._step("virtual network", self._res(net, f"virtualNetworks/{self.vnet}"), "network",
                       lambda: {"location": loc, "properties": {"addressSpace": {"addressPrefixes": [
                           self.cfg.get("vnet_cidr", "10.0.0.0/16")]}}}),
            self._step("network security group", self._res(net, f"networkSecurityGroups/{self.nsg}"), "network",
                       lambda: {"location": loc, "properties": {"securityRules": [
                           {"name": "allow-ssh", "properties": {
                               "priority": 1000, "access": "Allow", "direction": "Inbound", "protocol": "Tcp",
                               "sourceAddressPrefixes": list(ssh_sources), "sourcePortRange": "*",
                               "destinationAddressPrefix": "*", "destinationPortRange": "22"}},
                           {"name": "allow-vnet", "properties": {
                               "priority": 1010, "access": "Allow", "direction": "Inbound", "protocol": "*",
                               "sourceAddressPrefix": "VirtualNetwork", "sourcePortRange": "*",
                               "destinationAddressPrefix": "VirtualNetwork", "destinationPortRange": "*"}}]}}),
            self._step("NAT public IP", self._res(net, f"publicIPAddresses/{self.nat_ip}"), "network",
                       lambda: {"location": loc, "sku": {"name": "Standard"},
                                "properties": {"publicIPAllocationMethod": "Static"}}),
            self._step("NAT gateway", self._res(net, f"natGateways/{self.nat}"), "network",
                       lambda: {"location": loc, "sku": {"name": "Standard"}, "properties": {
                           "publicIpAddresses": [{"id": self._id(net, f"publicIPAddresses/{self.nat_ip}")}]}}),
        ]
        for kind, cidr in (("private", "10.0.0.0/17"), ("public", "10.0.128.0/17")):
            props = {"addressPrefix": self.cfg.get(f"{kind}_subnet_cidr", cidr),
                     "networkSecurityGroup": {"id": self._id(net, f"networkSecurityGroups/{self.nsg}")}}
            if kind == "private":
                props["natGateway"] = {"id": self._id(net, f"natGateways/{self.nat}")}
            out.append(self._step(f"{kind} subnet",
                                  self._res(net, f"virtualNetworks/{self.vnet}/subnets/{self.subnets[kind]}"),
                                  "network", lambda p=props: {"properties": p}))
        for role, roles in (("head", (ROLE_CONTRIBUTOR, ROLE_STORAGE_BLOB_OWNER)),
                            ("worker", (ROLE_STORAGE_BLOB_OWNER,))):
            url = self._res("Microsoft.ManagedIdentity", f"userAssignedIdentities/{self.identities[role]}")
            out.append(self._step(f"{role} identity", url, "identity", lambda: {"location": loc},
                                  after_create=lambda u=url, r=roles: self._assign(u, r, scope)))
        if config.get("managed_cloud_storage"):
            acct = self._res("Microsoft.Storage", f"storageAccounts/{self.account}")
            out.append(self._step("managed storage account", acct, "storage",
                                  lambda: {"location": loc, "kind": "StorageV2", "sku": {"name": "Standard_LRS"},
                                           "properties": {"isHnsEnabled": True, "minimumTlsVersion": "TLS1_2"}},
                                  managed="storage"))
            out.append(self._step("managed storage container",
                                  f"{acct}/blobServices/default/containers/{self.container}", "storage",
                                  lambda: {"properties": {}}, managed="storage"))
        if config.get("managed_cloud_database"):
            dbc = self.cfg.get("database", {})
            out.append(self._step("managed database", self._res("Microsoft.DBforMySQL", f"flexibleServers/{self.db}"),
                                  "mysql", lambda: {
                                      "location": loc,
                                      "sku": {"name": dbc.get("instance_type", "Standard_D4ds_v4"),
                                              "tier": "GeneralPurpose"},
                                      "properties": {"administratorLogin": dbc.get("admin_user", "cloudtik"),
                                                     "administratorLoginPassword": dbc.get("admin_password")
                                                     or uuid.uuid4().hex + "Aa1!",
                                                     "version": "8.0.21",
                                                     "storage": {"storageSizeGB": dbc.get("storage_size", 50)},
                                                     "highAvailability": {"mode": "ZoneRedundant" if
                                                                          dbc.get("high_availability") else
                                                                          "Disabled"}}},
                                  managed="database"))
        return out

    def info(self) -> Dict[str, Any]:
        return {"resource_group": self.rg, "vnet": self.vnet, "subnets": dict(self.subnets),
                "identities": dict(self.identities), "storage_account": self.account, "database": self.db}


# =============================================================================== AWS
class AWSWorkspace:
    """Steps: VPC -> internet gateway -> public / private subnets -> NAT gateway (+ EIP) ->
    route tables -> security group -> head / worker IAM roles + instance profiles ->
    [S3 bucket] -> [DB subnet group + RDS instance].  Resources carry the tag
    ``cloudtik-workspace=<name>`` and are found by it."""

    TAG = "cloudtik-workspace"

    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, client_factory=None):
        self.cfg = provider_config
        self.ws = workspace_name
        self.region = provider_config["region"]
        if client_factory is None:
            import boto3
            client_factory = lambda svc: boto3.client(svc, region_name=self.region)  # noqa: E731
        self.ec2 = client_factory("ec2")
        self.iam = client_factory("iam")
        self.s3 = client_factory("s3")
        self.rds = client_factory("rds")
        self.bucket = f"cloudtik-{workspace_name}-{hashlib.sha1(self.region.encode()).hexdigest()[:8]}"
        self.db = f"cloudtik-{workspace_name}-db"
        self.roles = {"head": f"cloudtik-{workspace_name}-head-role", "worker": f"cloudtik-{workspace_name}-worker-role"}

    def _tags(self, kind: str):
        return [{"ResourceType": kind, "Tags": [{"Key": self.TAG, "Value": self.ws},
                                               {"Key": "Name", "Value": f"cloudtik-{self.ws}-{kind}"}]}]

    def _filters(self, extra=None):
        return [{"Name": f"tag:{self.TAG}", "Values": [self.ws]}] + list(extra or [])

    def _vpc_id(self) -> Optional[str]:
        v = self.ec2.describe_vpcs(Filters=self._filters())["Vpcs"]
        return v[0]["VpcId"] if v else None

    def _subnet(self, kind: str) -> Optional[str]:
        s = self.ec2.describe_subnets(Filters=self._filters([{"Name": "tag:cloudtik-subnet", "Values": [kind]}]))
        return s["Subnets"][0]["SubnetId"] if s["Subnets"] else None

    def _igw(self) -> Optional[str]:
        g = self.ec2.describe_internet_gateways(Filters=self._filters())["InternetGateways"]
        return g[0]["InternetGatewayId"] if g else None

    def _nat(self) -> Optional[Dict[str, Any]]:
        n = self.ec2.describe_nat_gateways(Filters=self._filters([{"Name": "state",
                                                                  "Values": ["pending", "available"]}]))
        return n["NatGateways"][0] if n["NatGateways"] else None

    def _rtb(self, kind: str) -> Optional[str]:
        r = self.ec2.describe_route_tables(Filters=self._filters([{"Name": "tag:cloudtik-subnet",
                                                                   "Values": [kind]}]))["RouteTables"]
        return r[0]["RouteTableId"] if r else None

    def _sg(self) -> Optional[str]:
        g = self.ec2.describe_security_groups(Filters=self._filters())["SecurityGroups"]
        return g[0]["GroupId"] if g else None

    def _create_subnet(self, kind: str, cidr: str):
        tags = self._tags("subnet")
        tags[0]["Tags"].append({"Key": "cloudtik-subnet", "Value": kind})
        sid = self.ec2.create_subnet(VpcId=self._vpc_id(), CidrBlock=cidr, TagSpecifications=tags)["Subnet"]["SubnetId"]
        if kind == "public":
            self.ec2.modify_subnet_attribute(SubnetId=sid, MapPublicIpOnLaunch={"Value": True})

    def _create_nat(self):
        alloc = self.ec2.allocate_address(Domain="vpc", TagSpecifications=self._tags("elastic-ip"))["AllocationId"]
        self.ec2.create_nat_gateway(SubnetId=self._subnet("public"), AllocationId=alloc,
                                    TagSpecifications=self._tags("natgateway"))

    def _delete_nat(self):
        n = self._nat()
        self.ec2.delete_nat_gateway(NatGatewayId=n["NatGatewayId"])
        for a in n.get("NatGatewayAddresses", []):
            if a.get("AllocationId"):
                self.ec2.release_address(AllocationId=a["AllocationId"])

    def _create_rtb(self, kind: str):
        tags = self._tags("route-table")
        tags[0]["Tags"].append({"Key": "cloudtik-subnet", "Value": kind})
        rtb = self.ec2.create_route_table(VpcId=self._vpc_id(), TagSpecifications=tags)["RouteTable"]["RouteTableId"]
        if kind == "public":
            self.ec2.create_route(RouteTableId=rtb, DestinationCidrBlock="0.0.0.0/0", GatewayId=self._igw())
        else:
            self.ec2.create_route(RouteTableId=rtb, DestinationCidrBlock="0.0.0.0/0",
                                  NatGatewayId=self._nat()["NatGatewayId"])
        self.ec2.associate_route_table(RouteTableId=rtb, SubnetId=self._subnet(kind))

    def _delete_rtb(self, kind: str):
        rtb = self._rtb(kind)
        for a in self.ec2.describe_route_tables(RouteTableIds=[rtb])["RouteTables"][0].get("Associations", []):
            if not a.get("Main"):
                self.ec2.disassociate_route_table(AssociationId=a["RouteTableAssociationId"])
        self.ec2.delete_route_table(RouteTableId=rtb)

    def _create_sg(self, ssh_sources):
        gid = self.ec2.create_security_group(GroupName=f"cloudtik-{self.ws}-sg", Description="CloudTik workspace",
                                             VpcId=self._vpc_id(), TagSpecifications=self._tags("security-group"))[
            "GroupId"]
        self.ec2.authorize_security_group_ingress(GroupId=gid, IpPermissions=[
            {"IpProtocol": "tcp", "FromPort": 22, "ToPort": 22, "IpRanges": [{"CidrIp": c} for c in ssh_sources]},
            {"IpProtocol": "-1", "UserIdGroupPairs": [{"GroupId": gid}]}])

    def _role_exists(self, role: str) -> bool:
        try:
            self.iam.get_role(RoleName=self.roles[role])
            return True
        except Exception as e:                          # botocore NoSuchEntity
            if "NoSuchEntity" in type(e).__name__ or "NoSuchEntity" in str(e):
                return False
            raise

    def _create_role(self, role: str, policies):
        import json as _json
        trust = {"Version": "2012-10-17", "Statement": [{"Effect": "Allow", "Principal": {"Service":
                                                                                          "ec2.amazonaws.com"},
                                                         "Action": "sts:AssumeRole"}]}
        name = self.roles[role]
        self.iam.create_role(RoleName=name, AssumeRolePolicyDocument=_json.dumps(trust),
                             Tags=[{"Key": self.TAG, "Value": self.ws}])
        for p in policies:
            self.iam.attach_role_policy(RoleName=name, PolicyArn=f"arn:aws:iam::aws:policy/{p}")
        self.iam.create_instance_profile(InstanceProfileName=name)
        self.iam.add_role_to_instance_profile(InstanceProfileName=name, RoleName=name)

    def _delete_role(self, role: str, policies):
        name = self.roles[role]
        self.iam.remove_role_from_instance_profile(InstanceProfileName=name, RoleName=name)
        self.iam.delete_instance_profile(InstanceProfileName=name)
        for p in policies:
            self.iam.detach_role_policy(RoleName=name, PolicyArn=f"arn:aws:iam::aws:policy/{p}")
        self.iam.delete_role(RoleName=name)

    def _bucket_exists(self) -> bool:
        try:
            self.s3.head_bucket(Bucket=self.bucket)
            return True
        except Exception as e:
            if "404" in str(e) or "NoSuchBucket" in str(e) or "Not Found" in str(e):
                return False
            raise

    def _db_exists(self) -> bool:
        try:
            return bool(self.rds.describe_db_instances(DBInstanceIdentifier=self.db)["DBInstances"])
        except Exception as e:
            if "DBInstanceNotFound" in type(e).__name__ or "DBInstanceNotFound" in str(e):
                return False
            raise

    def _create_db(self):
        dbc = self.cfg.get("database", {})
        self.rds.create_db_subnet_group(DBSubnetGroupName=self.db, DBSubnetGroupDescription="CloudTik workspace",
                                        SubnetIds=[self._subnet("private"), self._subnet("public")])
        self.rds.create_db_instance(DBInstanceIdentifier=self.db, Engine=dbc.get("engine", "mysql"),
                                    DBInstanceClass=dbc.get("instance_type", "db.t3.xlarge"),
                                    AllocatedStorage=int(dbc.get("storage_size", 50)),
                                    MasterUsername=dbc.get("admin_user", "cloudtik"),
                                    MasterUserPassword=dbc.get("admin_password") or uuid.uuid4().hex,
                                    DBSubnetGroupName=self.db, VpcSecurityGroupIds=[self._sg()],
                                    MultiAZ=bool(dbc.get("high_availability")), PubliclyAccessible=False,
                                    Tags=[{"Key": self.TAG, "Value": self.ws}])

    def _delete_db(self):
        self.rds.delete_db_instance(DBInstanceIdentifier=self.db, SkipFinalSnapshot=True)
        self.rds.delete_db_subnet_group(DBSubnetGroupName=self.db)

    def steps(self, config: Dict[str, Any]) -> List[Step]:
        ssh = config.get("allowed_ssh_sources") or self.cfg.get("allowed_ssh_sources") or ["0.0.0.0/0"]
        head_pol = ("AmazonEC2FullAccess", "AmazonS3FullAccess", "IAMReadOnlyAccess")
        worker_pol = ("AmazonS3FullAccess",)
        out = [
            Step("VPC", lambda: self._vpc_id() is not None,
                 lambda: self.ec2.create_vpc(CidrBlock=self.cfg.get("vpc_cidr", "10.0.0.0/16"),
                                             TagSpecifications=self._tags("vpc")),
                 lambda: self.ec2.delete_vpc(VpcId=self._vpc_id())),
            Step("internet gateway", lambda: self._igw() is not None,
                 lambda: self.ec2.attach_internet_gateway(
                     InternetGatewayId=self.ec2.create_internet_gateway(TagSpecifications=self._tags(
                         "internet-gateway"))["InternetGateway"]["InternetGatewayId"], VpcId=self._vpc_id()),
                 lambda: (self.ec2.detach_internet_gateway(InternetGatewayId=self._igw(), VpcId=self._vpc_id()),
                          self.ec2.delete_internet_gateway(InternetGatewayId=self._igw()))),
            Step("public subnet", lambda: self._subnet("public") is not None,
                 lambda: self._create_subnet("public", self.cfg.get("public_subnet_cidr", "10.0.0.0/20")),
                 lambda: self.ec2.delete_subnet(SubnetId=self._subnet("public"))),
            Step("private subnet", lambda: self._subnet("private") is not None,
                 lambda: self._create_subnet("private", self.cfg.get("private_subnet_cidr", "10.0.16.0/20")),
                 lambda: self.ec2.delete_subnet(SubnetId=self._subnet("private"))),
            Step("NAT gateway", lambda: self._nat() is not None, self._create_nat, self._delete_nat),
            Step("public route table", lambda: self._rtb("public") is not None,
                 lambda: self._create_rtb("public"), lambda: self._delete_rtb("public")),
            Step("private route table", lambda: self._rtb("private") is not None,
                 lambda: self._create_rtb("private"), lambda: self._delete_rtb("private")),
            Step("security group", lambda: self._sg() is not None, lambda: self._create_sg(ssh),
                 lambda: self.ec2.delete_security_group(GroupId=self._sg())),
            Step("head role", lambda: self._role_exists("head"), lambda: self._create_role("head", head_pol),
                 lambda: self._delete_role("head", head_pol)),
            Step("worker role", lambda: self._role_exists("worker"), lambda: self._create_role("worker", worker_pol),
                 lambda: self._delete_role("worker", worker_pol)),
        ]
        if config.get("managed_cloud_storage"):
            kw = {} if self.region == "us-east-1" else {
                "CreateBucketConfiguration": {"LocationConstraint": self.region}}
            out.append(Step("managed bucket", self._bucket_exists,
                            lambda: self.s3.create_bucket(Bucket=self.bucket, **kw),
                            lambda: self.s3.delete_bucket(Bucket=self.bucket), managed="storage"))
        if config.get("managed_cloud_database"):
            out.append(Step("managed database", self._db_exists, self._create_db, self._delete_db,
                            managed="database"))
        return out

    def info(self) -> Dict[str, Any]:
        return {"vpc": self._vpc_id(), "roles": dict(self.roles), "bucket": self.bucket, "database": self.db}


def cloud_workspace(provider_config: Dict[str, Any], workspace_name: str, transport=None):
    """The step plan object for ``provider_config['type']``."""
    t = provider_config.get("type")
    if t == "gcp":
        from cloudtik_amd.providers.cloud.rest_providers import GCPNodeProvider, requests_transport
        call = transport or provider_config.get("_transport")
        if call is None:
            tok = GCPNodeProvider.__new__(GCPNodeProvider)
            tok.provider_config = provider_config
            call = requests_transport(tok._token)
        return GCPWorkspace(provider_config, workspace_name, call)
    if t == "azure":
        from cloudtik_amd.providers.cloud.rest_providers import AzureNodeProvider, requests_transport
        call = transport or provider_config.get("_transport")
        if call is None:
            tok = AzureNodeProvider.__new__(AzureNodeProvider)
            tok.provider_config = provider_config
            call = requests_transport(tok._token)
        return AzureWorkspace(provider_config, workspace_name, call)
    if t == "aws":
        return AWSWorkspace(provider_config, workspace_name, transport or provider_config.get("_client_factory"))
    if t == "aliyun":
        from cloudtik_amd.providers.cloud.signed_workspace import AliyunWorkspace
        return AliyunWorkspace(provider_config, workspace_name, transport)
    if t == "huaweicloud":
        from cloudtik_amd.providers.cloud.signed_workspace import HuaweiCloudWorkspace
        return HuaweiCloudWorkspace(provider_config, workspace_name, transport)
    if t == "kubernetes":
        from cloudtik_amd.providers.kubernetes.workspace import Kubectl, KubernetesWorkspace
        kubectl = provider_config.get("_kubectl") or Kubectl(provider_config.get("kubectl"))
        return KubernetesWorkspace(provider_config, workspace_name, kubectl,
                                   transport or provider_config.get("_cloud_transport"))
    return None
