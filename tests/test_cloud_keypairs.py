"""SSH key-pair bootstrap on the five clouds (providers/cloud/keypairs.py; reference
aws/config.py:3868, gcp/config.py:2678,3478, _azure/config.py:4068, aliyun/config.py:2153,
huaweicloud/config.py:1876) against fake cloud APIs: the key pair is created (or reused) once,
its private key lands in ~/.ssh with mode 0600, every node type's launch request carries the
key, and the SSH executor the updater uses passes that private key."""
import copy
import os
import stat

import pytest

from cloudtik_amd.core import tags as T
from cloudtik_amd.providers.cloud import keypairs


@pytest.fixture(autouse=True)
def home(tmp_path, monkeypatch):
    monkeypatch.setenv("HOME", str(tmp_path))
    return tmp_path


def _cfg(provider, node_config=None, **auth):
    nc = node_config or {}
    return {"cluster_name": "c1", "provider": provider, "auth": dict({"ssh_user": "ubuntu"}, **auth),
            "available_node_types": {"head.default": {"node_config": dict(nc)},
                                     "worker.gpu": {"node_config": dict(nc)}}}


class NotFound(Exception):
    def __init__(self):
        super().__init__("not found")
        self.response = {"Error": {"Code": "InvalidKeyPair.NotFound"}}


class FakeEC2:
    def __init__(self, existing=()):
        self.keys = set(existing)
        self.created, self.run = [], []

    def describe_key_pairs(self, KeyNames):
        if KeyNames[0] not in self.keys:
            raise NotFound()
        return {"KeyPairs": [{"KeyName": KeyNames[0]}]}

    def create_key_pair(self, KeyName):
        self.keys.add(KeyName)
        self.created.append(KeyName)
        return {"KeyName": KeyName, "KeyMaterial": f"-----BEGIN RSA PRIVATE KEY-----\n{KeyName}\n"}

    def describe_instances(self, **kw):
        return {"Reservations": []}

    def run_instances(self, **kw):
        self.run.append(kw)
        return {"Instances": [{"InstanceId": "i-1", "State": {"Name": "pending"}, "Tags": [],
                               "PrivateIpAddress": "10.0.0.1"}]}


def _ssh_key_of(cfg):
    from cloudtik_amd.core.executor import SSHCommandExecutor
    ex = SSHCommandExecutor(None, "", "n1", None, cfg["auth"], "c1", None, True)
    opts = ex.ssh_options.to_ssh_options_list()
    return opts[opts.index("-i") + 1]


def test_aws_creates_key_pair_once_and_launches_with_it(home):
    from cloudtik_amd.providers.cloud.node_provider import AWSNodeProvider
    ec2 = FakeEC2()
    pc = {"type": "aws", "region": "us-west-2", "_client_factory": lambda svc: ec2}
    cfg = AWSNodeProvider.bootstrap_config(_cfg(pc))
    key = cfg["auth"]["ssh_private_key"]
    assert ec2.created == ["cloudtik_aws_us-west-2"] and key == str(home / ".ssh" / "cloudtik_aws_us-west-2.pem")
    assert stat.S_IMODE(os.stat(key).st_mode) == 0o600
    assert all(nt["node_config"]["KeyName"] == "cloudtik_aws_us-west-2" for nt in cfg["available_node_types"].values())
    # the launch request carries the key; the updater's SSH uses the private half
    p = AWSNodeProvider(pc, "c1")
    p.create_node(cfg["available_node_types"]["worker.gpu"]["node_config"], {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 1)
    assert ec2.run[-1]["KeyName"] == "cloudtik_aws_us-west-2"
    assert _ssh_key_of(cfg) == key
    # a second bootstrap reuses the pair (cloud + local file both present)
    cfg2 = AWSNodeProvider.bootstrap_config(_cfg(pc))
    assert ec2.created == ["cloudtik_aws_us-west-2"] and cfg2["auth"]["ssh_private_key"] == key


def test_aws_skips_names_owned_elsewhere_and_checks_explicit_keys(home):
    from cloudtik_amd.providers.cloud.node_provider import AWSNodeProvider
    ec2 = FakeEC2(existing={"cloudtik_aws_r1"})          # in the cloud, but no local private key
    pc = {"type": "aws", "region": "r1", "_client_factory": lambda svc: ec2}
    cfg = AWSNodeProvider.bootstrap_config(_cfg(pc))
    assert ec2.created == ["cloudtik_aws_r1_1"]
    assert cfg["available_node_types"]["head.default"]["node_config"]["KeyName"] == "cloudtik_aws_r1_1"
    # explicit private key: every node type must name its key pair (or bring UserData)
    with pytest.raises(ValueError, match="KeyName"):
        AWSNodeProvider.bootstrap_config(_cfg(pc, ssh_private_key="~/.ssh/mine.pem"))
    ok = AWSNodeProvider.bootstrap_config(_cfg(pc, {"KeyName": "mine"}, ssh_private_key="~/.ssh/mine.pem"))
    assert ok["auth"]["ssh_private_key"] == "~/.ssh/mine.pem"


def test_aliyun_key_pair_via_signed_api(home):
    from cloudtik_amd.providers.cloud.signed_providers import AliyunNodeProvider
    calls = []
    keys = set()

    def transport(action, params):
        calls.append((action, dict(params)))
        if action == "DescribeKeyPairs":
            return {"KeyPairs": {"KeyPair": [{"KeyPairName": n} for n in keys if n == params["KeyPairName"]]}}
        if action == "CreateKeyPair":
            keys.add(params["KeyPairName"])
            return {"PrivateKeyBody": "ALIYUN-PRIVATE"}
        if action == "RunInstances":
            return {"InstanceIdSets": {"InstanceIdSet": ["i-a"]}}
        return {}

    pc = {"type": "aliyun", "region": "cn-hangzhou", "_transport": transport, "cache_stopped_nodes": False}
    cfg = AliyunNodeProvider.bootstrap_config(_cfg(pc))
    name = "cloudtik_aliyun_cn-hangzhou"
    assert open(cfg["auth"]["ssh_private_key"]).read().strip() == "ALIYUN-PRIVATE"
    AliyunNodeProvider(pc, "c1").create_node(cfg["available_node_types"]["worker.gpu"]["node_config"],
                                             {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 1)
    run = [p for a, p in calls if a == "RunInstances"][-1]
    assert run["KeyPairName"] == name


def test_huaweicloud_key_pair_via_kps(home):
    from cloudtik_amd.providers.cloud.rest_providers import CloudAPIError
    from cloudtik_amd.providers.cloud.signed_providers import HuaweiCloudNodeProvider
    calls = []
    keys = set()

    def transport(method, url, params, body):
        calls.append((method, url, body))
        if "/keypairs/" in url and method == "GET":
            name = url.rsplit("/", 1)[1]
            if name not in keys:
                raise CloudAPIError(404, "keypair not found")
            return {"keypair": {"name": name}}
        if url.endswith("/keypairs") and method == "POST":
            keys.add(body["keypair"]["name"])
            return {"keypair": {"name": body["keypair"]["name"], "private_key": "HW-PRIVATE"}}
        if "cloudservers" in url and method == "POST":
            return {"serverIds": ["s-1"]}
        return {}

    pc = {"type": "huaweicloud", "region": "cn-north-4", "project_id": "p1", "_transport": transport}
    cfg = HuaweiCloudNodeProvider.bootstrap_config(_cfg(pc))
    assert cfg["available_node_types"]["head.default"]["node_config"]["key_name"] == "cloudtik_huaweicloud_cn-north-4"
    assert any("kps.cn-north-4.myhuaweicloud.com/v3/p1/keypairs" in u for _, u, _ in calls)
    HuaweiCloudNodeProvider(pc, "c1").create_node(cfg["available_node_types"]["worker.gpu"]["node_config"],
                                                  {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 1)
    server = [b for m, u, b in calls if m == "POST" and "cloudservers" in u][-1]["server"]
    assert server["key_name"] == "cloudtik_huaweicloud_cn-north-4"


def test_gcp_public_key_in_instance_metadata(home):
    from cloudtik_amd.providers.cloud.rest_providers import GCPNodeProvider
    bodies = []

    def transport(method, url, params, body):
        if method == "POST" and url.endswith("/instances"):
            bodies.append(body)
            return {"name": "op", "status": "DONE"}
        return {"name": url.rsplit("/", 1)[-1], "status": "RUNNING"}

    pc = {"type": "gcp", "project_id": "proj", "availability_zone": "us-central1-a", "region": "us-central1",
          "_transport": transport}
    cfg = GCPNodeProvider.bootstrap_config(_cfg(pc))
    priv = cfg["auth"]["ssh_private_key"]
    pub = open(priv + ".pub").read().split()
    assert stat.S_IMODE(os.stat(priv).st_mode) == 0o600
    items = cfg["available_node_types"]["worker.gpu"]["node_config"]["metadata"]["items"]
    assert {"key": "ssh-keys", "value": f"ubuntu:{pub[0]} {pub[1]} ubuntu"} in items
    # idempotent: bootstrapping the bootstrapped config adds no second copy
    again = GCPNodeProvider.bootstrap_config(copy.deepcopy(cfg))
    assert again["available_node_types"]["worker.gpu"]["node_config"]["metadata"]["items"] == items
    GCPNodeProvider(pc, "c1").create_node(cfg["available_node_types"]["worker.gpu"]["node_config"],
                                          {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 1)
    assert any(i["key"] == "ssh-keys" for i in bodies[-1]["metadata"]["items"])
    assert _ssh_key_of(cfg) == priv


def test_azure_public_key_in_os_profile(home):
    from cloudtik_amd.providers.cloud.rest_providers import AzureNodeProvider
    pc = {"type": "azure", "subscription_id": "s", "resource_group": "rg", "location": "eastus", "subnet_id": "sn",
          "_transport": lambda *a: {"id": "x"}}
    cfg = AzureNodeProvider.bootstrap_config(_cfg(pc, {"azure_arm_parameters": {"vmSize": "Standard_ND96isr_MI300X_v5"}}))
    pub = open(cfg["auth"]["ssh_private_key"] + ".pub").read().strip()
    osp = cfg["available_node_types"]["head.default"]["node_config"]["properties"]["osProfile"]
    assert osp["adminUsername"] == "ubuntu" and osp["linuxConfiguration"]["disablePasswordAuthentication"]
    assert osp["linuxConfiguration"]["ssh"]["publicKeys"][0]["keyData"] == pub
    assert cfg["available_node_types"]["head.default"]["node_config"]["azure_arm_parameters"]["publicKey"] == pub


def test_key_pair_names():
    assert keypairs.key_pair_name("aws", "r", 0)[0] == "cloudtik_aws_r"
    assert keypairs.key_pair_name("aws", "r", 2)[0] == "cloudtik_aws_r_2"
    assert keypairs.key_pair_name("aws", "r", 1, "team")[0] == "team_key-1"
