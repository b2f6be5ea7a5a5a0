"""GCP and Azure node providers (providers/cloud/rest_providers.py) against in-memory fakes
of the Compute Engine and ARM REST APIs: the node-provider contract end to end (create,
list with tag filters, tags round trip, IPs, terminate) with the request shapes each API
expects.  No network: the transport is injected."""
import re

import pytest

from cloudtik_amd.core import tags as T
from cloudtik_amd.providers.cloud.rest_providers import (AzureNodeProvider, CloudAPIError, GCPNodeProvider,
                                                         gcp_label)


class FakeGCE:
    """instances.{list,get,insert,delete,setLabels,setMetadata} + zoneOperations.get."""

    def __init__(self):
        self.instances, self.ops, self.calls, self.n = {}, {}, [], 0

    def _op(self, done=False):
        self.n += 1
        op = {"name": f"op-{self.n}", "status": "DONE" if done else "RUNNING"}
        self.ops[op["name"]] = dict(op, status="DONE")
        return op

    def __call__(self, method, url, params, body):
        self.calls.append((method, url, params, body))
        m = re.match(r".*/projects/(?P<p>[^/]+)/zones/(?P<z>[^/]+)/(?P<rest>.*)$", url)
        assert m and m["p"] == "proj" and m["z"] == "us-central1-a", url
        rest = m["rest"].split("/")
        if rest[0] == "operations":
            return self.ops[rest[1]]
        if len(rest) == 1 and method == "GET":
            flt = params["filter"]
            want = dict(re.findall(r'labels\.([a-z0-9_-]+) = "([a-z0-9_-]*)"', flt))
            items = [i for i in self.instances.values()
                     if all(i["labels"].get(k) == v for k, v in want.items())]
            return {"items": items}
        if len(rest) == 1 and method == "POST":
            assert body["machineType"].startswith("zones/us-central1-a/machineTypes/")
            for k, v in body["labels"].items():
                assert k == gcp_label(k) and v == gcp_label(v)
            self.instances[body["name"]] = dict(body, status="RUNNING", labelFingerprint="f0",
                                                networkInterfaces=[{"networkIP": f"10.0.0.{len(self.instances) + 2}",
                                                                    "accessConfigs": [{"natIP": "34.1.2.3"}]}])
            self.instances[body["name"]]["metadata"] = dict(body.get("metadata", {}), fingerprint="m0")
            return self._op()
        name = rest[1]
        if name not in self.instances:
            raise CloudAPIError(404, "not found")
        inst = self.instances[name]
        if len(rest) == 2 and method == "GET":
            return inst
        if len(rest) == 2 and method == "DELETE":
            del self.instances[name]
            return self._op(done=True)
        if rest[2] == "setLabels":
            assert body["labelFingerprint"] == inst["labelFingerprint"]
            inst["labels"] = body["labels"]
            return self._op()
        if rest[2] == "setMetadata":
            assert body["fingerprint"] == inst["metadata"]["fingerprint"]
            inst["metadata"] = {"items": body["items"], "fingerprint": "m1"}
            return self._op()
        raise AssertionError(url)


class FakeARM:
    """virtualMachines / networkInterfaces / publicIPAddresses PUT, GET, PATCH, DELETE."""

    def __init__(self):
        self.res, self.calls = {}, []

    def __call__(self, method, url, params, body):
        self.calls.append((method, url, params, body))
        assert params is None or "api-version" in params
        m = re.match(r".*/subscriptions/sub/resourceGroups/rg/providers/(?P<prov>[^/]+)/(?P<kind>[^/]+)"
                     r"(?:/(?P<name>[^/]+))?(?P<iv>/instanceView)?$", url)
        assert m, url
        kind, name = m["kind"], m["name"]
        if name is None:
            return {"value": [r for (k, _), r in self.res.items() if k == kind]}
        key = (kind, name)
        if method == "PUT":
            rid = f"/subscriptions/sub/resourceGroups/rg/providers/{m['prov']}/{kind}/{name}"
            r = dict(body, id=rid, name=name)
            if kind == "networkInterfaces":
                r["properties"]["ipConfigurations"][0]["properties"]["privateIPAddress"] = "10.1.0.7"
            if kind == "publicIPAddresses":
                r["properties"]["ipAddress"] = "52.0.0.9"
            if kind == "virtualMachines":
                nic = body["properties"]["networkProfile"]["networkInterfaces"][0]["id"]
                assert nic.endswith(f"{name}-nic")
                r["properties"]["provisioningState"] = "Succeeded"
            self.res[key] = r
            return r
        if key not in self.res:
            raise CloudAPIError(404, "ResourceNotFound")
        if method == "GET" and m["iv"]:
            return {"statuses": [{"code": "ProvisioningState/succeeded"}, {"code": "PowerState/running"}]}
        if method == "GET":
            return self.res[key]
        if method == "PATCH":
            self.res[key]["tags"] = body["tags"]
            return self.res[key]
        if method == "DELETE":
            if kind == "networkInterfaces":
                assert ("virtualMachines", name[:-4]) not in self.res, "NIC deleted while its VM exists"
            del self.res[key]
            return {}
        raise AssertionError(url)


def _contract(provider, fake_kind_check=None):
    tags = {T.CLOUDTIK_TAG_NODE_KIND: "worker", T.CLOUDTIK_TAG_USER_NODE_TYPE: "Worker.GPU_8x"}
    created = provider.create_node({}, tags, 2)
    assert len(created) == 2
    head = provider.create_node({}, {T.CLOUDTIK_TAG_NODE_KIND: "head"}, 1)
    workers = provider.non_terminated_nodes({T.CLOUDTIK_TAG_NODE_KIND: "worker"})
    assert sorted(workers) == sorted(created)
    everyone = provider.non_terminated_nodes({})
    assert sorted(everyone) == sorted(list(created) + list(head))
    nid = workers[0]
    got = provider.node_tags(nid)
    assert got[T.CLOUDTIK_TAG_USER_NODE_TYPE] == "Worker.GPU_8x"       # exact, not the sanitised label
    assert got[T.CLOUDTIK_TAG_CLUSTER_NAME] == provider.cluster_name
    provider.set_node_tags(nid, {T.CLOUDTIK_TAG_NODE_STATUS: "up-to-date"})
    assert provider.node_tags(nid)[T.CLOUDTIK_TAG_NODE_STATUS] == "up-to-date"
    assert provider.node_tags(nid)[T.CLOUDTIK_TAG_USER_NODE_TYPE] == "Worker.GPU_8x"
    assert provider.non_terminated_nodes({T.CLOUDTIK_TAG_NODE_STATUS: "up-to-date"}) == [nid]
    assert provider.is_running(nid) and not provider.is_terminated(nid)
    assert provider.internal_ip(nid)
    provider.terminate_node(nid)
    assert nid not in provider.non_terminated_nodes({})
    return nid


def test_gcp_provider_contract():
    fake = FakeGCE()
    p = GCPNodeProvider({"project_id": "proj", "availability_zone": "us-central1-a", "poll_interval_s": 0},
                        "My.Cluster", transport=fake)
    _contract(p)
    inserts = [c for c in fake.calls if c[0] == "POST" and c[1].endswith("/instances")]
    assert inserts and all(c[3]["name"] == gcp_label(c[3]["name"]) for c in inserts)
    assert any(c[1].endswith("/operations/op-1") for c in fake.calls)       # waited for the insert
    assert p.external_ip(p.non_terminated_nodes({})[0]) == "34.1.2.3"


def test_azure_provider_contract():
    fake = FakeARM()
    p = AzureNodeProvider({"subscription_id": "sub", "resource_group": "rg", "location": "westus3",
                           "subnet_id": "/subscriptions/sub/.../subnets/s0", "use_public_ip": True,
                           "poll_interval_s": 0}, "c1", transport=fake)
    nid = _contract(p)
    assert ("networkInterfaces", f"{nid}-nic") not in fake.res              # NIC cleaned up after the VM
    other = p.non_terminated_nodes({})[0]
    assert p.internal_ip(other) == "10.1.0.7" and p.external_ip(other) == "52.0.0.9"
    vm_put = [c for c in fake.calls if c[0] == "PUT" and "/virtualMachines/" in c[1]][0]
    assert vm_put[3]["location"] == "westus3" and vm_put[3]["tags"][T.CLOUDTIK_TAG_CLUSTER_NAME] == "c1"


def test_provider_factory_resolves_rest_providers():
    from cloudtik_amd.core.provider_factory import get_node_provider_cls
    assert get_node_provider_cls({"type": "gcp"}) is GCPNodeProvider
    assert get_node_provider_cls({"type": "azure"}) is AzureNodeProvider


def test_gcp_launch_failure_is_structured():
    from cloudtik_amd.core.node_provider import NodeLaunchException

    def broken(method, url, params, body):
        if method == "POST":
            raise CloudAPIError(403, "QUOTA_EXCEEDED")
        return {"items": []}
    p = GCPNodeProvider({"project_id": "proj", "zone": "us-central1-a"}, "c", transport=broken)
    with pytest.raises(NodeLaunchException) as e:
        p.create_node({}, {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 1)
    assert e.value.category == "GCPInsertFailed" and "QUOTA" in e.value.description


# ------------------------------------------------------------- Aliyun / Huawei Cloud (signed)
from cloudtik_amd.providers.cloud.signed_providers import (AliyunNodeProvider, HuaweiCloudNodeProvider,  # noqa: E402
                                                           aliyun_sign, huawei_sign)


def test_aliyun_signature_known_answer():
    """The worked example of Aliyun's RPC signature v1.0 documentation (DescribeRegions)."""
    p = dict(Timestamp="2016-02-23T12:46:24Z", Format="XML", AccessKeyId="testid", Action="DescribeRegions",
             SignatureMethod="HMAC-SHA1", SignatureNonce="3ee8c1b8-83d3-44af-a94f-4e0ad82fd6cf",
             Version="2014-05-26", SignatureVersion="1.0")
    assert aliyun_sign(p, "testsecret") == "OLeaidS1JvxuMvnyHOwuJ+uX5qY="


def test_huawei_signature_shape_and_sensitivity():
    hdr = {"Host": "ecs.cn-north-4.myhuaweicloud.com", "X-Sdk-Date": "20240101T000000Z",
           "Content-Type": "application/json"}
    url = "https://ecs.cn-north-4.myhuaweicloud.com/v1/p/cloudservers/detail"
    a = huawei_sign("GET", url, {"offset": 1, "limit": 100}, hdr, b"", "AK", "SK")
    m = re.fullmatch(r"SDK-HMAC-SHA256 Access=AK, SignedHeaders=content-type;host;x-sdk-date, Signature=([0-9a-f]{64})", a)
    assert m
    # query order does not matter (canonical sort); any change of path / query / body / key does
    assert huawei_sign("GET", url, {"limit": 100, "offset": 1}, hdr, b"", "AK", "SK") == a
    for args in [("GET", url + "x", {"offset": 1, "limit": 100}, hdr, b"", "AK", "SK"),
                 ("GET", url, {"offset": 2, "limit": 100}, hdr, b"", "AK", "SK"),
                 ("POST", url, {"offset": 1, "limit": 100}, hdr, b"{}", "AK", "SK"),
                 ("GET", url, {"offset": 1, "limit": 100}, hdr, b"", "AK", "SK2")]:
        assert huawei_sign(*args) != a


class FakeAliyunECS:
    def __init__(self):
        self.inst, self.calls, self.n = {}, [], 0

    @staticmethod
    def _indexed(params, prefix):
        out, i = [], 1
        while f"{prefix}.{i}" in params:
            out.append(params[f"{prefix}.{i}"])
            i += 1
        return out

    def __call__(self, action, params):
        self.calls.append((action, params))
        assert params["RegionId"] == "cn-hangzhou"
        tags = {}
        i = 1
        while f"Tag.{i}.Key" in params:
            tags[params[f"Tag.{i}.Key"]] = params[f"Tag.{i}.Value"]
            i += 1
        if action == "RunInstances":
            ids = []
            for _ in range(int(params["Amount"])):
                self.n += 1
                iid = f"i-{self.n:04d}"
                self.inst[iid] = {"InstanceId": iid, "Status": "Pending", "InstanceType": params["InstanceType"],
                                  "Tags": {"Tag": [{"TagKey": k, "TagValue": v} for k, v in tags.items()]},
                                  "VpcAttributes": {"PrivateIpAddress": {"IpAddress": [f"172.16.0.{self.n}"]}},
                                  "PublicIpAddress": {"IpAddress": []}, "EipAddress": {"IpAddress": ""}}
                ids.append(iid)
            return {"InstanceIdSets": {"InstanceIdSet": ids}}
        if action == "DescribeInstances":
            sel = list(self.inst.values())
            if "InstanceIds" in params:
                want = set(__import__("json").loads(params["InstanceIds"]))
                sel = [x for x in sel if x["InstanceId"] in want]
            sel = [x for x in sel if all({t["TagKey"]: t["TagValue"] for t in x["Tags"]["Tag"]}.get(k) == v
                                         for k, v in tags.items())]
            if "Status" in params:
                sel = [x for x in sel if x["Status"] == params["Status"]]
            ps, pn = int(params["PageSize"]), int(params["PageNumber"])
            return {"Instances": {"Instance": sel[(pn - 1) * ps:pn * ps]}, "TotalCount": len(sel)}
        if action == "TagResources":
            assert params["ResourceType"] == "instance"
            for iid in self._indexed(params, "ResourceId"):
                inst = self.inst[iid]
                cur = {t["TagKey"]: t["TagValue"] for t in inst["Tags"]["Tag"]}
                cur.update(tags)
                inst["Tags"]["Tag"] = [{"TagKey": k, "TagValue": v} for k, v in cur.items()]
            return {}
        if action == "StopInstances":
            assert params["StoppedMode"] == "StopCharging"
            for iid in self._indexed(params, "InstanceId"):
                self.inst[iid]["Status"] = "Stopped"
            return {}
        if action == "StartInstances":
            for iid in self._indexed(params, "InstanceId"):
                assert self.inst[iid]["Status"] == "Stopped"
                self.inst[iid]["Status"] = "Starting"
            return {}
        if action == "DeleteInstances":
            assert params["Force"] == "true"
            for iid in self._indexed(params, "InstanceId"):
                del self.inst[iid]
            return {}
        raise AssertionError(action)


def test_aliyun_provider_contract():
    api = FakeAliyunECS()
    p = AliyunNodeProvider({"region": "cn-hangzhou", "_transport": api}, "c1")
    other = AliyunNodeProvider({"region": "cn-hangzhou", "_transport": api}, "c2")
    made = p.create_node({"InstanceType": "ecs.gn8-mi355x", "ImageId": "img"}, {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 2)
    other.create_node({"InstanceType": "ecs.g7"}, {T.CLOUDTIK_TAG_NODE_KIND: "head"}, 1)
    assert len(made) == 2 and sorted(p.non_terminated_nodes({})) == sorted(made)
    assert p.non_terminated_nodes({T.CLOUDTIK_TAG_NODE_KIND: "head"}) == []
    a = sorted(made)[0]
    assert not p.is_running(a) and not p.is_terminated(a)
    api.inst[a]["Status"] = "Running"
    p.non_terminated_nodes({})
    assert p.is_running(a) and p.internal_ip(a).startswith("172.16.") and p.external_ip(a) is None
    p.set_node_tags(a, {T.CLOUDTIK_TAG_NODE_STATUS: "up-to-date"})
    assert p.node_tags(a)[T.CLOUDTIK_TAG_NODE_STATUS] == "up-to-date"
    assert p.non_terminated_nodes({T.CLOUDTIK_TAG_NODE_STATUS: "up-to-date"}) == [a]
    p.terminate_nodes(list(made))
    assert p.non_terminated_nodes({}) == [] and len(other.non_terminated_nodes({})) == 1
    assert p.is_terminated(a)


def test_aliyun_stopped_node_caching():
    """Reference aliyun node_provider.py:213,357: terminate stops, launch restarts matching
    stopped instances first (same node type + launch hash), spot instances are deleted."""
    api = FakeAliyunECS()
    p = AliyunNodeProvider({"region": "cn-hangzhou", "_transport": api}, "c1")
    wt = {T.CLOUDTIK_TAG_NODE_KIND: "worker", T.CLOUDTIK_TAG_USER_NODE_TYPE: "gpu",
          T.CLOUDTIK_TAG_LAUNCH_CONFIG: "h1"}
    made = sorted(p.create_node({"InstanceType": "ecs.gn8"}, wt, 3))
    api.inst[made[2]]["SpotStrategy"] = "SpotAsPriceGo"
    p.terminate_nodes(made)
    assert api.inst[made[0]]["Status"] == api.inst[made[1]]["Status"] == "Stopped"
    assert made[2] not in api.inst                                  # spot: deleted
    assert p.non_terminated_nodes({}) == []
    # a different launch hash does not reuse them
    other = p.create_node({"InstanceType": "ecs.gn8"}, dict(wt, **{T.CLOUDTIK_TAG_LAUNCH_CONFIG: "h2"}), 1)
    assert not set(other) & set(made)
    # same configuration: both stopped ones restart, re-tagged, one more is run
    again = p.create_node({"InstanceType": "ecs.gn8"}, dict(wt, **{T.CLOUDTIK_TAG_NODE_STATUS: "pending"}), 3)
    assert len(again) == 3 and set(made[:2]) <= set(again)
    assert all(api.inst[i]["Status"] == "Starting" for i in made[:2])
    assert p.node_tags(made[0])[T.CLOUDTIK_TAG_NODE_STATUS] == "pending"
    assert sum(1 for a, _ in api.calls if a == "RunInstances") == 3
    # caching off: terminate deletes
    q = AliyunNodeProvider({"region": "cn-hangzhou", "_transport": api, "cache_stopped_nodes": False}, "c1")
    q.terminate_nodes(list(again))
    assert not set(again) & set(api.inst)


class FakeHuaweiECS:
    def __init__(self):
        self.srv, self.calls, self.n = {}, [], 0

    def __call__(self, method, url, params, body):
        self.calls.append((method, url, params, body))
        m = re.match(r"https://ecs\.cn-north-4\.myhuaweicloud\.com/(v1|v1\.1)/proj/cloudservers(.*)$", url)
        assert m, url
        ver, rest = m.groups()
        if ver == "v1.1" and method == "POST" and rest == "":
            s = body["server"]
            assert s["flavorRef"] and s["imageRef"] and s["nics"][0]["subnet_id"] == "sn"
            ids = []
            for _ in range(s["count"]):
                self.n += 1
                sid = f"srv-{self.n}"
                self.srv[sid] = {"id": sid, "status": "BUILD", "tags": [f"{t['key']}={t['value']}"
                                                                         for t in s["server_tags"]],
                                 "addresses": {"vpc": [{"addr": f"192.168.0.{self.n}", "OS-EXT-IPS:type": "fixed"}]}}
                ids.append(sid)
            return {"job_id": "j1", "serverIds": ids}
        if method == "GET" and rest == "/detail":
            lim, off = params["limit"], params["offset"]
            vals = list(self.srv.values())
            return {"servers": vals[(off - 1) * lim:off * lim], "count": len(vals)}
        if method == "POST" and rest == "/delete":
            for s in body["servers"]:
                self.srv.pop(s["id"])
            return {"job_id": "j2"}
        sid = rest.split("/")[1]
        if sid not in self.srv:
            raise CloudAPIError(404, "not found")
        if method == "GET":
            return {"server": self.srv[sid]}
        if rest.endswith("/tags/action"):
            assert body["action"] == "create"
            cur = dict(t.partition("=")[::2] for t in self.srv[sid]["tags"])
            cur.update({t["key"]: t["value"] for t in body["tags"]})
            self.srv[sid]["tags"] = [f"{k}={v}" for k, v in cur.items()]
            return {}
        raise AssertionError(url)


def test_huaweicloud_provider_contract():
    api = FakeHuaweiECS()
    cfg = {"region": "cn-north-4", "project_id": "proj", "_transport": api}
    p = HuaweiCloudNodeProvider(cfg, "c1")
    made = p.create_node({"flavor": "mi355x.8xlarge", "image_id": "img", "vpc_id": "vpc", "subnet_id": "sn"},
                         {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 3)
    HuaweiCloudNodeProvider(cfg, "c2").create_node({"flavor": "f", "image_id": "i", "subnet_id": "sn"}, {}, 1)
    assert sorted(p.non_terminated_nodes({})) == sorted(made)
    a = sorted(made)[0]
    assert not p.is_running(a) and not p.is_terminated(a)
    api.srv[a]["status"] = "ACTIVE"
    p.non_terminated_nodes({})
    assert p.is_running(a) and p.internal_ip(a).startswith("192.168.0.") and p.external_ip(a) is None
    p.set_node_tags(a, {T.CLOUDTIK_TAG_NODE_STATUS: "up-to-date"})
    assert p.non_terminated_nodes({T.CLOUDTIK_TAG_NODE_STATUS: "up-to-date"}) == [a]
    p.terminate_nodes(list(made))
    assert p.non_terminated_nodes({}) == [] and p.is_terminated(a)


def test_factory_resolves_signed_providers():
    from cloudtik_amd.core.provider_factory import _NODE_PROVIDERS
    assert _NODE_PROVIDERS["aliyun"]() is AliyunNodeProvider
    assert _NODE_PROVIDERS["huaweicloud"]() is HuaweiCloudNodeProvider
