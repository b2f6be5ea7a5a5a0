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
