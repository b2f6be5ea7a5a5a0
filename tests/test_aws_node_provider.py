"""AWS node provider (providers/cloud/node_provider.py; reference providers/_private/aws/
node_provider.py + tests/unit/aws/test_aws_batch_tag_update.py) against a fake EC2 client:
batched tag updates from concurrent updater threads, subnet failover on capacity errors,
instance profile / security group / data disks / spot in the launch request, tag cache."""
import threading
import time

from cloudtik_amd.core import tags as T
from cloudtik_amd.providers.cloud import node_provider as NP


class CapacityError(Exception):
    def __init__(self):
        super().__init__("no capacity")
        self.response = {"Error": {"Code": "InsufficientInstanceCapacity"}}


class FakeEC2:
    def __init__(self, full_subnets=()):
        self.instances, self.n = {}, 0
        self.create_tags_calls, self.tags_updated = 0, 0
        self.full = set(full_subnets)
        self.requests = []
        self.lock = threading.Lock()

    def run_instances(self, **kw):
        self.requests.append(kw)
        if kw.get("SubnetId") in self.full:
            raise CapacityError()
        out = []
        for _ in range(kw["MaxCount"]):
            self.n += 1
            iid = f"i-{self.n:04d}"
            tags = kw["TagSpecifications"][0]["Tags"]
            self.instances[iid] = {"InstanceId": iid, "State": {"Name": "pending"}, "Tags": list(tags),
                                   "PrivateIpAddress": f"10.0.0.{self.n}", "SubnetId": kw.get("SubnetId")}
            out.append(dict(self.instances[iid]))
        return {"Instances": out}

    def describe_instances(self, Filters=None, InstanceIds=None, NextToken=None):
        states = ("pending", "running")
        for f in Filters or []:
            if f["Name"] == "instance-state-name":
                states = tuple(f["Values"])
        rows = [i for i in self.instances.values() if i["State"]["Name"] in states]
        if InstanceIds:
            rows = [self.instances[i] for i in InstanceIds]
        for f in Filters or []:
            if f["Name"].startswith("tag:"):
                k = f["Name"][4:]
                rows = [r for r in rows if {t["Key"]: t["Value"] for t in r["Tags"]}.get(k) in f["Values"]]
        return {"Reservations": [{"Instances": [dict(r) for r in rows]}]}

    def create_tags(self, Resources, Tags):
        with self.lock:
            self.create_tags_calls += 1
            self.tags_updated += len(Resources)
            for iid in Resources:
                cur = {t["Key"]: t["Value"] for t in self.instances[iid]["Tags"]}
                cur.update({t["Key"]: t["Value"] for t in Tags})
                self.instances[iid]["Tags"] = [{"Key": k, "Value": v} for k, v in cur.items()]

    def terminate_instances(self, InstanceIds):
        for i in InstanceIds:
            self.instances[i]["State"]["Name"] = "terminated"

    def stop_instances(self, InstanceIds):
        for i in InstanceIds:
            self.instances[i]["State"]["Name"] = "stopped"

    def start_instances(self, InstanceIds):
        for i in InstanceIds:
            assert self.instances[i]["State"]["Name"] == "stopped"
            self.instances[i]["State"]["Name"] = "pending"


def _provider(fake, **cfg):
    return NP.AWSNodeProvider(dict(region="nowhere", _client_factory=lambda svc: fake, **cfg), "c1")


def test_concurrent_tag_updates_are_batched(monkeypatch):
    monkeypatch.setattr(NP, "TAG_BATCH_DELAY", 0.3)
    fake = FakeEC2()
    p = _provider(fake)
    ids = list(p.create_node({"instance_type": "m5.large"}, {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 100))
    threads = [threading.Thread(target=p.set_node_tags, args=(i, {"status": "up-to-date"})) for i in ids]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert p.node_tags(ids[0])["status"] == "up-to-date"        # visible before the flush
    time.sleep(0.6)
    assert fake.create_tags_calls < 10 and fake.tags_updated == 100
    # serial updates further apart than the delay go out one by one
    for i in ids[:3]:
        p.set_node_tags(i, {"x": i})
        time.sleep(0.4)
    assert fake.create_tags_calls >= 4


def test_launch_request_and_subnet_failover():
    fake = FakeEC2(full_subnets={"subnet-a"})
    p = _provider(fake, security_group_ids=["sg-1"], worker_instance_profile="cloudtik-ws-worker-role")
    out = p.create_node({"instance_type": "p5e.48xlarge", "SubnetIds": ["subnet-a", "subnet-b"], "spot": True,
                         "data_disks": [{"size": 1000}, 500]}, {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 2)
    assert len(out) == 2 and all(i["SubnetId"] == "subnet-b" for i in out.values())
    req = fake.requests[-1]
    assert req["InstanceType"] == "p5e.48xlarge" and req["SecurityGroupIds"] == ["sg-1"]
    assert req["IamInstanceProfile"] == {"Name": "cloudtik-ws-worker-role"}
    assert req["InstanceMarketOptions"]["MarketType"] == "spot"
    assert [b["Ebs"]["VolumeSize"] for b in req["BlockDeviceMappings"]] == [1000, 500]
    nid = next(iter(out))
    assert p.internal_ip(nid).startswith("10.0.0.") and p.node_tags(nid)[T.CLOUDTIK_TAG_CLUSTER_NAME] == "c1"
    assert sorted(p.non_terminated_nodes({T.CLOUDTIK_TAG_NODE_KIND: "worker"})) == sorted(out)
    p.terminate_nodes(list(out))
    assert p.non_terminated_nodes({}) == []


def test_all_subnets_full_raises_launch_exception():
    import pytest
    from cloudtik_amd.core.node_provider import NodeLaunchException
    fake = FakeEC2(full_subnets={"subnet-a", "subnet-b"})
    with pytest.raises(NodeLaunchException):
        _provider(fake).create_node({"SubnetIds": ["subnet-a", "subnet-b"]}, {}, 1)


def test_stopped_node_caching_reuses_matching_nodes():
    """cache_stopped_nodes (reference aws node_provider.py:63,233,530): terminate stops the
    instance; the next launch with the same launch hash / node type restarts it (re-tagged)
    and creates only what is missing; spot instances are terminated, never stopped."""
    fake = FakeEC2()
    p = _provider(fake)
    tags = {T.CLOUDTIK_TAG_NODE_KIND: "worker", T.CLOUDTIK_TAG_LAUNCH_CONFIG: "h1",
            T.CLOUDTIK_TAG_USER_NODE_TYPE: "gpu.8x"}
    ids = sorted(p.create_node({"instance_type": "m5.large"}, dict(tags, **{T.CLOUDTIK_TAG_NODE_STATUS: "up-to-date"}), 2))
    p.terminate_nodes(ids)
    assert all(fake.instances[i]["State"]["Name"] == "stopped" for i in ids)
    assert p.non_terminated_nodes({}) == []
    # another launch hash: no reuse
    other = p.create_node({"instance_type": "m5.large"}, dict(tags, **{T.CLOUDTIK_TAG_LAUNCH_CONFIG: "h2"}), 1)
    assert not set(other) & set(ids)
    # same launch config: both stopped nodes come back, one new instance is created
    n_before = fake.n
    got = p.create_node({"instance_type": "m5.large"}, dict(tags, **{T.CLOUDTIK_TAG_NODE_STATUS: "uninitialized"}), 3)
    assert set(ids) <= set(got) and len(got) == 3 and fake.n == n_before + 1
    assert all(p.node_tags(i)[T.CLOUDTIK_TAG_NODE_STATUS] == "uninitialized" for i in ids)
    assert {t["Key"]: t["Value"] for t in fake.instances[ids[0]]["Tags"]}[T.CLOUDTIK_TAG_NODE_STATUS] == "uninitialized"
    # spot: terminated even with caching on
    fake.instances[ids[0]]["InstanceLifecycle"] = "spot"
    p._nodes.pop(ids[0], None)
    p.terminate_nodes([ids[0]])
    assert fake.instances[ids[0]]["State"]["Name"] == "terminated"
    # caching off: terminate
    q = _provider(fake, cache_stopped_nodes=False)
    q.terminate_nodes([ids[1]])
    assert fake.instances[ids[1]]["State"]["Name"] == "terminated"


def test_stopping_node_is_waited_for_before_start(monkeypatch):
    """A cached node still 'stopping' is started only after EC2 reports it 'stopped'
    (StartInstances on a stopping instance fails); one that never stops is skipped and a
    new instance launched instead (reference aws node_provider.py:280-287)."""
    monkeypatch.setattr(NP, "STOPPING_POLL_S", 0.01)
    fake = FakeEC2()
    p = _provider(fake)
    tags = {T.CLOUDTIK_TAG_NODE_KIND: "worker", T.CLOUDTIK_TAG_LAUNCH_CONFIG: "h1",
            T.CLOUDTIK_TAG_USER_NODE_TYPE: "gpu.8x"}
    ids = sorted(p.create_node({"instance_type": "m5.large"}, dict(tags), 2))
    p.terminate_nodes(ids)
    fake.instances[ids[0]]["State"]["Name"] = "stopping"
    fake.instances[ids[1]]["State"]["Name"] = "stopping"
    polls = {"n": 0}
    orig = fake.describe_instances

    def describe(Filters=None, InstanceIds=None, NextToken=None):
        if InstanceIds:
            polls["n"] += 1
            if polls["n"] == 3:                       # ids[0] finishes stopping on the 3rd poll
                fake.instances[ids[0]]["State"]["Name"] = "stopped"
        return orig(Filters=Filters, InstanceIds=InstanceIds, NextToken=NextToken)
    fake.describe_instances = describe
    monkeypatch.setattr(NP, "STOPPING_WAIT_S", 0.2)
    n_before = fake.n
    got = p.create_node({"instance_type": "m5.large"}, dict(tags), 2)
    assert ids[0] in got and ids[1] not in got            # never started while stopping
    assert fake.instances[ids[0]]["State"]["Name"] == "pending"
    assert fake.instances[ids[1]]["State"]["Name"] == "stopping"
    assert fake.n == n_before + 1 and len(got) == 2
