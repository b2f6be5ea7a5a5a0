"""Public-cloud node providers (reference providers/_private/{aws,gcp,azure,aliyun,
huaweicloud}/node_provider.py; SURVEY.md §2.9 "keep interface; not needed for the MI355X
node").

The provider interface, config schema, defaults and instance templates are kept so cluster
YAML stays portable.  ``AWSNodeProvider`` is implemented against boto3 (EC2 instances as
nodes, tags as node tags, ``cloudtik-cluster-name`` filters); it needs boto3 and
credentials at run time.  GCP and Azure are implemented over their REST APIs in
rest_providers.py, Aliyun and Huawei Cloud over their signed HTTP APIs in signed_providers.py.
"""
from __future__ import annotations

import importlib
import threading
import time
from typing import Any, Dict, List, Optional

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.node_provider import NodeLaunchException, NodeProvider


def _require(module: str, provider: str):
    try:
        return importlib.import_module(module)
    except ImportError as e:
        raise RuntimeError(f"the {provider} provider needs the '{module}' package (pip install {module}); "
                           "it is not available in this environment") from e


TAG_BATCH_DELAY = 1.0     # seconds set_node_tags waits to batch concurrent updates
STOPPING_WAIT_S = 300.0   # how long a launch waits for a 'stopping' cached node to stop
STOPPING_POLL_S = 5.0


class AWSNodeProvider(NodeProvider):
    """EC2 instances as nodes (reference providers/_private/aws/node_provider.py).

    * node tags are EC2 tags; ``set_node_tags`` calls from the updater threads of many nodes
      are batched (one ``create_tags`` per distinct tag set every ``TAG_BATCH_DELAY``), as
      a 100-node launch otherwise floods the EC2 API;
    * ``create_node`` places instances in the workspace's private subnets (round-robin over
      ``SubnetIds``, moving to the next subnet on capacity errors), with the workspace
      security group and the head / worker instance profile (providers/cloud/workspace.py),
      optional spot market, and ``data_disks`` as extra gp3 EBS volumes;
    * stopped-node caching (``cache_stopped_nodes``, default true, reference aws
      node_provider.py:63,233,530): terminating a node STOPS it (spot instances, which cannot
      be stopped, are terminated); a launch first restarts stopped nodes of the same cluster,
      node kind, node type and launch hash, re-tagged, and creates only the remainder;
    * boto3 is loaded lazily; ``provider._client_factory`` injects a client (tests).
    """

    CAPACITY_ERRORS = ("InsufficientInstanceCapacity", "InsufficientFreeAddressesInSubnet",
                       "InsufficientCapacity", "Unsupported")

    def __init__(self, provider_config, cluster_name):
        super().__init__(provider_config, cluster_name)
        factory = provider_config.get("_client_factory")
        if factory is None:
            boto3 = _require("boto3", "aws")
            factory = lambda svc: boto3.client(svc, region_name=provider_config.get("region"))  # noqa: E731
        self.ec2 = factory("ec2")
        self._nodes: Dict[str, Dict[str, Any]] = {}
        self.tag_cache: Dict[str, Dict[str, str]] = {}
        self._lock = threading.RLock()
        self._pending_tags: Dict[str, Dict[str, str]] = {}
        self._batch_timer: Optional[threading.Timer] = None
        self._subnet_idx = 0
        self.cache_stopped_nodes = bool(provider_config.get("cache_stopped_nodes", True))

    # ------------------------------------------------------------------ queries
    def _filters(self, tag_filters):
        f = [{"Name": "instance-state-name", "Values": ["pending", "running"]}]
        f += [{"Name": f"tag:{k}", "Values": [v]} for k, v in dict(self.cluster_filter(), **tag_filters).items()]
        return f

    def _remember(self, inst: Dict[str, Any]):
        nid = inst["InstanceId"]
        self._nodes[nid] = inst
        with self._lock:
            tags = {t["Key"]: t["Value"] for t in inst.get("Tags") or []}
            tags.update(self._pending_tags.get(nid, {}))     # not yet flushed updates win
            self.tag_cache[nid] = tags

    def non_terminated_nodes(self, tag_filters):
        out, token = [], None
        while True:
            kw = {"Filters": self._filters(tag_filters)}
            if token:
                kw["NextToken"] = token
            r = self.ec2.describe_instances(**kw)
            for res in r.get("Reservations", []):
                for inst in res.get("Instances", []):
                    self._remember(inst)
                    out.append(inst["InstanceId"])
            token = r.get("NextToken")
            if not token:
                return out

    def _node(self, node_id):
        n = self._nodes.get(node_id)
        if n is None:
            r = self.ec2.describe_instances(InstanceIds=[node_id])
            n = r["Reservations"][0]["Instances"][0]
            self._remember(n)
        return n

    def is_running(self, node_id):
        return self._node(node_id)["State"]["Name"] == "running"

    def is_terminated(self, node_id):
        return self._node(node_id)["State"]["Name"] not in ("running", "pending")

    def node_tags(self, node_id):
        with self._lock:
            if node_id in self.tag_cache:
                return dict(self.tag_cache[node_id])
        self._node(node_id)
        with self._lock:
            return dict(self.tag_cache.get(node_id, {}))

    def external_ip(self, node_id):
        return self._node(node_id).get("PublicIpAddress")

    def internal_ip(self, node_id):
        return self._node(node_id).get("PrivateIpAddress")

    # ------------------------------------------------------------------ tags (batched)
    def set_node_tags(self, node_id, tags):
        with self._lock:
            self._pending_tags.setdefault(node_id, {}).update(tags)
            self.tag_cache.setdefault(node_id, {}).update(tags)
            if self._batch_timer is None:
                self._batch_timer = threading.Timer(TAG_BATCH_DELAY, self._flush_tags)
                self._batch_timer.daemon = True
                self._batch_timer.start()

    def _flush_tags(self):
        with self._lock:
            pending, self._pending_tags = self._pending_tags, {}
            self._batch_timer = None
        # one create_tags per distinct tag set
        groups: Dict[tuple, List[str]] = {}
        for nid, tags in pending.items():
            groups.setdefault(tuple(sorted(tags.items())), []).append(nid)
        self._create_tags({k: v for k, v in groups.items()})

    def _create_tags(self, batch_updates: Dict[tuple, List[str]]):
        for tag_items, node_ids in batch_updates.items():
            self.ec2.create_tags(Resources=node_ids, Tags=[{"Key": k, "Value": v} for k, v in tag_items])

    def flush_tags(self):
        """Apply pending tag updates now (also before terminate)."""
        with self._lock:
            if self._batch_timer is not None:
                self._batch_timer.cancel()
        self._flush_tags()

    # ------------------------------------------------------------------ launch
    def _workspace_defaults(self):
        """Subnets, security group and instance profiles of the cluster's workspace
        (providers/cloud/workspace.py AWSWorkspace) for keys the config does not set."""
        pc = self.provider_config
        if pc.get("_workspace_filled") or not pc.get("workspace_name") or pc.get("use_working_vpc"):
            return
        pc["_workspace_filled"] = True
        try:
            from cloudtik_amd.providers.cloud.workspace import AWSWorkspace
            ws = AWSWorkspace(pc, pc["workspace_name"], pc.get("_client_factory"))
            sub = ws.ec2.describe_subnets(Filters=ws._filters([{"Name": "tag:cloudtik-subnet",
                                                                  "Values": ["private"]}]))["Subnets"]
            pc.setdefault("subnet_ids", [x["SubnetId"] for x in sub])
            sg = ws._sg()
            if sg:
                pc.setdefault("security_group_ids", [sg])
            pc.setdefault("head_instance_profile", ws.roles["head"])
            pc.setdefault("worker_instance_profile", ws.roles["worker"])
        except Exception as e:  # noqa: BLE001 - no workspace resources: launch with the config as given
            import logging
            logging.getLogger(__name__).warning("AWS workspace defaults unavailable: %s", e)

    # ------------------------------------------------------------------ SSH key pair
    def key_pair_exists(self, name: str) -> bool:
        try:
            return bool(self.ec2.describe_key_pairs(KeyNames=[name]).get("KeyPairs"))
        except Exception as e:  # noqa: BLE001 - botocore ClientError InvalidKeyPair.NotFound
            code = getattr(e, "response", {}).get("Error", {}).get("Code", "")
            if code == "InvalidKeyPair.NotFound":
                return False
            raise

    def create_key_pair(self, name: str) -> str:
        return self.ec2.create_key_pair(KeyName=name)["KeyMaterial"]

    @staticmethod
    def bootstrap_config(cluster_config):
        """Key pair for the updater's SSH (reference aws/config.py:3868)."""
        from cloudtik_amd.providers.cloud import keypairs
        p = AWSNodeProvider(cluster_config["provider"], cluster_config.get("cluster_name", "default"))
        return keypairs.configure_cloud_key_pair(cluster_config, "aws", cluster_config["provider"]["region"],
                                                 p.key_pair_exists, p.create_key_pair)

    def _subnets(self, node_config) -> List[str]:
        ids = node_config.get("SubnetIds") or ([node_config["SubnetId"]] if node_config.get("SubnetId") else [])
        return list(ids or self.provider_config.get("subnet_ids", []))

    def _reuse_stopped(self, tags, count) -> Dict[str, Any]:
        """Restart up to ``count`` stopped nodes launched from the same configuration."""
        keys = (T.CLOUDTIK_TAG_NODE_KIND, T.CLOUDTIK_TAG_LAUNCH_CONFIG, T.CLOUDTIK_TAG_USER_NODE_TYPE)
        filters = [{"Name": "instance-state-name", "Values": ["stopped", "stopping"]},
                   {"Name": f"tag:{T.CLOUDTIK_TAG_CLUSTER_NAME}", "Values": [self.cluster_name]}]
        filters += [{"Name": f"tag:{k}", "Values": [tags[k]]} for k in keys if k in tags]
        found = []
        for res in self.ec2.describe_instances(Filters=filters).get("Reservations", []):
            found += res.get("Instances", [])
        # prefer instances that are already stopped; a 'stopping' one is usable only once
        # EC2 reports it stopped (StartInstances on it fails with IncorrectInstanceState and
        # would fail the whole scale-up; reference aws node_provider.py:280-287 waits too)
        found = sorted(found, key=lambda i: (i["State"]["Name"] != "stopped", i["InstanceId"]))[:count]
        stopping = [i["InstanceId"] for i in found if i["State"]["Name"] != "stopped"]
        if stopping:
            ready = self._wait_stopped(stopping)
            found = [i for i in found if i["State"]["Name"] == "stopped" or i["InstanceId"] in ready]
        if not found:
            return {}
        ids = [i["InstanceId"] for i in found]
        self.ec2.start_instances(InstanceIds=ids)
        # the reused nodes take the new launch's tags (status, node seq id, ...)
        self.ec2.create_tags(Resources=ids, Tags=[{"Key": k, "Value": str(v)} for k, v in tags.items()])
        out = {}
        for inst in found:
            cur = {t["Key"]: t["Value"] for t in inst.get("Tags") or []}
            cur.update({k: str(v) for k, v in tags.items()})
            inst = dict(inst, Tags=[{"Key": k, "Value": v} for k, v in cur.items()], State={"Name": "pending"})
            self._remember(inst)
            out[inst["InstanceId"]] = inst
        return out

    def _wait_stopped(self, ids, timeout=None, poll=None):
        """Poll until the given 'stopping' instances are 'stopped'; returns the ids that got
        there within ``timeout`` (the rest are left alone and new instances are launched)."""
        timeout = STOPPING_WAIT_S if timeout is None else timeout
        poll = STOPPING_POLL_S if poll is None else poll
        deadline = time.time() + timeout
        pending = set(ids)
        done = set()
        while pending:
            resp = self.ec2.describe_instances(InstanceIds=sorted(pending))
            for res in resp.get("Reservations", []):
                for inst in res.get("Instances", []):
                    if inst["State"]["Name"] == "stopped":
                        done.add(inst["InstanceId"])
                    elif inst["State"]["Name"] != "stopping":      # terminated / started elsewhere
                        pending.discard(inst["InstanceId"])
            pending -= done
            if not pending or time.time() >= deadline:
                break
            time.sleep(poll)
        return done

    def create_node(self, node_config, tags, count):
        reused: Dict[str, Any] = {}
        if self.cache_stopped_nodes:
            reused = self._reuse_stopped(dict(tags, **{T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name}), count)
            count -= len(reused)
            if count <= 0:
                return reused
        out = self._launch(node_config, tags, count)
        out.update(reused)
        return out

    def _launch(self, node_config, tags, count):
        self._workspace_defaults()
        conf = {k: v for k, v in node_config.items()
                if k not in ("SubnetIds", "SubnetId", "data_disks", "spot", "instance_type")}
        tags = dict(tags, **{T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name})
        conf.setdefault("TagSpecifications", []).append(
            {"ResourceType": "instance", "Tags": [{"Key": k, "Value": str(v)} for k, v in tags.items()]})
        conf["MinCount"] = conf["MaxCount"] = count
        if "instance_type" in node_config:
            conf["InstanceType"] = node_config["instance_type"]
        kind = tags.get(T.CLOUDTIK_TAG_NODE_KIND, "worker")
        profile = self.provider_config.get(f"{kind}_instance_profile")
        if profile and "IamInstanceProfile" not in conf:
            conf["IamInstanceProfile"] = {"Name": profile}
        sgs = self.provider_config.get("security_group_ids")
        if sgs and "SecurityGroupIds" not in conf:
            conf["SecurityGroupIds"] = list(sgs)
        if node_config.get("spot"):
            conf["InstanceMarketOptions"] = {"MarketType": "spot", "SpotOptions": {
                "SpotInstanceType": "one-time", "InstanceInterruptionBehavior": "terminate"}}
        disks = node_config.get("data_disks") or []
        if disks:
            conf["BlockDeviceMappings"] = list(conf.get("BlockDeviceMappings", [])) + [
                {"DeviceName": f"/dev/sd{chr(ord('f') + i)}",
                 "Ebs": {"VolumeSize": int(d.get("size", 200) if isinstance(d, dict) else d), "VolumeType": "gp3",
                         "DeleteOnTermination": True}} for i, d in enumerate(disks)]
        subnets = self._subnets(node_config)
        attempts = subnets if subnets else [None]
        last = None
        for i in range(len(attempts)):
            subnet = attempts[(self._subnet_idx + i) % len(attempts)]
            if subnet:
                conf["SubnetId"] = subnet
            try:
                r = self.ec2.run_instances(**conf)
            except Exception as e:  # noqa: BLE001 -- botocore ClientError
                code = getattr(e, "response", {}).get("Error", {}).get("Code", type(e).__name__)
                last = NodeLaunchException(code, str(e))
                if any(c in code for c in self.CAPACITY_ERRORS) and i + 1 < len(attempts):
                    continue                                   # next subnet / availability zone
                raise last
            self._subnet_idx = (self._subnet_idx + i + 1) % max(1, len(attempts))
            out = {}
            for inst in r.get("Instances", []):
                inst.setdefault("Tags", [{"Key": k, "Value": str(v)} for k, v in tags.items()])
                self._remember(inst)
                out[inst["InstanceId"]] = inst
            return out
        raise last

    def terminate_node(self, node_id):
        self.terminate_nodes([node_id])

    def terminate_nodes(self, node_ids: List[str]):
        if not node_ids:
            return
        self.flush_tags()
        terminate, stop = list(node_ids), []
        if self.cache_stopped_nodes:
            # spot instances cannot be stopped: those are terminated
            spot = {n for n in node_ids if self._node(n).get("InstanceLifecycle") == "spot"}
            stop = [n for n in node_ids if n not in spot]
            terminate = [n for n in node_ids if n in spot]
        if stop:
            self.ec2.stop_instances(InstanceIds=stop)
        if terminate:
            self.ec2.terminate_instances(InstanceIds=terminate)
        for n in node_ids:
            self._nodes.pop(n, None)


# GCP and Azure speak the clouds' REST APIs directly (no SDK needed): rest_providers.py
from cloudtik_amd.providers.cloud.rest_providers import AzureNodeProvider, GCPNodeProvider  # noqa: E402,F401


# Aliyun and Huawei Cloud speak the clouds' signed HTTP APIs (no SDK needed): signed_providers.py
from cloudtik_amd.providers.cloud.signed_providers import AliyunNodeProvider, HuaweiCloudNodeProvider  # noqa: E402,F401,E501
