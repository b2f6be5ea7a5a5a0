"""On-premise provider against a live cloud-simulator service, Kubernetes provider against a
fake kubectl, and the provider registry."""
import json
import os
import socket
import sys
import threading

import pytest
import yaml

from cloudtik_amd.core import tags as T


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def simulator(tmp_path, monkeypatch):
    from cloudtik_amd.providers.onpremise.simulator import serve
    monkeypatch.setenv("CLOUDTIK_SIMULATOR_PROCESS_FILE", str(tmp_path / "sim.json"))
    pool = {"instance_types": {"mi355x-8gpu": {"CPU": 128, "GPU": 8, "accelerator_type:MI355X": 8},
                               "cpu-node": {"CPU": 64}},
            "nodes": [{"ip": "10.1.0.1", "instance_type": "mi355x-8gpu"},
                      {"ip": "10.1.0.2", "instance_type": "mi355x-8gpu"},
                      {"ip": "10.1.0.3", "instance_type": "cpu-node"}]}
    (tmp_path / "pool.yaml").write_text(yaml.safe_dump(pool))
    port = _port()
    srv = serve(str(tmp_path / "pool.yaml"), "127.0.0.1", port, str(tmp_path / "state.json"))
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    yield f"127.0.0.1:{port}"
    srv.shutdown()
    srv.server_close()


def test_onpremise_provider_pool(simulator):
    from cloudtik_amd.core.node_provider import NodeLaunchException
    from cloudtik_amd.providers.onpremise.node_provider import OnPremiseNodeProvider
    pa = OnPremiseNodeProvider({"type": "onpremise", "cloud_simulator_address": simulator}, "a")
    pb = OnPremiseNodeProvider({"type": "onpremise", "cloud_simulator_address": simulator}, "b")
    got = pa.create_node({"instance_type": "mi355x-8gpu"}, {T.CLOUDTIK_TAG_NODE_KIND: "head"}, 1)
    (nid,) = got
    assert pa.non_terminated_nodes({}) == [nid] and pb.non_terminated_nodes({}) == []
    assert pa.node_tags(nid)[T.CLOUDTIK_TAG_NODE_KIND] == "head"
    pa.set_node_tags(nid, {"x": "1"})
    assert pa.node_tags(nid)["x"] == "1" and pa.is_running(nid)
    pb.create_node({"instance_type": "mi355x-8gpu"}, {}, 1)
    with pytest.raises(NodeLaunchException):
        pb.create_node({"instance_type": "mi355x-8gpu"}, {}, 1)      # pool exhausted
    assert pa.get_node_info(nid)["resources"]["GPU"] == 8
    pa.terminate_node(nid)
    assert pa.non_terminated_nodes({}) == [] and pa.is_terminated(nid)
    # resources are filled from the simulator's instance types
    cfg = {"provider": {"type": "onpremise", "cloud_simulator_address": simulator},
           "available_node_types": {"w": {"node_config": {"instance_type": "cpu-node"}}}}
    OnPremiseNodeProvider.fillout_available_node_types_resources(cfg)
    assert cfg["available_node_types"]["w"]["resources"] == {"CPU": 64}


def test_simulator_reload_workspaces_discovery_and_shutdown(simulator, tmp_path, monkeypatch):
    """Reference cloudtik_cloud_simulator.py:196-227 / cloud_simulator_scheduler.py:146-158 /
    onpremise/config.py:20-50: the pool is reloaded in place (new hosts free, removed free hosts
    gone, removed allocated hosts drain), workspaces live in the simulator, providers find the
    simulator through its process file, and --shutdown stops it."""
    from cloudtik_amd.core.workspace import Existence
    from cloudtik_amd.providers.onpremise import simulator as S
    from cloudtik_amd.providers.onpremise.node_provider import OnPremiseNodeProvider
    from cloudtik_amd.providers.onpremise.workspace_provider import OnPremiseWorkspaceProvider
    # discovery: no address configured -> the process file of the running simulator
    assert S.discover_simulator() == simulator
    pa = OnPremiseNodeProvider({"type": "onpremise"}, "a")
    (nid,) = pa.create_node({"instance_type": "mi355x-8gpu"}, {T.CLOUDTIK_TAG_NODE_KIND: "head",
                                                               T.CLOUDTIK_TAG_WORKSPACE_NAME: "w1"}, 1)
    # workspaces
    wp = OnPremiseWorkspaceProvider({"type": "onpremise"}, "w1")
    assert wp.check_workspace_existence({}) == Existence.NOT_EXIST
    wp.create_workspace({})
    assert wp.check_workspace_existence({}) == Existence.COMPLETED
    assert S.request(None, "list_workspaces") == ["w1"]
    with pytest.raises(RuntimeError, match="running clusters"):
        wp.delete_workspace({})
    # reload: 10.1.0.2 (free) and 10.1.0.1 (allocated to cluster a) leave, 10.1.0.9 joins
    pool = {"instance_types": {"mi355x-8gpu": {"CPU": 128, "GPU": 8}, "cpu-node": {"CPU": 64}},
            "nodes": [{"ip": "10.1.0.3", "instance_type": "cpu-node"},
                      {"ip": "10.1.0.9", "instance_type": "mi355x-8gpu"}]}
    (tmp_path / "pool.yaml").write_text(yaml.safe_dump(pool))
    S.main(["--reload", "--bind-address", simulator.split(":")[0], "--port", simulator.split(":")[1]])
    st = S.request(None, "pool_status")
    assert st["total"] == 3 and st["draining"] == [nid] and st["free"] == 2
    (n2,) = OnPremiseNodeProvider({"type": "onpremise"}, "b").create_node({"instance_type": "mi355x-8gpu"}, {}, 1)
    assert n2 == "10.1.0.9"                                 # never a draining host
    pa.terminate_node(nid)                                  # the draining host leaves the pool
    assert S.request(None, "pool_status")["total"] == 2
    wp.delete_workspace({})
    assert wp.check_workspace_existence({}) == Existence.NOT_EXIST
    # shutdown over the API
    S.main(["--shutdown"])
    import time
    deadline = time.time() + 5
    while time.time() < deadline and os.path.exists(str(tmp_path / "sim.json")):
        time.sleep(0.05)
    assert not os.path.exists(str(tmp_path / "sim.json"))
    with pytest.raises(Exception):
        S.request(simulator, "pool_status")


FAKE_KUBECTL = r'''#!/usr/bin/env python3
import json, os, sys
db = os.environ["FAKE_K8S_DB"]
state = json.load(open(db)) if os.path.exists(db) else {}
a = sys.argv[1:]
a = a[2:] if a[:1] == ["-n"] else a
def save(): json.dump(state, open(db, "w"))
if a[0] == "apply":
    pod = json.load(sys.stdin); pod["status"] = {"phase": "Running", "podIP": "10.2.0.%d" % (len(state) + 1)}
    state[pod["metadata"]["name"]] = pod; save()
elif a[0] == "get" and a[1] == "pods":
    sel = dict(kv.split("=") for kv in a[3].split(","))
    items = [p for p in state.values() if all(p["metadata"]["labels"].get(k) == v for k, v in sel.items())]
    print(json.dumps({"items": items}))
elif a[0] == "get" and a[1] == "pod":
    print(json.dumps(state[a[2]]))
elif a[0] in ("label", "annotate"):
    key = "labels" if a[0] == "label" else "annotations"
    for kv in a[4:]:
        k, v = kv.split("=", 1); state[a[2]]["metadata"][key][k] = v
    save()
elif a[0] == "delete":
    state[a[2]]["status"]["phase"] = "Succeeded"; save()
'''


def test_kubernetes_provider_with_fake_kubectl(tmp_path, monkeypatch):
    from cloudtik_amd.providers.kubernetes.node_provider import KubernetesNodeProvider
    k = tmp_path / "kubectl"
    k.write_text(FAKE_KUBECTL)
    k.chmod(0o755)
    monkeypatch.setenv("FAKE_K8S_DB", str(tmp_path / "db.json"))
    p = KubernetesNodeProvider({"type": "kubernetes", "namespace": "ns"}, "kc", kubectl=[sys.executable, str(k)])
    created = p.create_node({"resources": {"GPU": 8}}, {T.CLOUDTIK_TAG_NODE_KIND: "worker",
                                                        T.CLOUDTIK_TAG_USER_NODE_TYPE: "worker.mi355x"}, 2)
    assert len(created) == 2
    pod = next(iter(created.values()))
    assert pod["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == 8
    nodes = p.non_terminated_nodes({T.CLOUDTIK_TAG_NODE_KIND: "worker"})
    assert sorted(nodes) == sorted(created)
    p.set_node_tags(nodes[0], {T.CLOUDTIK_TAG_NODE_STATUS: "up-to-date"})
    assert p.node_tags(nodes[0])[T.CLOUDTIK_TAG_NODE_STATUS] == "up-to-date"
    assert p.node_tags(nodes[0])[T.CLOUDTIK_TAG_USER_NODE_TYPE] == "worker.mi355x"   # exact, via annotation
    assert p.internal_ip(nodes[0]).startswith("10.2.0.")
    p.terminate_node(nodes[0])
    assert p.non_terminated_nodes({}) == [nodes[1]]


def test_provider_registry_resolves_every_type():
    from cloudtik_amd.core.provider_factory import get_node_provider_cls, get_workspace_provider
    for t in ["local", "virtual", "onpremise", "aws", "gcp", "azure", "aliyun", "huaweicloud", "kubernetes", "mock"]:
        assert get_node_provider_cls({"type": t}) is not None
    with pytest.raises(RuntimeError, match="boto3"):
        get_node_provider_cls({"type": "aws"})({"type": "aws", "region": "us-west-2"}, "c")
