"""Head scaler / resource demand scheduler with the mock provider (reference test strategy:
tests/unit scaler tests over MockProvider + MockProcessRunner)."""
import copy
import json
import socket
import time

import pytest

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.head.resource_demand_scheduler import ResourceDemandScheduler, bin_pack


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


BASE = {
    "provider": {"type": "mock"},
    "available_node_types": {
        "head.default": {"node_config": {"instance_type": "m.head"}, "resources": {"CPU": 8}},
        "cpu.small": {"node_config": {"instance_type": "m.cpu"}, "resources": {"CPU": 4},
                      "min_workers": 0, "max_workers": 10},
        "gpu.mi355x": {"node_config": {"instance_type": "m.gpu"},
                       "resources": {"CPU": 128, "GPU": 8, "accelerator_type:MI355X": 8},
                       "min_workers": 0, "max_workers": 4},
    },
    "head_node_type": "head.default",
    "max_workers": 12,
    "runtime": {"types": ["ai"], "ai": {"with_gpu": True}},
    "options": {"idle_timeout_minutes": 5},
}


@pytest.fixture
def state(tmp_path):
    from cloudtik_amd.core.state.state_client import StateClient, StateServer
    srv = StateServer(port=_port(), data_dir=str(tmp_path)).start()
    yield StateClient.create(srv.address)
    srv.stop()


def _setup(name, state, mutate=None):
    from cloudtik_amd.core.cluster_config import bootstrap_config
    from cloudtik_amd.core.head.scaler import ClusterScaler
    from cloudtik_amd.core.provider_factory import get_node_provider
    from cloudtik_amd.providers.mock.node_provider import MockProvider
    MockProvider.reset(name)
    cfg = copy.deepcopy(BASE)
    cfg["cluster_name"] = name
    if mutate:
        mutate(cfg)
    cfg = bootstrap_config(cfg, no_config_cache=True)
    provider = get_node_provider(cfg["provider"], name, use_cache=False)
    return cfg, provider, ClusterScaler(cfg, provider, state, head_ip="10.0.0.1", synchronous=True)


def _workers(provider, name, status=None):
    out = provider.non_terminated_nodes({T.CLOUDTIK_TAG_CLUSTER_NAME: name, T.CLOUDTIK_TAG_NODE_KIND: "worker"})
    if status:
        out = [n for n in out if provider.node_tags(n).get(T.CLOUDTIK_TAG_NODE_STATUS) == status]
    return out


def test_scheduler_bin_packing_and_gpu_conservation():
    types = copy.deepcopy(BASE["available_node_types"])
    s = ResourceDemandScheduler(types, 12, "head.default")
    launch, infeasible = s.get_nodes_to_launch({}, {}, [{"CPU": 2}] * 5, {})
    assert launch == {"cpu.small": 3}               # CPU demands never pick the 8-GPU node
    launch, _ = s.get_nodes_to_launch({}, {}, [{"GPU": 8}] * 2 + [{"CPU": 1}], {})
    assert launch == {"gpu.mi355x": 2}              # the CPU bundle fits on a GPU node's spare CPUs
    launch, infeasible = s.get_nodes_to_launch({}, {}, [{"GPU": 16}], {})
    assert launch == {} and infeasible == [{"GPU": 16}]
    # free capacity of running nodes is used first
    launch, _ = s.get_nodes_to_launch({"cpu.small": 1}, {}, [{"CPU": 4}], {"n1": {"CPU": 4}})
    assert launch == {}
    # per-type max
    launch, _ = s.get_nodes_to_launch({"gpu.mi355x": 4}, {}, [{"GPU": 8}], {})
    assert launch == {}
    assert bin_pack([{"CPU": 3}, {"CPU": 2}], [{"CPU": 4}, {"CPU": 1}]) == [{"CPU": 2}]


def test_min_workers_launched_and_set_up(state):
    name = "sc-min"
    cfg, provider, scaler = _setup(name, state, lambda c: c["available_node_types"]["cpu.small"].update(min_workers=2))
    scaler.update()
    ws = _workers(provider, name, T.STATUS_UP_TO_DATE)
    assert len(ws) == 2
    cmds = provider.runner.commands_for(ws[0])
    assert any("runtime install ai" in c for c in cmds)
    assert any("node start --node-ip" in c and "--address=" in c for c in cmds)
    st = json.loads(state.kv_get(b"scaling_status", namespace="scaling"))
    assert st["workers"] == 2
    scaler.update()                                   # steady state: nothing new
    assert len(_workers(provider, name)) == 2


def test_max_workers_and_outdated_config(state):
    name = "sc-max"
    cfg, provider, scaler = _setup(name, state, lambda c: c["available_node_types"]["cpu.small"].update(
        min_workers=1, max_workers=2))
    scaler.update()
    from cloudtik_amd.core.cluster_utils import node_tags
    provider.create_node({"instance_type": "m.cpu"}, node_tags(cfg, "cpu.small", "worker", 7), 2)
    scaler.update()
    assert len(_workers(provider, name)) == 2
    # change the node config: every worker is replaced
    old = set(_workers(provider, name))
    new_cfg = copy.deepcopy(cfg)
    new_cfg["available_node_types"]["cpu.small"]["node_config"]["instance_type"] = "m.cpu2"
    scaler.reset_config(new_cfg)
    scaler.update()
    now = set(_workers(provider, name))
    assert now and not (now & old)


def test_failed_setup_is_replaced(state):
    name = "sc-fail"
    cfg, provider, scaler = _setup(name, state, lambda c: c["available_node_types"]["cpu.small"].update(min_workers=1))
    provider.runner.fail_cmds.append("runtime install ai")
    scaler.update()
    (n,) = _workers(provider, name)
    assert provider.node_tags(n)[T.CLOUDTIK_TAG_NODE_STATUS] == T.STATUS_UPDATE_FAILED
    provider.runner.fail_cmds.clear()
    scaler.update()                                   # terminate the failed node + launch a new one
    ws = _workers(provider, name, T.STATUS_UP_TO_DATE)
    assert len(ws) == 1 and ws[0] != n


def test_gpu_request_and_launch_failure_backoff(state):
    name = "sc-gpu"
    cfg, provider, scaler = _setup(name, state)
    state.kv_put(b"cluster_requests", json.dumps({"bundles": [{"GPU": 8}] * 2}), namespace="scaling")
    provider.fail_launches_of("m.gpu")
    scaler.update()
    st = scaler.summary()
    assert "gpu.mi355x" in st["failed_launches"] and not _workers(provider, name)
    provider.world["fail_launch"].clear()
    scaler.tracker.failures.clear()
    scaler.update()
    ws = _workers(provider, name, T.STATUS_UP_TO_DATE)
    assert len(ws) == 2 and all(provider.node_tags(w)[T.CLOUDTIK_TAG_USER_NODE_TYPE] == "gpu.mi355x" for w in ws)


def test_lost_heartbeat_triggers_recovery(state, monkeypatch):
    from cloudtik_amd.core import constants as C
    from cloudtik_amd.core.state.state_client import NODE_TABLE
    name = "sc-hb"
    cfg, provider, scaler = _setup(name, state, lambda c: c["available_node_types"]["cpu.small"].update(min_workers=1))
    scaler.update()
    (n,) = _workers(provider, name)
    monkeypatch.setattr(C, "CLOUDTIK_HEARTBEAT_TIMEOUT_S", 1)
    provider.set_node_tags(n, {"cloudtik-up-time": str(time.time() - 100)})
    state.table_put(NODE_TABLE, n, {"node_id": n, "node_ip": provider.internal_ip(n),
                                    "last_heartbeat_time": time.time() - 100})
    before = len(provider.runner.commands_for(n))
    scaler.update()
    after = provider.runner.commands_for(n)
    assert len(after) > before and any("node start" in c for c in after[before:])
    assert any("lost heartbeat" in e for e in scaler.events)


def test_idle_workers_scale_down_to_min(state):
    name = "sc-idle"
    cfg, provider, scaler = _setup(name, state, lambda c: (c["available_node_types"]["cpu.small"].update(
        min_workers=1), c["options"].update(idle_timeout_minutes=0.001)))
    state.kv_put(b"cluster_requests", json.dumps({"bundles": [{"CPU": 4}] * 3}), namespace="scaling")
    scaler.update()
    assert len(_workers(provider, name)) == 3
    state.kv_put(b"cluster_requests", json.dumps({"bundles": []}), namespace="scaling")
    scaler.update()                                   # records activity
    time.sleep(0.2)
    scaler.update()
    assert len(_workers(provider, name)) == 1


def test_scaling_with_load_requests_more_nodes():
    from cloudtik_amd.core.head.scaling_policies import ScalingWithLoad, create_scaling_policy
    cfg = copy.deepcopy(BASE)
    cfg["runtime"]["scaling"] = {"scaling_policy": "scaling-with-load", "scaling_step": 2}
    metrics = {"n1": {"cpu_count": 4, "load_avg": [3.9], "memory_total": 10, "memory_used": 1, "gpus": []},
               "n2": {"cpu_count": 4, "load_avg": [3.8], "memory_total": 10, "memory_used": 1, "gpus": []}}
    p = create_scaling_policy(cfg, "10.0.0.1", metrics_source=lambda: metrics)
    assert isinstance(p, ScalingWithLoad)
    st = p.get_scaling_state()
    assert len(st.autoscaling_instructions["resource_requests"]) == 1 + 2
    assert st.node_resource_states["n1"]["used"]["CPU"] == 3.9
    metrics["n1"]["load_avg"] = [0.1]
    metrics["n2"]["load_avg"] = [0.1]
    assert p.get_scaling_state().autoscaling_instructions["resource_requests"] == []
    # GPU-busy driven scaling
    cfg["runtime"]["scaling"] = {"scaling_policy": "scaling-with-load", "scaling_resource": "GPU"}
    p = create_scaling_policy(cfg, "10.0.0.1",
                              metrics_source=lambda: {"g": {"cpu_count": 128, "load_avg": [1],
                                                            "gpus": [{"busy_percent": 97}] * 8}})
    assert len(p.get_scaling_state().autoscaling_instructions["resource_requests"]) == 1


def test_scaling_with_time_table():
    from cloudtik_amd.core.head.scaling_policies import ScalingWithTime
    cfg = copy.deepcopy(BASE)
    cfg["available_node_types"]["cpu.small"]["min_workers"] = 2
    cfg["runtime"]["scaling"] = {"scaling_policy": "scaling-with-time", "scaling_math_base": "on-previous-time",
                                 "scaling_time_table": {"08:00": "+3", "12:00": "*2", "20:00": 1}}
    p = ScalingWithTime(cfg, "h")
    t = time.mktime(time.strptime("2026-01-05 13:00", "%Y-%m-%d %H:%M"))
    assert p.nodes_at(t) == 8                        # 1 (yesterday's 20:00) + 3 at 08:00, *2 at 12:00
    t = time.mktime(time.strptime("2026-01-05 07:00", "%Y-%m-%d %H:%M"))
    assert p.nodes_at(t) == 1                        # wraps from the previous day's 20:00 entry


def test_quorum_runtime_sets_up_complete_membership(state):
    name = "sc-quorum"

    def mutate(c):
        c["runtime"]["types"] = ["zookeeper"]
        c["runtime"]["zookeeper"] = {"minimal_nodes": 3}
        c["available_node_types"]["cpu.small"].update(min_workers=3)
        c["options"]["upscaling_speed"] = 0.1        # launches trickle in: max(5,...) still caps at 3 here
    cfg, provider, scaler = _setup(name, state, mutate)
    provider.create_node({}, {T.CLOUDTIK_TAG_CLUSTER_NAME: name, T.CLOUDTIK_TAG_NODE_KIND: "head",
                              T.CLOUDTIK_TAG_WORKSPACE_NAME: "default"}, 1)
    # launch only 2 first by shrinking min_workers, nothing may be set up
    scaler.config["available_node_types"]["cpu.small"]["min_workers"] = 2
    scaler.scheduler.node_types["cpu.small"]["min_workers"] = 2
    scaler.update()
    ws = _workers(provider, name)
    assert len(ws) == 2 and all(provider.node_tags(w)[T.CLOUDTIK_TAG_NODE_STATUS] == T.STATUS_UNINITIALIZED
                                for w in ws)
    scaler.config["available_node_types"]["cpu.small"]["min_workers"] = 3
    scaler.scheduler.node_types["cpu.small"]["min_workers"] = 3
    scaler.update()
    ws = _workers(provider, name, T.STATUS_UP_TO_DATE)
    assert len(ws) == 3
    qids = {provider.node_tags(w)[T.CLOUDTIK_TAG_QUORUM_ID] for w in ws}
    assert len(qids) == 1
    # the initial members form the quorum directly (no join); the runtime got the membership
    assert not any(T.CLOUDTIK_TAG_QUORUM_JOIN in provider.node_tags(w) for w in ws)
    (note,) = scaler.quorum.notifications
    assert note["runtimes"] == ["zookeeper"] and sorted(note["members"]) == sorted(ws)
    assert note["quorum_id"] == next(iter(qids))
    # the zookeeper runtime registered this ensemble in the workspace registry (head tags)
    from cloudtik_amd.core.provider_factory import get_workspace_provider
    from cloudtik_amd.core import service_discovery as sd
    gv = get_workspace_provider(cfg["provider"], "default").subscribe_global_variables(cfg)
    rec = sd.decode_service_address(gv[sd.service_global_key(name, "zookeeper-ensemble")])
    assert sorted(rec["hosts"]) == sorted(provider.internal_ip(w) for w in ws) and rec["quorum_id"] in qids


def _zk_types(c, zk_min=3, extra=None):
    """A dedicated ZooKeeper node type (its own runtime section) next to compute types."""
    c["available_node_types"]["zk.node"] = {"node_config": {"instance_type": "m.zk"}, "resources": {"CPU": 4},
                                            "min_workers": zk_min, "max_workers": 5, "launch_priority": 0,
                                            "runtime": {"types": ["zookeeper"]}}
    c["available_node_types"]["cpu.small"].update(min_workers=2, launch_priority=1)
    c["max_workers"] = 20
    c.setdefault("options", {})["launch_with_strong_priority"] = True
    if extra:
        extra(c)


def _by_type(provider, name, nt):
    return [w for w in _workers(provider, name) if provider.node_tags(w)[T.CLOUDTIK_TAG_USER_NODE_TYPE] == nt]


def test_per_node_type_quorum_gates_other_types(state, monkeypatch):
    """Reference quorum_manager.py:299,341,430: the constraint is per node type (only zk.node
    runs ZooKeeper); with launch_with_strong_priority the compute type launches only once every
    zk node is up to date; the runtime hook receives head + member info and the quorum id."""
    from cloudtik_amd.runtime.catalog import CatalogRuntime
    seen = []
    monkeypatch.setattr(CatalogRuntime, "node_constraints_reached",
                        lambda self, cfg, nt, head, nodes, quorum_id=None: seen.append((self.name, nt, head, nodes,
                                                                                        quorum_id)))
    name = "sc-quorum-types"
    cfg, provider, scaler = _setup(name, state, _zk_types)
    assert set(scaler.quorum.constraints) == {"zk.node"}
    c = scaler.quorum.constraints["zk.node"]
    assert (c.minimal, c.quorum, c.scalable, c.runtimes) == (3, True, True, ["zookeeper"])
    scaler.update()
    zk = _by_type(provider, name, "zk.node")
    assert len(zk) == 3 and not _by_type(provider, name, "cpu.small")      # compute waits (priority)
    assert all(provider.node_tags(w)[T.CLOUDTIK_TAG_NODE_STATUS] == T.STATUS_UP_TO_DATE for w in zk)
    (rt, nt, head, nodes, qid), = seen
    assert rt == "zookeeper" and nt == "zk.node" and sorted(nodes) == sorted(zk) and qid
    assert head["node_seq_id"] == T.CLOUDTIK_TAG_HEAD_NODE_SEQ_ID
    assert all(nodes[w]["node_ip"] == provider.internal_ip(w) and nodes[w]["quorum_id"] == qid for w in zk)
    assert json.loads(state.kv_get(b"cluster_nodes_info_zk.node", namespace="cluster")).keys() == set(zk)
    # strong priority: while a zk node is not up to date, compute may not launch
    provider.set_node_tags(zk[0], {T.CLOUDTIK_TAG_NODE_STATUS: T.STATUS_SETTING_UP})
    scaler.quorum.update(_workers(provider, name), {}, {})
    assert scaler.quorum.is_launch_allowed("cpu.small") == (False, None)
    provider.set_node_tags(zk[0], {T.CLOUDTIK_TAG_NODE_STATUS: T.STATUS_UP_TO_DATE})
    scaler.update()
    assert len(_by_type(provider, name, "cpu.small")) == 2
    assert not any(T.CLOUDTIK_TAG_QUORUM_ID in provider.node_tags(w) for w in _by_type(provider, name, "cpu.small"))


def test_scalable_quorum_grows_one_joining_node_at_a_time(state, monkeypatch):
    from cloudtik_amd.runtime.catalog import CatalogRuntime
    seen = []
    monkeypatch.setattr(CatalogRuntime, "node_constraints_reached",
                        lambda self, cfg, nt, head, nodes, quorum_id=None: seen.append((sorted(nodes), quorum_id)))
    name = "sc-quorum-join"
    cfg, provider, scaler = _setup(name, state, _zk_types)
    scaler.update()
    zk = sorted(_by_type(provider, name, "zk.node"))
    qid = provider.node_tags(zk[0])[T.CLOUDTIK_TAG_QUORUM_ID]
    provider.terminate_node(zk[0])                          # 2 of 3 left: the quorum keeps its majority
    scaler.update()
    now = sorted(_by_type(provider, name, "zk.node"))
    (joiner,) = set(now) - set(zk)
    t = provider.node_tags(joiner)
    assert t[T.CLOUDTIK_TAG_QUORUM_ID] == qid                # joined the running quorum
    assert t[T.CLOUDTIK_TAG_QUORUM_JOIN] == T.QUORUM_JOIN_STATUS_SUCCESS
    assert seen[-1] == (sorted(now), qid)                    # runtime told about the new member set
    # while a join is in progress no second node launches
    provider.set_node_tags(joiner, {T.CLOUDTIK_TAG_QUORUM_JOIN: T.QUORUM_JOIN_STATUS_INIT})
    scaler.quorum.update(_workers(provider, name), {}, {})
    assert scaler.quorum.is_launch_allowed("zk.node") == (False, None)


def test_unscalable_quorum_lost_majority_is_replaced(state, monkeypatch):
    """MinIO-like quorum (not scalable): members of a quorum below its majority are terminated
    (terminate_for_quorum) and a fresh quorum forms on new nodes; a healthy non-scalable quorum
    launches nothing."""
    from cloudtik_amd.runtime import catalog
    monkeypatch.setitem(catalog.QUORUM_CONSTRAINTS, "zookeeper", (True, True, False))
    name = "sc-quorum-minio"
    cfg, provider, scaler = _setup(name, state, _zk_types)
    scaler.update()
    zk = sorted(_by_type(provider, name, "zk.node"))
    qid = provider.node_tags(zk[0])[T.CLOUDTIK_TAG_QUORUM_ID]
    provider.terminate_node(zk[0])
    scaler.update()                      # majority kept, not scalable: no replacement launched
    assert sorted(_by_type(provider, name, "zk.node")) == zk[1:]
    provider.terminate_node(zk[1])       # 1 of 3: the quorum lost its majority
    scaler.update()                      # the last member goes; the scheduler relaunches 3
    scaler.update()
    now = _by_type(provider, name, "zk.node")
    assert zk[2] not in now and len(now) == 3
    qids = {provider.node_tags(w)[T.CLOUDTIK_TAG_QUORUM_ID] for w in now}
    assert len(qids) == 1 and qids != {qid}


def test_unhealthy_gpu_node_is_replaced(state, monkeypatch):
    """A worker whose GPUs keep reporting uncorrectable RAS errors is terminated and a
    replacement is launched (SURVEY.md §5.3 GPU health)."""
    from cloudtik_amd.core import constants as C
    from cloudtik_amd.core.state.state_client import NODE_METRICS_TABLE, NODE_TABLE
    name = "sc-gpuhealth"
    cfg, provider, scaler = _setup(name, state, lambda c: c["available_node_types"]["gpu.mi355x"].update(min_workers=1))
    scaler.update()
    (n,) = _workers(provider, name)
    monkeypatch.setattr(C, "CLOUDTIK_GPU_UNHEALTHY_TIMEOUT_S", 0)
    state.table_put(NODE_TABLE, n, {"node_id": n, "node_ip": provider.internal_ip(n),
                                    "last_heartbeat_time": time.time()})
    state.table_put(NODE_METRICS_TABLE, n, {"node_id": n, "gpu_healthy": False,
                                            "gpu_health_issues": ["gpu3: umc: 2 uncorrectable error(s)"]})
    scaler.update()
    assert any("GPUs unhealthy" in e and "umc" in e for e in scaler.events)
    scaler.update()
    now = _workers(provider, name)
    assert n not in now and len(now) == 1


def test_gpu_ras_health_from_sysfs(tmp_path):
    from cloudtik_amd.core.node.metrics import gpu_metrics
    card = tmp_path / "card0" / "device"
    (card / "ras").mkdir(parents=True)
    (card / "hwmon" / "hwmon0").mkdir(parents=True)
    (card / "vendor").write_text("0x1002\n")
    (card / "mem_info_vram_total").write_text(str(288 << 30))
    (card / "mem_info_vram_used").write_text("0")
    (card / "gpu_busy_percent").write_text("5")
    (card / "hwmon" / "hwmon0" / "temp1_input").write_text("45000")
    (card / "hwmon" / "hwmon0" / "temp2_input").write_text("61000")
    (card / "ras" / "umc_err_count").write_text("ue: 0\nce: 3\n")
    (card / "ras" / "xgmi_wafl_err_count").write_text("ue: 0\nce: 0\n")
    (g,) = gpu_metrics(str(tmp_path))
    assert g["healthy"] and g["ras"]["umc"] == {"ue": 0, "ce": 3} and g["temperature_max_c"] == 61.0
    (card / "ras" / "xgmi_wafl_err_count").write_text("ue: 1\nce: 0\n")
    (g,) = gpu_metrics(str(tmp_path))
    assert not g["healthy"] and "xgmi_wafl" in g["health_issues"][0]


def test_scaling_by_node_type_routes_metrics_and_bundles():
    """scaling-by-node-type (reference scaling_policies.py:595): CPU workers scale with load,
    GPU workers follow a time table; each requests bundles of its own type."""
    from cloudtik_amd.core.head.scaling_policies import ScalingByNodeType, create_scaling_policy
    cfg = {"head_node_type": "head",
           "available_node_types": {
               "head": {"resources": {"CPU": 8}},
               "cpu": {"min_workers": 1, "resources": {"CPU": 64, "memory": 256}},
               "gpu": {"min_workers": 0, "resources": {"CPU": 128, "GPU": 8}}},
           "runtime": {"scaling": {"scaling_policy_by_node_type": {
               "cpu": {"scaling_policy": "scaling-with-load", "scaling_resource": "CPU", "cpu_load_threshold": 0.5},
               "gpu": {"scaling_policy": "scaling-with-time", "scaling_time_table": {"00:00": 2}},
               "head": {"scaling_policy": "scaling-with-load"}}}}}
    metrics = {"n1": {"node_type": "cpu", "cpu_count": 64, "load_avg": [60.0], "resources": {"CPU": 64}},
               "n2": {"node_type": "gpu", "cpu_count": 128, "load_avg": [1.0], "resources": {"CPU": 128, "GPU": 8}},
               "n3": {"cpu_count": 8, "load_avg": [0.1]}}
    p = create_scaling_policy(cfg, "10.0.0.1", metrics_source=lambda: metrics)
    assert isinstance(p, ScalingByNodeType) and set(p.policies) == {"cpu", "gpu"}
    st = p.get_scaling_state()
    reqs = st.autoscaling_instructions["resource_requests"]
    assert sum(1 for r in reqs if r.get("GPU") == 8) == 2               # time table: 2 GPU nodes
    assert sum(1 for r in reqs if r.get("CPU") == 64 and "GPU" not in r) == 1   # load 0.94 > 0.5: +1 step
    assert set(st.node_resource_states) == {"n1", "n2", "n3"}


def _docker(c):
    c["docker"] = {"enabled": True, "image": "cloudtik/ai-rocm:latest", "container_name": "cloudtik-ai"}
    c["provider"]["cache_stopped_nodes"] = True
    c["available_node_types"]["cpu.small"].update(min_workers=1, max_workers=1)


def test_setup_commands_with_stopped_node_caching_docker(state):
    """Reference tests/unit/test_cloudtik.py:1507: with docker, a node restarted from the
    stopped-node cache keeps its runtime hash but its container is gone, so the container is
    started again (docker run) and the initialization + setup commands run again inside it."""
    name = "sc-docker-cache"
    cfg, provider, scaler = _setup(name, state, _docker)
    runner = provider.runner
    scaler.update()
    (w,) = _workers(provider, name, T.STATUS_UP_TO_DATE)
    cmds = runner.commands_for(w)
    assert any(c.startswith("docker pull cloudtik/ai-rocm:latest") for c in cmds)
    assert any(c.startswith("docker run") and "cloudtik/ai-rocm:latest" in c for c in cmds)
    setup_cmds = [c for c in cmds if "docker exec" in c and "runtime install ai" in c]
    assert setup_cmds                                    # setup ran INSIDE the container
    rh = provider.node_tags(w)[T.CLOUDTIK_TAG_RUNTIME_CONFIG]

    # stop the node (cached, not terminated); the scaler relaunches it from the cache
    provider.terminate_node(w)
    assert _workers(provider, name) == []
    runner.clear_history()
    scaler.update()
    (w2,) = _workers(provider, name)
    assert w2 == w                                      # the SAME node came back
    cmds = runner.commands_for(w)
    assert any(c.startswith("docker run") for c in cmds)
    assert any("docker exec" in c and "runtime install ai" in c for c in cmds)
    assert provider.node_tags(w)[T.CLOUDTIK_TAG_RUNTIME_CONFIG] == rh
    assert provider.node_tags(w)[T.CLOUDTIK_TAG_NODE_STATUS] == T.STATUS_UP_TO_DATE

    # container still running with the right image and mounts: nothing is re-run
    runner.respond_to_call(".State.Running", ["true"])
    runner.respond_to_call(".Config.Image", ["cloudtik/ai-rocm:latest"])
    runner.respond_to_call("json .Mounts", ["[]"])
    runner.clear_history()
    from cloudtik_amd.core.cluster_utils import create_updater
    u = create_updater(cfg, provider, w, is_head=False, head_ip="10.0.0.1")
    u.run()
    cmds = runner.commands_for(w)
    assert u.exitcode == 0 and not any(c.startswith("docker run") for c in cmds)
    assert not any("runtime install ai" in c for c in cmds)


def test_docker_container_restarted_when_image_changes(state):
    name = "sc-docker-image"
    cfg, provider, scaler = _setup(name, state, _docker)
    runner = provider.runner
    scaler.update()
    (w,) = _workers(provider, name, T.STATUS_UP_TO_DATE)
    runner.respond_to_call(".State.Running", ["true"])
    runner.respond_to_call(".Config.Image", ["cloudtik/ai-rocm:old"])     # drifted
    runner.respond_to_call("json .Mounts", ["[]"])
    runner.clear_history()
    from cloudtik_amd.core.cluster_utils import create_updater
    u = create_updater(cfg, provider, w, is_head=False, head_ip="10.0.0.1")
    u.run()
    cmds = runner.commands_for(w)
    assert u.exitcode == 0
    stop = [i for i, c in enumerate(cmds) if c.startswith("docker stop cloudtik-ai")]
    run = [i for i, c in enumerate(cmds) if c.startswith("docker run")]
    assert stop and run and stop[0] < run[0]
    assert any("docker exec" in c and "runtime install ai" in c for c in cmds)


def test_docker_file_mounts_bind_mounted_and_pull_policy(state, tmp_path):
    name = "sc-docker-mounts"
    src = tmp_path / "data"
    src.mkdir()

    def mut(c):
        _docker(c)
        c["file_mounts"] = {"/root/test-folder": str(src)}
        c["docker"]["pull_before_run"] = False

    cfg, provider, scaler = _setup(name, state, mut)
    runner = provider.runner
    scaler.update()
    (w,) = _workers(provider, name, T.STATUS_UP_TO_DATE)
    cmds = runner.commands_for(w)
    host_loc = f"/tmp/cloudtik_docker_mounts/{name}/root/test-folder"
    assert any(c.startswith("rsync-up") and host_loc in c for c in cmds)       # synced to the host location
    run = [c for c in cmds if c.startswith("docker run")][0]
    assert f"-v {host_loc}:/root/test-folder" in run                          # bind-mounted into the container
    assert any("image inspect cloudtik/ai-rocm:latest" in c and "|| docker pull" in c for c in cmds)
    assert not any(c.startswith("docker pull") for c in cmds)
    # a running container that lacks a requested mount is restarted
    runner.respond_to_call(".State.Running", ["true"])
    runner.respond_to_call(".Config.Image", ["cloudtik/ai-rocm:latest"])
    runner.respond_to_call("json .Mounts", ['[{"Destination": "/some/other"}]'])
    runner.clear_history()
    from cloudtik_amd.core.cluster_utils import create_updater
    u = create_updater(cfg, provider, w, is_head=False, head_ip="10.0.0.1")
    u.run()
    cmds = runner.commands_for(w)
    assert u.exitcode == 0 and any(c.startswith("docker stop") for c in cmds) and any(
        c.startswith("docker run") for c in cmds)


def test_docker_home_mounts_follow_image_user(state, tmp_path):
    """'~/' file mounts land in the IMAGE user's home (a non-root image: /home/cloudtik), and
    the drift check compares against the same place, so an up-to-date container is not
    restarted on the next update (reference docker_command_executor.py reads $HOME first)."""
    name = "sc-docker-home"
    src = tmp_path / "cfg"
    src.mkdir()

    def mut(c):
        _docker(c)
        c["file_mounts"] = {"~/conf": str(src)}

    cfg, provider, scaler = _setup(name, state, mut)
    runner = provider.runner
    runner.respond_to_call("--entrypoint printenv", ["/home/cloudtik"])
    scaler.update()
    (w,) = _workers(provider, name, T.STATUS_UP_TO_DATE)
    cmds = runner.commands_for(w)
    run = [c for c in cmds if c.startswith("docker run") and "--name" in c][0]
    assert f"-v /tmp/cloudtik_docker_mounts/{name}/conf:/home/cloudtik/conf" in run
    assert "/root/conf" not in run
    # the running container has the mount at /home/cloudtik/conf: no restart
    runner.respond_to_call(".State.Running", ["true"])
    runner.respond_to_call(".Config.Image", ["cloudtik/ai-rocm:latest"])
    runner.respond_to_call("json .Mounts", ['[{"Destination": "/home/cloudtik/conf"}]'])
    runner.clear_history()
    from cloudtik_amd.core.cluster_utils import create_updater
    u = create_updater(cfg, provider, w, is_head=False, head_ip="10.0.0.1", restart_only=True)
    provider.set_node_tags(w, {T.CLOUDTIK_TAG_FILE_MOUNTS_CONTENTS: "changed"})
    u.run()
    cmds = runner.commands_for(w)
    assert u.exitcode == 0 and not any(c.startswith("docker stop") for c in cmds)


def test_restart_only_with_changed_runtime_hash_starts_container(state):
    """restart_only drops only the setup commands: when the runtime hash changed and the
    container is not running, the initialization commands and the docker run still happen
    before the start commands (reference node_updater.py:467-537)."""
    name = "sc-docker-restart-only"
    cfg, provider, scaler = _setup(name, state, _docker)
    runner = provider.runner
    scaler.update()
    (w,) = _workers(provider, name, T.STATUS_UP_TO_DATE)
    provider.set_node_tags(w, {T.CLOUDTIK_TAG_RUNTIME_CONFIG: "old-hash"})
    runner.respond_to_call(".State.Running", ["false"])
    runner.clear_history()
    from cloudtik_amd.core.cluster_utils import create_updater
    u = create_updater(cfg, provider, w, is_head=False, head_ip="10.0.0.1", restart_only=True)
    u.run()
    cmds = runner.commands_for(w)
    assert u.exitcode == 0
    run = [i for i, c in enumerate(cmds) if c.startswith("docker run") and "--name" in c]
    start = [i for i, c in enumerate(cmds) if "docker exec" in c and "node start" in c]
    assert run and start and run[0] < start[0]
    assert not any("docker exec" in c and "runtime install ai" in c for c in cmds)   # no setup
