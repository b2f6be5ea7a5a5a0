"""Virtual provider container nodes (providers/virtual/containers.py; reference
providers/_private/virtual/virtual_container_scheduler.py): exclusive GPU slices passed
through by render node, NUMA-local cpusets, memory / shm limits, data disks, bridge network,
labels, allocation bookkeeping across launches and release on terminate -- against a fake
docker CLI on a synthetic 8-GPU / 2-socket host."""
import json

import pytest

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.node_provider import NodeLaunchException
from cloudtik_amd.providers.virtual.containers import ContainerScheduler, _ranges
from cloudtik_amd.providers.virtual.node_provider import VirtualNodeProvider

GPUS = [{"index": i, "render_minor": 128 + 8 * i, "numa": 0 if i < 4 else 1} for i in range(8)]
NUMA = {0: list(range(0, 64)), 1: list(range(64, 128))}


class FakeDocker:
    def __init__(self):
        self.containers = {}
        self.networks = set()
        self.n = 0

    def __call__(self, cmd):
        args = cmd[1:]
        if args[:2] == ["network", "inspect"]:
            return (0, "[]", "") if args[2] in self.networks else (1, "", "no such network")
        if args[:2] == ["network", "create"]:
            self.networks.add(args[-1])
            return 0, "", ""
        if args[0] == "run":
            name = args[args.index("--name") + 1]
            assert args[args.index("--network") + 1] in self.networks
            self.n += 1
            self.containers[name] = {"args": args, "ip": f"172.18.0.{self.n + 1}"}
            return 0, "cid", ""
        if args[0] == "inspect":
            c = self.containers[args[-1]]
            net = args and self.containers[args[-1]]["args"][c["args"].index("--network") + 1]
            return 0, json.dumps({net: {"IPAddress": c["ip"]}}), ""
        if args[:2] == ["rm", "-f"]:
            self.containers.pop(args[2], None)
            return 0, "", ""
        raise AssertionError(cmd)


def _provider(tmp_path, monkeypatch, docker, **cfg):
    monkeypatch.setenv("CLOUDTIK_LOCAL_STATE_DIR", str(tmp_path))
    pc = dict(type="virtual", use_containers=True, workspace_name="ws", _docker_runner=docker, _host_gpus=GPUS,
              _host_numa_cpus=NUMA, image="rocm/pytorch:test", **cfg)
    return VirtualNodeProvider(pc, "c1")


def _arg(args, flag):
    return [args[i + 1] for i, a in enumerate(args) if a == flag]


def test_container_nodes_get_exclusive_numa_local_slices(tmp_path, monkeypatch):
    docker = FakeDocker()
    p = _provider(tmp_path, monkeypatch, docker)
    worker = {"resources": {"CPU": 16, "GPU": 4}, "memory": "64g", "data_disks": 2, "data_dirs": ["/data/imagenet"]}
    a = p.create_node(worker, {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 1)
    b = p.create_node(worker, {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 1)
    (na, ia), (nb, ib) = next(iter(a.items())), next(iter(b.items()))
    assert ia["alloc"]["gpus"] == [0, 1, 2, 3] and ib["alloc"]["gpus"] == [4, 5, 6, 7]
    assert max(ia["alloc"]["cpus"]) < 64 and min(ib["alloc"]["cpus"]) >= 64          # NUMA-local cores
    args = docker.containers[na]["args"]
    assert _arg(args, "--device") == ["/dev/kfd", "/dev/dri/renderD128", "/dev/dri/renderD136",
                                      "/dev/dri/renderD144", "/dev/dri/renderD152"]
    assert _arg(args, "--cpuset-cpus") == ["0-15"] and _arg(args, "--memory") == ["65536m"]
    assert _arg(args, "--shm-size") == ["19660m"]
    vols = _arg(args, "-v")
    assert any(v.endswith(":/mnt/cloudtik/data_disk_2") for v in vols)
    assert "/data/imagenet:/cloudtik/data/imagenet" in vols
    assert "cloudtik-cluster-name=c1" in _arg(args, "--label") and "cloudtik-ws" in docker.networks
    assert args[-3:] == ["rocm/pytorch:test", "sleep", "infinity"]
    assert p.internal_ip(na) == "172.18.0.2" and p.internal_ip(nb) == "172.18.0.3"
    with pytest.raises(NodeLaunchException, match="GPUs"):
        p.create_node(worker, {}, 1)                                        # the host is full
    p.terminate_node(na)
    assert na not in docker.containers
    c = p.create_node(worker, {}, 1)
    assert next(iter(c.values()))["alloc"]["gpus"] == [0, 1, 2, 3]            # freed slice reused
    p.cleanup_cluster({}, deep=True)
    assert not docker.containers


def test_scheduler_cpu_spill_and_reserve():
    s = ContainerScheduler(GPUS[:2], {0: [0, 1, 2, 3], 1: [4, 5, 6, 7]}, reserve_cpus=2)
    a = s.allocate({}, 1, 4)
    assert a == {"gpus": [0], "cpus": [2, 3, 4, 5]}                         # reserved 0,1; spills to node 1
    with pytest.raises(NodeLaunchException, match="CPUs"):
        s.allocate({"x": a}, 0, 3)
    assert _ranges([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8"


def test_container_executor_runs_inside(tmp_path, monkeypatch):
    docker = FakeDocker()
    p = _provider(tmp_path, monkeypatch, docker)
    nid = next(iter(p.create_node({"resources": {"CPU": 2}}, {}, 1)))

    class Runner:
        def __init__(self):
            self.cmds = []

        def check_call(self, cmd, **kw):
            self.cmds.append(cmd)
            return 0

        def check_output(self, cmd, **kw):
            self.cmds.append(cmd)
            return b"ok"

    r = Runner()
    ex = p.get_command_executor(None, "", nid, {}, "c1", r, True)
    assert ex.run("echo hi", with_output=True) == b"ok"
    assert r.cmds[-1][:4] == ["docker", "exec", nid, "bash"]
    ex.run_rsync_up("/tmp/x", "/root/y/z")
    assert r.cmds[-1] == ["docker", "cp", "/tmp/x", f"{nid}:/root/y/z"]


def test_reference_virtual_node_config_format(tmp_path, monkeypatch):
    """The reference's virtual configs size nodes with instance_type {CPU, memory} and give
    data_disks as host disk roots (examples/lab/config/*.yaml)."""
    docker = FakeDocker()
    p = _provider(tmp_path, monkeypatch, docker)
    disks = tmp_path / "disks"
    nc = {"instance_type": {"CPU": 4, "memory": "4G"}, "data_disks": [str(disks)], "data_dirs": [str(tmp_path / "share")]}
    nid, node = next(iter(p.create_node(nc, {T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 1).items()))
    args = docker.containers[nid]["args"]
    assert len(node["alloc"]["cpus"]) == 4 and _arg(args, "--memory") == ["4096m"]
    assert f"{disks}/{nid}:/mnt/cloudtik/data_disk_1" in _arg(args, "-v") and (disks / nid).is_dir()
    p.terminate_node(nid)
    assert not (disks / nid).exists()


@pytest.mark.skipif(not __import__("os").path.isdir("/root/reference/examples/lab/config"),
                    reason="reference lab configs not present")
def test_reference_lab_configs_bootstrap(tmp_path):
    import glob
    import os
    from cloudtik_amd.core.cluster_config import load_cluster_config
    src = "/root/reference/examples/lab/config"
    for f in sorted(glob.glob(f"{src}/*.yaml")):
        text = open(f).read().replace("{%user%}", "cloudtik")
        dst = tmp_path / os.path.basename(f)
        dst.write_text(text)
    # the lab's inheritance (from: bootstrap / lab) resolves against its own directory
    for f in sorted(tmp_path.glob("*.yaml")):
        cfg = load_cluster_config(str(f))
        assert cfg["provider"]["type"] == "virtual", f
