"""HDFS / YARN / Spark runtimes configure themselves: executor sizing (reference
runtime/spark/utils.py:102-156), rendered core-/hdfs-/yarn-site.xml and spark-defaults.conf,
the one-time namenode format in the start steps (recorded, not executed), spark-submit
commands, the YARN scaling policy and job waiter against canned ResourceManager replies
(style of reference tests/unit/test_cloudtik.py:91-205)."""
import os
import xml.etree.ElementTree as ET

import pytest

from cloudtik_amd.runtime.hadoop import (HdfsRuntime, SparkRuntime, YarnJobWaiter, YarnRuntime,
                                         YarnScalingPolicy, spark_executor_resource)


@pytest.mark.parametrize("cpu,cores,executors", [(16, 4, 4), (6, 6, 1), (10, 5, 2), (11, 6, 2), (18, 4, 5),
                                                 (2, 2, 1), (256, 4, 64)])
def test_spark_executor_cores(cpu, cores, executors):
    r = spark_executor_resource(cpu, 65536 * 4, 65536)
    assert r["spark_executor_cores"] == cores


def test_spark_executor_memory_and_driver():
    r = spark_executor_resource(16, 65536, 65536)
    # YARN share 52224 MB - (1024 app master + 1024) = 50176 over 4 executors -> 12 GB each,
    # minus 10% off-heap overhead
    assert r == {"spark_driver_memory": 6144, "spark_executor_cores": 4, "spark_executor_memory": 12288 - 1228}
    big = spark_executor_resource(256, 2 * 1024 * 1024, 2 * 1024 * 1024)   # 2 TiB MI355X node
    assert big["spark_driver_memory"] == 8192 and big["spark_executor_memory"] > 20000


def _cluster(types=("hdfs", "yarn", "spark"), workers=2):
    return {"cluster_name": "t", "head_node_type": "head", "min_workers": workers,
            "available_node_types": {
                "head": {"resources": {"CPU": 16, "memory": 64 * 1024 ** 3}},
                "worker": {"min_workers": workers, "resources": {"CPU": 16, "memory": 64 * 1024 ** 3, "GPU": 8}}},
            "runtime": {"types": list(types), "yarn": {"scaling": {"scaling_mode": "apps-pending"}}}}


def _props(path):
    return {p.find("name").text: (p.find("value").text or "") for p in ET.parse(path).getroot().findall("property")}


@pytest.fixture
def node_env(tmp_path, monkeypatch):
    monkeypatch.setenv("RUNTIME_PATH", str(tmp_path))
    monkeypatch.setenv("CLOUDTIK_HEAD_IP", "10.0.0.1")
    monkeypatch.setenv("CLOUDTIK_NODE_CPUS", "16")
    monkeypatch.setenv("CLOUDTIK_NODE_MEMORY_MB", "65536")
    return tmp_path


def _export(rt, cfg, monkeypatch, root):
    for k, v in rt.with_environment_variables(cfg, None, "n1").items():
        monkeypatch.setenv(k, v.replace("$RUNTIME_PATH", str(root)))


def test_hdfs_and_yarn_site_rendered(node_env, monkeypatch):
    cfg = _cluster()
    hdfs = HdfsRuntime({})
    cfg = hdfs.prepare_config(cfg)
    assert cfg["runtime"]["hdfs"]["dfs_replication"] == 2
    _export(hdfs, cfg, monkeypatch, node_env)
    out = hdfs.render(head=True)
    core = _props(out["core-site.xml"])
    site = _props(out["hdfs-site.xml"])
    assert core["fs.defaultFS"] == "hdfs://10.0.0.1:8020"
    assert site["dfs.replication"] == "2"
    assert site["dfs.namenode.rpc-address"] == "10.0.0.1:8020"
    assert site["dfs.namenode.name.dir"].startswith(str(node_env))
    yarn = YarnRuntime({})
    _export(yarn, cfg, monkeypatch, node_env)
    y = _props(yarn.render(head=False)["yarn-site.xml"])
    assert y["yarn.resourcemanager.hostname"] == "10.0.0.1"
    assert y["yarn.nodemanager.resource.memory-mb"] == str(52224)     # 64 GB x 0.8, whole GB
    assert y["yarn.nodemanager.resource.cpu-vcores"] == "16"
    assert "CapacityScheduler" in y["yarn.resourcemanager.scheduler.class"]
    assert not any("{%" in v for v in list(core.values()) + list(site.values()) + list(y.values()))


def test_spark_defaults_rendered_from_sizing(node_env, monkeypatch):
    cfg = SparkRuntime({}).prepare_config(_cluster())
    er = cfg["runtime"]["spark"]["spark_executor_resource"]
    assert er["spark_executor_cores"] == 4
    spark = SparkRuntime({})
    _export(spark, cfg, monkeypatch, node_env)
    path = spark.render(head=True)["spark-defaults.conf"]
    conf = dict(line.split(None, 1) for line in open(path).read().splitlines()
                if line.strip() and not line.startswith("#"))
    assert conf["spark.master"] == "yarn"
    assert conf["spark.executor.cores"] == "4"
    assert conf["spark.executor.memory"] == f"{er['spark_executor_memory']}m"
    assert conf["spark.eventLog.dir"] == "hdfs://10.0.0.1:8020/shared/spark-events"


def test_hdfs_start_formats_namenode_once(node_env, monkeypatch):
    import subprocess
    ran = []
    monkeypatch.setattr(subprocess, "run", lambda args, env=None, **kw: ran.append(args[-1]) or
                        subprocess.CompletedProcess(args, 0))
    HdfsRuntime({}).node_services("start", head=True)
    assert "namenode -format" in ran[0] and "current/VERSION" in ran[0]
    assert ran[1].endswith("--daemon start namenode")
    ran.clear()
    HdfsRuntime({}).node_services("start", head=False)
    assert ran == ["$HADOOP_HOME/bin/hdfs --daemon start datanode"]


def test_spark_runnable_commands():
    rt = SparkRuntime({})
    assert rt.get_runnable_command("/job/etl.py", ["--num-executors", "4"]) == \
        ["spark-submit", "--num-executors", "4", '"/job/etl.py"']
    assert rt.get_runnable_command("/job/a.jar", None) == ["spark-submit", '"/job/a.jar"']
    assert rt.get_runnable_command("/job/s.scala", None) == ["spark-shell", "-i", '"/job/s.scala"']
    assert rt.get_runnable_command("/job/x.sh", None) is None


METRICS = {"clusterMetrics": {"appsPending": 2, "appsRunning": 1, "availableMB": 512, "totalMB": 65536,
                              "availableVirtualCores": 2, "totalVirtualCores": 32}}
NODES = {"nodes": {"node": [
    {"nodeHostName": "127.0.0.2", "state": "RUNNING", "availableVirtualCores": 4, "usedVirtualCores": 12,
     "availMemoryMB": 1024, "usedMemoryMB": 31744},
    {"nodeHostName": "127.0.0.3", "state": "LOST", "availableVirtualCores": 0, "usedVirtualCores": 0,
     "availMemoryMB": 0, "usedMemoryMB": 0}]}}


def _fetch(path):
    return METRICS if path.endswith("metrics") else NODES


def test_yarn_scaling_policy_apps_pending_and_nodes():
    cfg = _cluster()
    p = YarnScalingPolicy(cfg, "10.0.0.1", fetch=_fetch)
    st = p.get_scaling_state()
    reqs = st.autoscaling_instructions["resource_requests"]
    assert len(reqs) == 1 and reqs[0]["GPU"] == 8 and reqs[0]["CPU"] == 16
    assert st.node_resource_states["127.0.0.2"]["total"]["CPU"] == 16
    assert st.node_resource_states["127.0.0.2"]["available"]["memory"] == 1024 << 20
    assert st.lost_nodes == {"127.0.0.3": "127.0.0.3"}
    # plenty of free memory -> nothing requested
    p2 = YarnScalingPolicy(cfg, "h", fetch=lambda path: {"clusterMetrics": dict(METRICS["clusterMetrics"],
                                                                                 availableMB=40000)}
                           if path.endswith("metrics") else NODES)
    assert p2.get_scaling_state().autoscaling_instructions["resource_requests"] == []


def test_yarn_scaling_policy_aggressive_cpu():
    cfg = _cluster()
    cfg["runtime"]["yarn"]["scaling"] = {"scaling_mode": "aggressive", "scaling_resource": "CPU", "scaling_step": 2,
                                         "aggressive_free_ratio_threshold": 0.1}
    p = YarnScalingPolicy(cfg, "h", fetch=_fetch)        # 2/32 vcores free < 10%
    assert len(p.get_scaling_state().autoscaling_instructions["resource_requests"]) == 2


def test_yarn_policy_and_waiter_from_runtime():
    from cloudtik_amd.core.head.scaling_policies import create_scaling_policy
    from cloudtik_amd.core.job_waiter import create_job_waiter
    cfg = _cluster()
    assert isinstance(create_scaling_policy(cfg, "10.0.0.1"), YarnScalingPolicy)
    assert isinstance(create_job_waiter(cfg, "yarn"), YarnJobWaiter)
    cfg["runtime"]["yarn"]["scaling"]["scaling_mode"] = "none"
    assert not isinstance(create_scaling_policy(cfg, "10.0.0.1"), YarnScalingPolicy)


def test_yarn_job_waiter_until_idle():
    seq = iter([(1, 0), (0, 2), (0, 0)])

    def fetch(path):
        p, r = next(seq)
        return {"clusterMetrics": {"appsPending": p, "appsRunning": r}}
    assert YarnJobWaiter({}, fetch=fetch, interval=0).wait_for_completion("n", "cmd")
    with pytest.raises(TimeoutError):
        YarnJobWaiter({}, fetch=lambda p: {"clusterMetrics": {"appsPending": 1, "appsRunning": 0}},
                      interval=0).wait_for_completion("n", "cmd", timeout=0)
