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


# ---------------------------------------------------------------- cloud storage in core-site
from cloudtik_amd.runtime.hadoop import HadoopRuntime  # noqa: E402
from cloudtik_amd.runtime.hadoop import cloud_storage as cs  # noqa: E402


def _with_storage(provider):
    cfg = _cluster(types=("hadoop",))
    cfg["provider"] = provider
    return cfg


def test_hadoop_core_site_aws_keys_go_to_credential_store(node_env, monkeypatch):
    """Reference hadoop-cloud-credential.sh update_credential_config_for_aws: the access key
    in core-site, the secret only in the JCEKS store core-site points at."""
    cfg = _with_storage({"type": "aws", "storage": {"aws_s3_storage": {
        "s3.bucket": "b1", "s3.access.key.id": "AKIA1", "s3.secret.access.key": "s3cr3t"}}})
    rt = HadoopRuntime({})
    _export(rt, cfg, monkeypatch, node_env)
    path = rt.render(head=True)["core-site.xml"]
    core = _props(path)
    assert core["fs.defaultFS"] == "s3a://b1"
    assert core["fs.s3a.access.key"] == "AKIA1"
    assert core["hadoop.security.credential.provider.path"].startswith("jceks://file@" + str(node_env))
    assert "s3cr3t" not in open(path).read()
    steps = rt.configure_steps(True)
    assert any('credential create fs.s3a.secret.key -value "$AWS_S3_SECRET_ACCESS_KEY"' in s for s in steps)
    assert not any("s3cr3t" in s for s in steps)          # the value never enters a step string


def test_hadoop_core_site_instance_identities(node_env, monkeypatch):
    # no keys: instance profile, or web identity on EKS
    props, secrets = cs.cloud_storage_conf({"AWS_CLOUD_STORAGE": "true"})
    assert props["fs.s3a.aws.credentials.provider"].endswith("InstanceProfileCredentialsProvider") and not secrets
    props, _ = cs.cloud_storage_conf({"AWS_CLOUD_STORAGE": "true", "AWS_WEB_IDENTITY": "true"})
    assert props["fs.s3a.aws.credentials.provider"].endswith("WebIdentityTokenCredentialsProvider")


def test_azure_workload_identity_token_provider(node_env, monkeypatch):
    """N7 patch 0001: on AKS the projected pod identity feeds WorkloadIdentityTokenProvider
    (tenant, client id, authority, federated token file), all via the credential store."""
    env = cs.export_cloud_storage_env({"type": "azure", "tenant_id": "t0", "storage": {"azure_cloud_storage": {
        "azure.storage.type": "datalake", "azure.storage.account": "acct", "azure.container": "c"}}})
    assert cs.cloud_storage_uri(env) == "abfs://c@acct.dfs.core.windows.net"
    props, secrets = cs.cloud_storage_conf(env)
    assert props["fs.azure.account.oauth.provider.type"].endswith(".MsiTokenProvider")
    assert secrets == {"fs.azure.account.oauth2.msi.tenant": "t0"}
    env.update(AZURE_WORKLOAD_IDENTITY="true", AZURE_TENANT_ID="t1", AZURE_CLIENT_ID="cid",
               AZURE_FEDERATED_TOKEN_FILE="/var/run/secrets/azure/tokens/azure-identity-token",
               AZURE_AUTHORITY_HOST="https://login.microsoftonline.com/")
    props, secrets = cs.cloud_storage_conf(env)
    assert props["fs.azure.account.auth.type"] == "OAuth"
    assert props["fs.azure.account.oauth.provider.type"] == \
        "org.apache.hadoop.fs.azurebfs.oauth2.WorkloadIdentityTokenProvider"
    assert secrets["fs.azure.account.oauth2.msi.tenant"] == "t1"
    assert secrets["fs.azure.account.oauth2.client.id"] == "cid"
    assert secrets["fs.azure.account.oauth2.token.file"].endswith("azure-identity-token")
    assert "fs.azure.account.oauth2.msi.authority" in secrets
    # an account key wins over identities
    props, secrets = cs.cloud_storage_conf(dict(env, AZURE_ACCOUNT_KEY="k=="))
    assert props["fs.azure.account.auth.type"] == "SharedKey"
    assert secrets == {"fs.azure.account.key.acct.dfs.core.windows.net": "k=="}


def test_aliyun_ecs_ram_role_and_huawei_agency(node_env, monkeypatch):
    """N7 patch 0002: without OSS keys the ECS RAM role provider reads the role name from
    fs.oss.ecs.ramRoleName; Huawei Cloud uses the ECS agency provider."""
    env = cs.export_cloud_storage_env({"type": "aliyun", "region": "cn-hangzhou",
                                       "storage": {"aliyun_oss_storage": {"oss.bucket": "ob"}}})
    env["ALIYUN_ECS_RAM_ROLE_NAME"] = "cloudtik-worker-role"
    props, secrets = cs.cloud_storage_conf(env)
    assert props["fs.oss.credentials.provider"].endswith("AliyunEcsRamRoleCredentialsProvider")
    assert props["fs.oss.endpoint"] == "oss-cn-hangzhou-internal.aliyuncs.com"
    assert secrets == {"fs.oss.ecs.ramRoleName": "cloudtik-worker-role"}
    assert cs.cloud_storage_uri(env) == "oss://ob"
    keyed = dict(env, ALIYUN_OSS_ACCESS_KEY_ID="id", ALIYUN_OSS_ACCESS_KEY_SECRET="sk")
    props, secrets = cs.cloud_storage_conf(keyed)
    assert "fs.oss.credentials.provider" not in props and secrets["fs.oss.accessKeySecret"] == "sk"
    hw = cs.export_cloud_storage_env({"type": "huaweicloud", "region": "cn-north-4",
                                      "storage": {"huaweicloud_obs_storage": {"obs.bucket": "hb"}}})
    props, secrets = cs.cloud_storage_conf(hw)
    assert props["fs.obs.security.provider"] == "com.obs.services.EcsObsCredentialsProvider"
    assert props["fs.obs.endpoint"] == "obs.cn-north-4.myhuaweicloud.com" and not secrets
    # no cloud storage: nothing rendered, no credential steps
    rt = HadoopRuntime({})
    _export(rt, _cluster(types=("hadoop",)), monkeypatch, node_env)
    core = _props(rt.render(head=True)["core-site.xml"])
    assert "hadoop.security.credential.provider.path" not in core
    assert not any("credential create" in s for s in rt.configure_steps(True))


def test_kubernetes_cloud_provider_identities():
    env = cs.export_cloud_storage_env({"type": "kubernetes", "cloud_provider": {
        "type": "azure", "storage": {"azure_cloud_storage": {"azure.storage.account": "a", "azure.container": "c"}}}})
    assert env["AZURE_WORKLOAD_IDENTITY"] == "true" and cs.cloud_storage_kind(env) == "azure"
    props, _ = cs.cloud_storage_conf(dict(env, AZURE_CLIENT_ID="x"))
    assert props["fs.azure.account.oauth.provider.type"].endswith("WorkloadIdentityTokenProvider")
    env = cs.export_cloud_storage_env({"type": "kubernetes", "cloud_provider": {
        "type": "aws", "storage": {"aws_s3_storage": {"s3.bucket": "b"}}}})
    props, _ = cs.cloud_storage_conf(env)
    assert props["fs.s3a.aws.credentials.provider"].endswith("WebIdentityTokenCredentialsProvider")
