"""Config compatibility: every reference example cluster YAML bootstraps (instance templates
``from: aws/gpu/t4/standard`` etc. are generated), every generated template is well formed,
and the runtime / workspace / storage / database schemas validate keys and types."""
import glob
import os

import pytest

from cloudtik_amd.core.config import schema as jschema
from cloudtik_amd.core.config.instance_templates import available, synthesize

REF = "/root/reference/examples/cluster"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference examples not present")
def test_every_reference_example_cluster_bootstraps(monkeypatch, tmp_path):
    from cloudtik_amd.core.cluster_config import load_cluster_config
    from cloudtik_amd.providers.cloud import keypairs
    # no cloud API here: the key-pair step sees a cloud without key pairs and a fresh ~/.ssh
    monkeypatch.setenv("HOME", str(tmp_path))
    orig = keypairs.configure_cloud_key_pair
    monkeypatch.setattr(keypairs, "configure_cloud_key_pair",
                        lambda cfg, cloud, region, describe, create: orig(cfg, cloud, region, lambda n: False,
                                                                          lambda n: "PRIVATE KEY"))
    files = [f for f in sorted(glob.glob(f"{REF}/**/*.yaml", recursive=True))
             if not f.endswith("example-cloud-simulator-config.yaml")]      # simulator config, not a cluster
    assert len(files) >= 45
    for f in files:
        cfg = load_cluster_config(f)
        assert cfg["provider"]["type"] and cfg["available_node_types"], f


def test_generated_templates_are_well_formed():
    names = available()
    assert len(names) > 150
    for n in names:
        t = synthesize(n)
        assert t and t["provider"]["type"] == n.split("/")[0], n
        nts = t["available_node_types"]
        assert "head.default" in nts and nts["head.default"]["node_config"], n
    assert synthesize("aws/gpu/t4/standard")["available_node_types"]["worker.default"]["resources"]["GPU"] == 1
    assert synthesize("azure/gpu/mi300x/very-large")["available_node_types"]["worker.default"]["node_config"][
        "azure_arm_parameters"]["vmSize"] == "Standard_ND96isr_MI300X_v5"
    assert synthesize("kubernetes/eks/small")["provider"]["cloud_provider"]["type"] == "aws"
    assert synthesize("aws/nonexistent") is None and synthesize("nope/standard") is None


def _rt_schema():
    from cloudtik_amd.core.cluster_config import load_schema
    return load_schema("runtime")


def test_runtime_schema_keys_and_types():
    s = _rt_schema()
    good = {"types": ["ai", "spark", "hdfs", "yarn"], "ai": {"with_gpu": True, "rccl": {"min_channels": 8}},
            "spark": {"hive_metastore_uri": "thrift://h:9083", "metastore_service_selector": {"runtimes": ["metastore"]}},
            "hdfs": {"dfs_replication": 2}, "yarn": {"scaling": {"scaling_mode": "apps-pending", "scaling_step": 2}},
            "scaling": {"scaling_policy": "scaling-with-load"}, "kafka": {"zookeeper_connect": "z:2181"},
            "mycustom": {"anything": 1}}
    jschema.validate(good, s)
    for bad in ({"hdfs": {"dfs_replicaton": 2}},                       # typo -> unknown key
                {"yarn": {"yarn_scheduler": "fifo"}},                  # not an allowed scheduler
                {"ai": {"with_gpu": 3}},                               # wrong type
                {"postgres": {"port": 70000}},                         # out of range
                {"scaling": {"scaling_policy": "scale-by-magic"}},
                {"spark": {"metastore_service_selector": {"runtime": ["x"]}}}):
        with pytest.raises(jschema.ValidationError):
            jschema.validate(bad, s)


def test_cluster_validation_uses_runtime_schema():
    from cloudtik_amd.core.cluster_config import validate_config
    cfg = {"cluster_name": "c", "provider": {"type": "local"}, "head_node_type": "h", "max_workers": 0,
           "available_node_types": {"h": {"node_config": {}, "max_workers": 0}},
           "runtime": {"types": ["hdfs"], "hdfs": {"bogus_key": 1}}}
    with pytest.raises(jschema.ValidationError, match="runtime"):
        validate_config(cfg)


@pytest.mark.parametrize("kind,ok,bad", [
    ("workspace", {"workspace_name": "ws1", "provider": {"type": "aws"}}, {"workspace_name": "WS_1", "provider": {}}),
    ("storage", {"storage_name": "s1", "provider": {"type": "gcp"}, "storage": {"bucket": "b"}},
     {"storage_name": "s1", "provider": {"type": "gcp"}, "storage": {"bucket": 3}}),
    ("database", {"database_name": "d1", "provider": {"type": "azure"}, "database": {"engine": "mysql"}},
     {"database_name": "d1", "provider": {"type": "azure"}, "database": {"engine": "oracle"}}),
])
def test_object_schemas(kind, ok, bad):
    from cloudtik_amd.core.cluster_config import load_schema
    s = load_schema(kind)
    jschema.validate(ok, s)
    with pytest.raises(jschema.ValidationError):
        jschema.validate(bad, s)
