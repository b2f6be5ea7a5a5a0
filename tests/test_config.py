"""Config pipeline tests (reference test strategy: python/cloudtik/tests/unit/test_utils.py
config merge cases, schema validation of the example configs, encrypted config cache)."""
import copy
import os

import pytest
import yaml

from cloudtik_amd.core.config import crypto, schema
from cloudtik_amd.core.config.merge import merged_copy, update_nested_dict


def test_merge_nested_and_replace():
    base = {"a": {"b": 1, "c": [1, 2]}, "d": 1}
    out = merged_copy(base, {"a": {"c": [3]}, "e": 2})
    assert out == {"a": {"b": 1, "c": [3]}, "d": 1, "e": 2}
    assert base["a"]["c"] == [1, 2]  # merged_copy does not mutate


def test_merge_named_list_item():
    base = {"disks": [{"name": "boot", "size": 100, "type": "ssd"}]}
    out = merged_copy(base, {"disks": [{"name": "boot", "size": 200}]})
    assert out["disks"] == [{"name": "boot", "size": 200, "type": "ssd"}]
    # different names replace
    out = merged_copy(base, {"disks": [{"name": "data", "size": 5}]})
    assert out["disks"] == [{"name": "data", "size": 5}]


def test_merge_list_append_prepend():
    base = {"setup_commands": ["a", "b"]}
    out = merged_copy(base, {"setup_commands++": ["c"]})
    assert out["setup_commands"] == ["a", "b", "c"]
    out = merged_copy(base, {"++setup_commands": ["z"]})
    assert out["setup_commands"] == ["z", "a", "b"]
    out = merged_copy({}, {"x++": [1]})
    assert out["x"] == [1]


def test_update_nested_dict_flags():
    t = {"l": [{"name": "x", "v": 1}]}
    update_nested_dict(t, {"l": [{"name": "x", "w": 2}]}, match_list_item_with_name=False)
    assert t["l"] == [{"name": "x", "w": 2}]


def test_schema_validation_types_and_required():
    s = {"type": "object", "required": ["a"], "properties": {
        "a": {"type": "integer", "minimum": 0},
        "b": {"type": "array", "items": {"type": "string"}},
        "c": {"enum": ["x", "y"]}}, "additionalProperties": False}
    schema.validate({"a": 1, "b": ["s"], "c": "x"}, s)
    for bad in ({}, {"a": -1}, {"a": 1, "b": [1]}, {"a": 1, "c": "z"}, {"a": 1, "q": 1}):
        with pytest.raises(schema.ValidationError):
            schema.validate(bad, s)


def test_schema_refs_and_oneof():
    s = {"definitions": {"port": {"type": "integer", "maximum": 65535}},
         "type": "object", "properties": {"p": {"$ref": "#/definitions/port"},
                                          "q": {"anyOf": [{"type": "string"}, {"type": "null"}]}}}
    schema.validate({"p": 80, "q": None}, s)
    with pytest.raises(schema.ValidationError):
        schema.validate({"p": 70000}, s)


def test_aes_fips197_vector():
    # FIPS-197 appendix C.3 (AES-256)
    key = bytes(range(32))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    c = crypto.AESCipher(key)
    ct = c.encrypt_block(pt)
    assert ct.hex() == "8ea2b7ca516745bfeafc49904b496089"
    assert c.decrypt_block(ct) == pt


def test_aes_cbc_roundtrip_and_config_privacy():
    c = crypto.AESCipher(crypto.AESCipher.generate_key())
    for s in ["", "x", "a" * 15, "a" * 16, "héllo wörld" * 7]:
        assert c.decrypt(c.encrypt(s)) == s
    cfg = {"provider": {"type": "aws", "aws_credentials": {"secret_access_key": "S3CRET"}},
           "auth": {"ssh_password": "pw"}, "plain": "v"}
    enc = crypto.encrypt_config(copy.deepcopy(cfg))
    assert "S3CRET" not in str(enc)
    assert crypto.decrypt_config(enc) == cfg
    hidden = crypto.with_privacy(copy.deepcopy(cfg))
    assert "S3CRET" not in str(hidden) and hidden["plain"] == "v"


def test_template_yaml_files_parse():
    root = os.path.join(os.path.dirname(__file__), "..", "cloudtik_amd")
    n = 0
    for d, _, files in os.walk(root):
        for f in files:
            if f.endswith(".yaml"):
                with open(os.path.join(d, f)) as fh:
                    yaml.safe_load(fh)
                n += 1
    assert n >= 5


def test_bootstrap_local_template(tmp_path, monkeypatch):
    from cloudtik_amd.core import cluster_config as cc
    from cloudtik_amd.providers.local import node_provider as lnp
    monkeypatch.setattr(lnp, "STATE_DIR", str(tmp_path))
    monkeypatch.setattr(cc, "CONFIG_CACHE_DIR", str(tmp_path / "cache"))
    path = os.path.join(os.path.dirname(__file__), "..", "cloudtik_amd", "templates", "local",
                        "mi355x-8gpu.yaml")
    cfg = cc.load_cluster_config(path, override_cluster_name="t1")
    assert cfg["cluster_name"] == "t1"
    assert cfg["bootstrapped"]
    head = cfg["available_node_types"][cfg["head_node_type"]]
    assert head["resources"]["GPU"] == 8
    cmds = cfg["merged_commands"]
    assert any("node start --head" in c for c in cmds["head"]["start"])
    assert any("runtime install ai" in c for c in cmds["head"]["setup"])
    # second load hits the encrypted cache and gives the same config
    cfg2 = cc.load_cluster_config(path, override_cluster_name="t1")
    assert cfg2 == cfg
    assert os.listdir(tmp_path / "cache")


def test_validate_rejects_bad_head_type(tmp_path, monkeypatch):
    from cloudtik_amd.core import cluster_config as cc
    from cloudtik_amd.providers.local import node_provider as lnp
    monkeypatch.setattr(lnp, "STATE_DIR", str(tmp_path))
    cfg = {"cluster_name": "x", "provider": {"type": "local"}, "head_node_type": "nope",
           "available_node_types": {"head": {"node_config": {}, "resources": {"CPU": 1}}}}
    with pytest.raises(Exception):
        cc.bootstrap_config(cfg, no_config_cache=True)


def test_hash_launch_and_runtime_conf(tmp_path):
    from cloudtik_amd.core.cluster_config import hash_launch_conf, hash_runtime_conf
    a = hash_launch_conf({"instance_type": "x"}, {"ssh_user": "u", "ssh_private_key": "k"})
    b = hash_launch_conf({"instance_type": "y"}, {"ssh_user": "u", "ssh_private_key": "k"})
    assert a != b
    f = tmp_path / "f.txt"
    f.write_text("1")
    h1 = hash_runtime_conf({"/remote/f": str(f)}, None, {"x": 1})
    f.write_text("2")
    h2 = hash_runtime_conf({"/remote/f": str(f)}, None, {"x": 1})
    assert h1 != h2


def test_runtime_catalog_and_dependency_order():
    from cloudtik_amd.core import runtime_factory as rf
    names = rf.list_runtimes()
    for n in ["ai", "spark", "hdfs", "zookeeper", "kafka", "mysql", "prometheus", "grafana"]:
        assert n in names, n
    order = rf.reorder_runtimes_for_dependency(["kafka", "zookeeper"])
    assert order.index("zookeeper") < order.index("kafka")
    rt = rf.get_runtime("spark", {})
    services = rt.get_runtime_services({"cluster_name": "c"})
    assert services
    assert rt.get_head_service_ports()


def test_ai_runtime_env_and_services():
    from cloudtik_amd.core import runtime_factory as rf
    rt = rf.get_runtime("ai", {"with_gpu": True})
    env = rt.with_environment_variables({"runtime": {"ai": {"with_gpu": True}}}, None, "n1")
    assert any(k.startswith("NCCL_") or k.startswith("RCCL_") or k.startswith("HSA_") for k in env)
