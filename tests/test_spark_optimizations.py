"""Spark SQL optimizations of the analytics runtime (reference: the optimized-Spark patch set
source/runtime/spark/*/optimizations/*.patch and its switches,
docs/source/UserGuide/RunningOptimizedAnalytics/spark-optimizations.md): the properties a
cluster's runtime.spark.optimizations renders for a patched build and for upstream Spark
versions, and their way into spark-defaults.conf."""
import pytest

from cloudtik_amd.runtime.hadoop.spark_optimizations import (OPTIMIZATIONS, render_properties,
                                                            spark_optimization_properties)


def _by_source(entries):
    out = {}
    for name, k, v, src in entries:
        out.setdefault(name, set()).add(src)
    return out


def test_patched_build_uses_the_patch_set_switches():
    e = spark_optimization_properties("3.2.1", "all", optimized_build=True)
    props = {k: v for _, k, v, _ in e if k}
    assert props["spark.sql.rankLimit.enabled"] == "true"
    assert props["spark.sql.optimizer.sizeBasedJoinReorder.enabled"] == "true"
    assert props["spark.sql.optimizer.distinctBeforeIntersect.enabled"] == "true"
    assert props["spark.sql.optimizer.runtime.bloomFilter.enabled"] == "true"
    assert props["spark.sql.optimizer.mergeSingleRowAggregate.enabled"] == "true"
    assert props["spark.sql.optimizer.removeInSubqueryDuplicateJoins.enabled"] == "true"
    assert _by_source(e)["flatten_scalar_subquery"] == {"builtin"}     # rule always on once patched
    assert set(_by_source(e)) == set(OPTIMIZATIONS)


@pytest.mark.parametrize("version,runtime_filter,top_n,merge_scalar", [
    ("3.2.1", "unavailable", "unavailable", "unavailable"),
    ("3.3.0", "upstream", "unavailable", "unavailable"),
    ("3.4.1", "upstream", "unavailable", "builtin"),
    ("3.5.1", "upstream", "upstream", "builtin")])
def test_upstream_spark_gets_only_what_it_has(version, runtime_filter, top_n, merge_scalar):
    e = spark_optimization_properties(version, ["runtime_filter", "top_n", "flatten_scalar_subquery",
                                                "size_based_join_reorder"])
    src = _by_source(e)
    assert src["runtime_filter"] == {runtime_filter}
    assert src["top_n"] == {top_n}
    assert src["flatten_scalar_subquery"] == {merge_scalar}
    assert src["size_based_join_reorder"] == {"unavailable"}           # never upstreamed
    text = render_properties(e)
    assert "sizeBasedJoinReorder" not in text                          # no property that does nothing
    assert ("spark.sql.optimizer.runtime.bloomFilter.enabled" in text) == (runtime_filter == "upstream")


def test_selection_forms_and_typos():
    assert spark_optimization_properties("3.5.0", None) == []
    assert spark_optimization_properties("3.5.0", {"top_n": True, "runtime_filter": False})[0][0] == "top_n"
    with pytest.raises(ValueError, match="unknown Spark optimization"):
        spark_optimization_properties("3.5.0", ["runtime_filtre"])


def test_spark_defaults_carry_optimizations_and_user_config(tmp_path, monkeypatch):
    from cloudtik_amd.runtime.hadoop import SparkRuntime
    monkeypatch.setenv("RUNTIME_PATH", str(tmp_path))
    monkeypatch.setenv("CLOUDTIK_HEAD_IP", "10.0.0.1")
    monkeypatch.setenv("CLOUDTIK_NODE_CPUS", "16")
    monkeypatch.setenv("CLOUDTIK_NODE_MEMORY_MB", "65536")
    cfg = {"cluster_name": "t", "head_node_type": "head",
           "available_node_types": {"head": {"resources": {"CPU": 16, "memory": 64 * 1024 ** 3}},
                                    "worker": {"min_workers": 1, "resources": {"CPU": 16, "memory": 64 * 1024 ** 3}}},
           "runtime": {"types": ["spark"],
                       "spark": {"optimized_build": True, "optimizations": ["top_n", "distinct_before_intersect"],
                                 "config": {"spark.sql.shuffle.partitions": "512"}}}}
    rt = SparkRuntime({})
    cfg = rt.prepare_config(cfg)
    env = rt.with_environment_variables(cfg, None, "n1")
    assert "\n" not in env["SPARK_EXTRA_PROPERTIES"]                   # one exported line
    for k, v in env.items():
        monkeypatch.setenv(k, v.replace("$RUNTIME_PATH", str(tmp_path)))
    path = rt.render(head=True)["spark-defaults.conf"]
    conf = dict(line.split(None, 1) for line in open(path).read().splitlines()
                if line.strip() and not line.startswith("#"))
    assert conf["spark.sql.rankLimit.enabled"] == "true"
    assert conf["spark.sql.optimizer.distinctBeforeIntersect.enabled"] == "true"
    assert conf["spark.sql.shuffle.partitions"] == "512"
    assert "{%" not in open(path).read()
