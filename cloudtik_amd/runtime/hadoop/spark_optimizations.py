"""Spark SQL optimizations of the analytics runtime, as Spark properties.

The reference ships an optimized Spark: source patches against Spark 3.2.1 / 3.3.0
(``source/runtime/spark/spark-3.2.1/optimizations/0001-Runtime-Filter.patch`` ..
``0004-Distinct-Before-Intersect.patch``, ``spark-3.3.0/optimizations/0001-Top-N.patch`` ..
``0003-Flatten-Scalar-Subquery.patch``) whose rules are switched on by Spark properties
(``docs/source/UserGuide/RunningOptimizedAnalytics/spark-optimizations.md``).  Those are JVM
patches; this framework does not rebuild Spark.  What it carries is the switchboard: a
cluster's ``runtime.spark.optimizations`` names the optimizations to turn on, and this module
renders the properties that enable each one on the Spark that is actually installed --

* ``optimized_build: true`` (a Spark built with the reference patch set): the patch set's own
  properties;
* an upstream Spark: the upstream equivalent where the optimization was merged into Apache
  Spark (the row-level runtime bloom / semi-join filters in 3.3, scalar-subquery merging in
  3.4), and nothing where it was not (an unknown ``spark.sql.*`` key is silently accepted
  by Spark, which would suggest an optimization that does not run).

Each returned entry says which of the two it used, so ``cloudtik runtime configure`` output
and the tests can tell an enabled optimization from a skipped one.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

# name -> (properties of the patched build, minimum upstream version, upstream properties)
OPTIMIZATIONS: Dict[str, Tuple[Dict[str, str], Optional[Tuple[int, int]], Dict[str, str]]] = {
    # 0001-Runtime-Filter.patch (3.2.1), 0002-Runtime-Filter.patch (3.3.0); upstream SPARK-32268
    "runtime_filter": (
        {"spark.sql.optimizer.runtime.bloomFilter.enabled": "true",
         "spark.sql.optimizer.runtimeFilter.semiJoinReduction.enabled": "true"},
        (3, 3),
        {"spark.sql.optimizer.runtime.bloomFilter.enabled": "true",
         "spark.sql.optimizer.runtimeFilter.semiJoinReduction.enabled": "true"}),
    # 0002-Top-N.patch / 0001-Top-N.patch: RankLimit below row_number / rank / dense_rank filters
    # (upstream 3.5 plans a group limit for the same pattern: spark.sql.optimizer.windowGroupLimitThreshold)
    "top_n": (
        {"spark.sql.rankLimit.enabled": "true"},
        (3, 5),
        {"spark.sql.optimizer.windowGroupLimitThreshold": "1000"}),
    # 0003-Size-Based-Join-Reorder.patch (no upstream equivalent)
    "size_based_join_reorder": (
        {"spark.sql.optimizer.sizeBasedJoinReorder.enabled": "true"}, None, {}),
    # 0004-Distinct-Before-Intersect.patch (no upstream equivalent)
    "distinct_before_intersect": (
        {"spark.sql.optimizer.distinctBeforeIntersect.enabled": "true"}, None, {}),
    # 0003-Flatten-Scalar-Subquery.patch: the MergeScalarSubqueries rule, always on once patched
    # (no property; upstream Apache Spark 3.4 carries the rule, also always on)
    "flatten_scalar_subquery": ({}, (3, 4), {}),
    # flatten single-row aggregates under a cross join (no upstream equivalent)
    "flatten_single_row_aggregate": (
        {"spark.sql.optimizer.mergeSingleRowAggregate.enabled": "true"}, None, {}),
    # remove duplicate joins of IN subqueries (no upstream equivalent)
    "remove_in_subquery_duplicate_joins": (
        {"spark.sql.optimizer.removeInSubqueryDuplicateJoins.enabled": "true"}, None, {}),
}


def _version(v: str) -> Tuple[int, int]:
    parts = (str(v).split(".") + ["0", "0"])[:2]
    try:
        return int(parts[0]), int(parts[1])
    except ValueError:
        return 0, 0


def spark_optimization_properties(spark_version: str, optimizations, optimized_build: bool = False
                                  ) -> List[Tuple[str, str, str, str]]:
    """[(optimization, property, value, source)] for the requested optimizations, where source
    is ``patched`` (the patch set's property), ``upstream`` (the upstream equivalent), ``builtin``
    (always on in this upstream version: nothing to set) or ``unavailable`` (not in this Spark:
    no property emitted).  ``optimizations``: a list of names, ``{name: bool}``, or ``"all"``.
    Unknown names raise ValueError (a typo must not silently do nothing)."""
    if optimizations in (None, False):
        return []
    if optimizations in ("all", True):
        wanted = list(OPTIMIZATIONS)
    elif isinstance(optimizations, dict):
        wanted = [k for k, on in optimizations.items() if on]
    else:
        wanted = list(optimizations)
    bad = [w for w in wanted if w not in OPTIMIZATIONS]
    if bad:
        raise ValueError(f"unknown Spark optimization(s) {bad}; known: {sorted(OPTIMIZATIONS)}")
    ver = _version(spark_version)
    out: List[Tuple[str, str, str, str]] = []
    for name in wanted:
        patched, since, upstream = OPTIMIZATIONS[name]
        if optimized_build:
            if patched:
                out += [(name, k, v, "patched") for k, v in patched.items()]
            else:
                out.append((name, "", "", "builtin"))
        elif since is not None and ver >= since:
            if upstream:
                out += [(name, k, v, "upstream") for k, v in upstream.items()]
            else:
                out.append((name, "", "", "builtin"))
        else:
            out.append((name, "", "", "unavailable"))
    return out


def render_properties(entries) -> str:
    """spark-defaults.conf lines for the entries that set a property."""
    lines = [f"{k:<38} {v}" for _, k, v, src in entries if k]
    return "\n".join(lines)
