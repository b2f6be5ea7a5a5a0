"""Cluster benchmark drivers: TPC-DS on Spark, HiBench, Kafka, Presto/Trino power tests,
TPCx-AI.  ``python -m cloudtik_amd.benchmarks --help``."""
from .cluster_bench import HiBench, KafkaBench, SparkTPCDS, SQLEnginePowerTest, TPCxAI  # noqa: F401
