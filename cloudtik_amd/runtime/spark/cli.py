"""``cloudtik spark ...``: Spark runtime commands contributed to the CLI (reference
runtime/spark/scripts.py command group)."""
from __future__ import annotations

import json

import click


@click.group(name="spark")
def spark():
    """Spark runtime: YARN applications, endpoints and default storage of a cluster."""


@spark.command()
@click.argument("cluster_config_file")
@click.option("--app-id", default=None, help="One application (default: all).")
def applications(cluster_config_file, app_id):
    """List YARN applications (ResourceManager REST API through the head)."""
    from cloudtik_amd.runtime.spark.api import SparkCluster
    click.echo(json.dumps(SparkCluster(cluster_config_file).applications(app_id or ""), indent=2))


@spark.command()
@click.argument("cluster_config_file")
def endpoints(cluster_config_file):
    """Spark history server / Jupyter endpoints."""
    from cloudtik_amd.runtime.spark.api import SparkCluster
    click.echo(json.dumps(SparkCluster(cluster_config_file).get_endpoints(), indent=2))


@spark.command(name="default-storage")
@click.argument("cluster_config_file")
def default_storage(cluster_config_file):
    """fs.defaultFS the cluster's Spark jobs use."""
    from cloudtik_amd.runtime.spark.api import SparkCluster
    click.echo(json.dumps(SparkCluster(cluster_config_file).get_default_storage(), indent=2))
