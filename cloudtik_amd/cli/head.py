"""``cloudtik head ...``: cluster commands run ON the head against its bootstrap config
(reference scripts/head_scripts.py:62-1076)."""
from __future__ import annotations

import json
import os

import click
import yaml

DEFAULT_BOOTSTRAP_CONFIG = "~/cloudtik_bootstrap_config.yaml"


def _cfg():
    p = os.path.expanduser(DEFAULT_BOOTSTRAP_CONFIG)
    if not os.path.exists(p):
        raise click.ClickException(f"not a head node: {p} missing")
    with open(p) as f:
        return yaml.safe_load(f)


@click.group()
def head():
    """Commands run on the head node."""


@head.command()
def info():
    from cloudtik_amd.core import cluster_operator as op
    click.echo(json.dumps(op.get_cluster_info(_cfg()), indent=2, default=str))


@head.command()
def status():
    from cloudtik_amd.core import cluster_operator as op
    for n in op.get_cluster_nodes_info(_cfg()):
        click.echo(f"{n['node_id']}\t{n['node_ip']}\t{n['node_kind']}\t{n['node_type']}\t{n['node_status']}")


@head.command(name="worker-ips")
def worker_ips():
    from cloudtik_amd.core import cluster_operator as op
    for ip in op.get_worker_node_ips(_cfg()):
        click.echo(ip)


@head.command()
@click.option("--cpus", type=int, default=None)
@click.option("--gpus", type=int, default=None)
@click.option("--workers", type=int, default=None)
def scale(cpus, gpus, workers):
    from cloudtik_amd.core import cluster_operator as op
    op.scale_cluster(_cfg(), cpus, gpus, workers)


@head.command()
@click.option("--workers-only", is_flag=True, default=True)
@click.option("--keep-min-workers", is_flag=True, default=False)
def teardown(workers_only, keep_min_workers):
    from cloudtik_amd.core import cluster_operator as op
    op.teardown_cluster(_cfg(), workers_only=True, keep_min_workers=keep_min_workers)


@head.command(name="health-check")
def health_check():
    from cloudtik_amd.core import cluster_operator as op
    r = op.health_check(_cfg())
    click.echo(json.dumps(r, indent=2))
    if not r["healthy"]:
        raise SystemExit(1)


@head.command(name="exec", context_settings={"ignore_unknown_options": True})
@click.argument("cmd", nargs=-1, required=True)
@click.option("--node-ip", default=None)
@click.option("--all-nodes", is_flag=True, default=False)
def exec_cmd(cmd, node_ip, all_nodes):
    from cloudtik_amd.core import cluster_operator as op
    op.exec_cluster(_cfg(), " ".join(cmd), node_ip, all_nodes)
