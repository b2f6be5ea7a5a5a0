"""``cloudtik ai ...``: AI runtime commands contributed to the CLI (reference: runtime
command groups registered from runtime/<name>/scripts.py, scripts/scripts.py:66)."""
from __future__ import annotations

import json

import click


@click.group(name="ai")
def ai():
    """AI runtime: distributed launches and endpoints of a cluster."""


@ai.command(context_settings={"ignore_unknown_options": True})
@click.argument("cluster_config_file")
@click.argument("script")
@click.argument("script_args", nargs=-1, type=click.UNPROCESSED)
@click.option("--nproc-per-node", type=int, default=0, help="Ranks per node (default: one per GPU).")
@click.option("--head-only", is_flag=True, default=False)
def launch(cluster_config_file, script, script_args, nproc_per_node, head_only):
    """cloudtik-run SCRIPT over the head and every ready worker (one rank per GPU)."""
    from cloudtik_amd.runtime.ai.api import AICluster
    AICluster(cluster_config_file).run_distributed(script, list(script_args), all_nodes=not head_only,
                                                   nproc_per_node=nproc_per_node)


@ai.command()
@click.argument("cluster_config_file")
def endpoints(cluster_config_file):
    """The AI runtime's service endpoints (MLflow tracking server, ...)."""
    from cloudtik_amd.runtime.ai.api import AICluster
    click.echo(json.dumps(AICluster(cluster_config_file).get_endpoints(), indent=2))


@ai.command()
@click.argument("cluster_config_file")
def gpus(cluster_config_file):
    """GPUs of every node (rocm-smi product / memory / utilisation)."""
    from cloudtik_amd.core import cluster_operator as op
    op.exec_cluster(cluster_config_file, "hostname; rocm-smi --showproductname --showmeminfo vram --showuse "
                    "2>/dev/null || echo 'no ROCm GPU'", all_nodes=True)
