"""``cloudtik head ...``: cluster commands run ON the head against its bootstrap config
(reference scripts/head_scripts.py:62-1076)."""
from __future__ import annotations

import json
import os

import click

from cloudtik_amd.cli.dump_options import dump_options
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


# ---------------------------------------------------------------------- round-2 head commands
# (reference scripts/head_scripts.py:70-1054): the same operations as the top-level commands,
# against the head's own bootstrap config -- no config file argument, no SSH to the head.
def _cfg_file():
    p = os.path.expanduser(DEFAULT_BOOTSTRAP_CONFIG)
    if not os.path.exists(p):
        raise click.ClickException(f"not a head node: {p} missing")
    return p


@head.command()
@click.option("--node-ip", default=None, help="Attach to this worker instead of the head.")
def attach(node_ip):
    """Open an interactive shell on a node of this cluster."""
    from cloudtik_amd.core import cluster_operator as op
    raise SystemExit(op.attach_cluster(_cfg_file(), node_ip))


@head.command(context_settings={"ignore_unknown_options": True})
@click.argument("script")
@click.argument("script_args", nargs=-1, type=click.UNPROCESSED)
@click.option("--node-ip", default=None)
@click.option("--job-waiter", default=None)
def run(script, script_args, node_ip, job_waiter):
    """Run a built-in script (registered alias or runtime script) on the cluster."""
    from cloudtik_amd.core import cluster_operator as op
    op.run_script(_cfg_file(), script, list(script_args), node_ip=node_ip, job_waiter=job_waiter)


@head.command()
@click.argument("source")
@click.argument("target")
@click.option("--node-ip", default=None)
@click.option("--all-workers", is_flag=True, default=False)
def upload(source, target, node_ip, all_workers):
    """Copy a local file / directory to worker node(s)."""
    from cloudtik_amd.core import cluster_operator as op
    op.rsync(_cfg_file(), source, target, False, node_ip, all_workers)


@head.command()
@click.argument("source")
@click.argument("target")
@click.option("--node-ip", default=None)
def download(source, target, node_ip):
    """Copy a file / directory from a node to the head."""
    from cloudtik_amd.core import cluster_operator as op
    op.rsync(_cfg_file(), source, target, True, node_ip, False)


head.add_command(upload, name="rsync-up")
head.add_command(download, name="rsync-down")


@head.command(name="head-ip")
def head_ip():
    from cloudtik_amd.core import cluster_operator as op
    click.echo(op.get_head_node_ip(_cfg()))


@head.command()
@click.option("--lines", type=int, default=100)
@click.option("--follow", "-f", is_flag=True, default=False)
def monitor(lines, follow):
    """Tail the cluster controller log."""
    from cloudtik_amd.core import cluster_operator as op
    op.monitor_cluster(_cfg_file(), lines, follow)


@head.command()
@click.option("--node-ip", default=None)
@click.option("--runtime", "runtime_name", default=None, help="Only this runtime's log directory.")
@click.option("--lines", type=int, default=50)
def logs(node_ip, runtime_name, lines):
    """Show the tail of the runtime logs on a node (default: the head)."""
    from cloudtik_amd.core import cluster_operator as op
    from cloudtik_amd.core import runtime_factory as rf
    from cloudtik_amd.core.cluster_config import get_runtime_types
    cfg = _cfg()
    dirs = []
    for t in get_runtime_types(cfg):
        if runtime_name and t != runtime_name:
            continue
        for _, d in (rf.get_runtime(t, cfg["runtime"].get(t, {}) or {}).get_logs() or {}).items():
            dirs.append(d)
    dirs.append("/tmp/cloudtik/session_latest/logs")
    cmd = " ; ".join(f"for f in {d}/*.log {d}/*.out; do [ -f \"$f\" ] && echo \"==> $f\" && tail -n {lines} \"$f\"; "
                     f"done 2>/dev/null" for d in dirs)
    op.exec_cluster(cfg, cmd, node_ip)


@head.command(name="kill-node")
@click.option("--node-ip", default=None)
@click.option("--hard", is_flag=True, default=False)
@click.option("--yes", "-y", is_flag=True, default=False)
def kill_node(node_ip, hard, yes):
    """Kill a random (or the given) worker node."""
    from cloudtik_amd.core import cluster_operator as op
    if not yes:
        click.confirm("Kill a worker node?", abort=True)
    click.echo(op.kill_node(_cfg_file(), node_ip, hard))


@head.command(name="wait-for-ready")
@click.option("--min-workers", type=int, default=None)
@click.option("--timeout", type=int, default=1800)
def wait_for_ready(min_workers, timeout):
    """Block until min_workers workers are up-to-date."""
    from cloudtik_amd.core import cluster_operator as op
    click.echo(op.wait_for_ready(_cfg_file(), min_workers, timeout))


@head.command(name="process-status")
def process_status():
    """Runtime daemon processes on every node."""
    from cloudtik_amd.core import cluster_operator as op
    for nid, v in sorted(op.cluster_process_status(_cfg()).items()):
        click.echo(f"{nid}\t{json.dumps(v, default=str)}")


@head.command(name="cluster-dump")
@click.option("--output", "-o", default=None)
@click.option("--hosts", default=None, help="Only these nodes (IPs or node ids, comma separated).")
@click.option("--head-only", is_flag=True, default=False)
@click.option("--silent", is_flag=True, default=False)
@dump_options
def cluster_dump(output, hosts, head_only, silent, params):
    """Collect every node's logs, debug state, packages, processes and GPU state (in parallel)."""
    from cloudtik_amd.core import cluster_operator as op
    out = op.cluster_dump(_cfg_file(), output, hosts=hosts, head_only=head_only, params=params, on_head=True)
    if not silent:
        click.echo(out)


@head.command(name="debug-status")
def debug_status():
    """Scaling status published by the cluster controller."""
    from cloudtik_amd.core import cluster_operator as op
    click.echo(json.dumps(op.get_scaling_status(_cfg()), indent=2, default=str))


@head.command(name="resource-metrics")
def resource_metrics():
    """Per-node resource metrics (CPU load, memory, GPU busy) from the state service."""
    from cloudtik_amd.core import cluster_operator as op
    click.echo(json.dumps(op.get_cluster_metrics(_cfg()), indent=2, default=str))


@head.group(name="runtime")
def head_runtime():
    """Start / stop runtime services on the cluster's nodes."""


def _runtime_services(command, runtimes, node_ip, workers_only, yes):
    from cloudtik_amd.core import cluster_operator as op
    if not yes:
        click.confirm(f"{command} runtime services on the cluster?", abort=True)
    op.runtime_services(_cfg(), command, [r for r in (runtimes or "").split(",") if r] or None, node_ip=node_ip,
                        workers_only=workers_only)


@head_runtime.command(name="start")
@click.option("--runtimes", default=None, help="Comma-separated runtimes (default: all of the cluster).")
@click.option("--node-ip", default=None)
@click.option("--workers-only", is_flag=True, default=False)
@click.option("--yes", "-y", is_flag=True, default=False)
def runtime_start(runtimes, node_ip, workers_only, yes):
    _runtime_services("start", runtimes, node_ip, workers_only, yes)


@head_runtime.command(name="stop")
@click.option("--runtimes", default=None)
@click.option("--node-ip", default=None)
@click.option("--workers-only", is_flag=True, default=False)
@click.option("--yes", "-y", is_flag=True, default=False)
def runtime_stop(runtimes, node_ip, workers_only, yes):
    _runtime_services("stop", runtimes, node_ip, workers_only, yes)
