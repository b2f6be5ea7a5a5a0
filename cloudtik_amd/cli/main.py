"""``cloudtik`` command line (reference python/cloudtik/scripts/scripts.py:69-1560 -- cluster
commands; workspace.py / storage.py / database.py; node_scripts.py; runtime_scripts.py;
head_scripts.py).  Same command names and options so existing scripts keep working:

    cloudtik start|up CONFIG            cloudtik stop|down CONFIG
    cloudtik exec CONFIG CMD            cloudtik submit CONFIG SCRIPT [ARGS]
    cloudtik attach CONFIG              cloudtik scale CONFIG --gpus N
    cloudtik upload|download CONFIG SRC DST
    cloudtik status|info|head-ip|worker-ips|monitor|health-check|process-status|
             resource-metrics|debug-status|cluster-dump|kill-node|wait-for-ready CONFIG
    cloudtik workspace|storage|database create|delete|info ...
    cloudtik node start|stop|resources|nodes|dump ...   (run on cluster nodes)
    cloudtik runtime install|configure|services|list ...
    cloudtik head ...                   (run on the head, against its bootstrap config)
"""
from __future__ import annotations

import json
import logging
import os
import sys

import click

from cloudtik_amd.cli.dump_options import dump_options

from cloudtik_amd.core import constants as C


def _setup_logging(level: str):
    logging.basicConfig(level=getattr(logging, level.upper(), logging.INFO), format=C.LOGGER_FORMAT)


def _parse_kv(s):
    if not s:
        return None
    try:
        return json.loads(s)
    except ValueError:
        out = {}
        for part in s.split(","):
            k, v = part.split("=", 1) if "=" in part else part.split(":", 1)
            out[k.strip()] = float(v)
        return out


def _echo_json(obj):
    click.echo(json.dumps(obj, indent=2, default=str, sort_keys=True))


def _load(config_file, cluster_name=None, no_config_cache=False):
    from cloudtik_amd.core.cluster_config import load_cluster_config
    return load_cluster_config(config_file, cluster_name, no_config_cache=no_config_cache)


def _fail(msg: str):
    click.secho(msg, fg="red", err=True)
    sys.exit(1)


@click.group()
@click.option("--logging-level", default="warning", type=click.Choice(C.LOGGER_LEVEL_CHOICES))
@click.version_option(package_name=None, version="1.0.0", prog_name="cloudtik (MI355X)")
def cli(logging_level):
    """CloudTik for AMD Instinct MI355X: workspace / cluster / runtime management."""
    _setup_logging(logging_level)


_cluster_name = click.option("--cluster-name", "-n", default=None, help="Override the configured cluster name.")
_yes = click.option("--yes", "-y", is_flag=True, default=False, help="Don't ask for confirmation.")


# ---------------------------------------------------------------------- lifecycle
@cli.command()
@click.argument("cluster_config_file")
@click.option("--min-workers", type=int, default=None, help="Override min_workers of every worker type.")
@click.option("--max-workers", type=int, default=None, help="Override the global max_workers.")
@click.option("--no-restart", is_flag=True, default=False, help="Skip restarting services on the head.")
@click.option("--restart-only", is_flag=True, default=False, help="Only restart services (skip setup).")
@click.option("--no-config-cache", is_flag=True, default=False)
@_yes
@_cluster_name
def start(cluster_config_file, min_workers, max_workers, no_restart, restart_only, no_config_cache, yes,
          cluster_name):
    """Create or update a cluster."""
    from cloudtik_amd.core.config.loader import load_config_file
    from cloudtik_amd.core import cluster_operator as op
    overrides = {}
    if max_workers is not None:
        overrides["max_workers"] = max_workers
    cfg = load_config_file(cluster_config_file, overrides or None)
    if cluster_name:
        cfg["cluster_name"] = cluster_name
    if min_workers is not None:
        for t, nt in cfg.get("available_node_types", {}).items():
            if t != cfg.get("head_node_type"):
                nt["min_workers"] = min_workers
    from cloudtik_amd.core.cluster_config import bootstrap_config
    cfg.setdefault("cluster_name", "default")
    cfg = bootstrap_config(cfg, no_config_cache)
    try:
        op.create_or_update_cluster(cfg, no_restart=no_restart, restart_only=restart_only)
    except Exception as e:  # noqa: BLE001
        _fail(f"cluster start failed: {e}")
    info = op.get_cluster_info(cfg)
    click.secho(f"Cluster {cfg['cluster_name']} is up: head {info['head_ip']} ({info['head_status']}).", fg="green")
    click.echo(f"  cloudtik status {cluster_config_file}    cloudtik attach {cluster_config_file}")
    for name, ep in info["endpoints"].items():
        click.echo(f"  {name}: {ep.get('url')}")


cli.add_command(start, name="up")


@cli.command()
@click.argument("cluster_config_file")
@click.option("--workers-only", is_flag=True, default=False, help="Only tear down the workers.")
@click.option("--keep-min-workers", is_flag=True, default=False)
@click.option("--hard", is_flag=True, default=False, help="Terminate without running stop commands.")
@click.option("--deep", is_flag=True, default=False, help="Also clean up provider-side cluster state.")
@_yes
@_cluster_name
def stop(cluster_config_file, workers_only, keep_min_workers, hard, deep, yes, cluster_name):
    """Tear down a cluster."""
    from cloudtik_amd.core import cluster_operator as op
    op.teardown_cluster(cluster_config_file, workers_only, keep_min_workers, cluster_name, hard, deep)
    click.secho("Cluster stopped." if not workers_only else "Workers stopped.", fg="green")


cli.add_command(stop, name="down")


@cli.command()
@click.argument("cluster_config_file")
@click.option("--node-ip", default=None)
@_cluster_name
def attach(cluster_config_file, node_ip, cluster_name):
    """Open an interactive shell on the head (or a node)."""
    from cloudtik_amd.core import cluster_operator as op
    sys.exit(op.attach_cluster(cluster_config_file, node_ip, cluster_name))


@cli.command(name="exec", context_settings={"ignore_unknown_options": True})
@click.argument("cluster_config_file")
@click.argument("cmd", nargs=-1, required=True)
@click.option("--node-ip", default=None)
@click.option("--all-nodes", is_flag=True, default=False)
@click.option("--start", is_flag=True, default=False, help="Start the cluster if needed.")
@click.option("--run-env", default="auto", type=click.Choice(["auto", "host", "docker"]))
@_cluster_name
def exec_cmd(cluster_config_file, cmd, node_ip, all_nodes, start, run_env, cluster_name):
    """Execute a shell command on the head (or nodes)."""
    from cloudtik_amd.core import cluster_operator as op
    try:
        op.exec_cluster(cluster_config_file, " ".join(cmd), node_ip, all_nodes, run_env=run_env, start=start,
                        override_cluster_name=cluster_name)
    except Exception as e:  # noqa: BLE001
        _fail(str(e))


@cli.command(context_settings={"ignore_unknown_options": True})
@click.argument("cluster_config_file")
@click.argument("script")
@click.argument("script_args", nargs=-1, type=click.UNPROCESSED)
@click.option("--node-ip", default=None)
@click.option("--job-waiter", default=None)
@click.option("--runtime-options", default=None,
              help="Options for the runtime's runner, e.g. the AI runtime's cloudtik-run: "
                   "\"--nproc-per-node 8 --max-restarts 2\" (reference scripts.py submit).")
@_cluster_name
def submit(cluster_config_file, script, script_args, node_ip, job_waiter, runtime_options, cluster_name):
    """Upload a script to the cluster and run it (python / bash / ...)."""
    import shlex
    from cloudtik_amd.core import cluster_operator as op
    try:
        op.submit_and_exec(cluster_config_file, script, list(script_args), node_ip, job_waiter, cluster_name,
                           runtime_options=shlex.split(runtime_options) if runtime_options else None)
    except Exception as e:  # noqa: BLE001
        _fail(str(e))


@cli.command(context_settings={"ignore_unknown_options": True})
@click.argument("cluster_config_file")
@click.argument("script")
@click.argument("script_args", nargs=-1, type=click.UNPROCESSED)
@click.option("--node-ip", default=None)
@click.option("--job-waiter", default=None, help="Run detached in tmux and wait with this waiter (e.g. yarn).")
@_cluster_name
def run(cluster_config_file, script, script_args, node_ip, job_waiter, cluster_name):
    """Run a built-in script: a registered alias (e.g. ai.launch) or <runtime>/<script>.

    Use exec / submit for your own commands and scripts."""
    from cloudtik_amd.core import cluster_operator as op
    try:
        op.run_script(cluster_config_file, script, list(script_args), node_ip, job_waiter, cluster_name)
    except Exception as e:  # noqa: BLE001
        _fail(str(e))


@cli.command()
@click.argument("cluster_config_file")
@click.option("--cpus", type=int, default=None)
@click.option("--gpus", type=int, default=None)
@click.option("--workers", type=int, default=None)
@click.option("--worker-type", default=None)
@click.option("--resources", default=None, help='JSON or "GPU=8,CPU=64" bundle to request.')
@click.option("--up-only", is_flag=True, default=False)
@_cluster_name
def scale(cluster_config_file, cpus, gpus, workers, worker_type, resources, up_only, cluster_name):
    """Request the cluster to scale to a resource level."""
    from cloudtik_amd.core import cluster_operator as op
    req = op.scale_cluster(cluster_config_file, cpus, gpus, workers, worker_type, _parse_kv(resources), up_only,
                           cluster_name)
    click.echo(f"scale request: {len(req['bundles'])} bundle(s)")


@cli.command()
@click.argument("cluster_config_file")
@click.argument("source")
@click.argument("target")
@click.option("--node-ip", default=None)
@click.option("--all-workers", is_flag=True, default=False)
@_cluster_name
def upload(cluster_config_file, source, target, node_ip, all_workers, cluster_name):
    """Upload files to the cluster."""
    from cloudtik_amd.core import cluster_operator as op
    op.rsync(cluster_config_file, source, target, False, node_ip, all_workers, cluster_name)


@cli.command()
@click.argument("cluster_config_file")
@click.argument("source")
@click.argument("target")
@click.option("--node-ip", default=None)
@_cluster_name
def download(cluster_config_file, source, target, node_ip, cluster_name):
    """Download files from the cluster."""
    from cloudtik_amd.core import cluster_operator as op
    op.rsync(cluster_config_file, source, target, True, node_ip, False, cluster_name)


for _n, _c in (("rsync-up", upload), ("rsync_up", upload), ("rsync-down", download), ("rsync_down", download)):
    cli.add_command(_c, name=_n)


# ---------------------------------------------------------------------- info
@cli.command()
@click.argument("cluster_config_file")
@_cluster_name
def status(cluster_config_file, cluster_name):
    """Show the nodes of a cluster and their status."""
    from tabulate import tabulate
    from cloudtik_amd.core import cluster_operator as op
    cfg = _load(cluster_config_file, cluster_name)
    nodes = op.get_cluster_nodes_info(cfg)
    rows = [[n["node_id"], n["node_ip"], n["node_kind"], n["node_type"], n["node_status"], n.get("instance_type")]
            for n in nodes]
    click.echo(tabulate(rows, headers=["node id", "ip", "kind", "node type", "status", "instance type"]))
    st = op.get_scaling_status(cfg)
    if st:
        click.echo(f"\nlaunching: {st['launching'] or '-'}   updating: {st['updating'] or '-'}   "
                   f"demands: {len(st['resource_demands'])}   requests: {len(st['cluster_requests'])}")
        if st.get("failed_launches"):
            click.echo(f"failed launches: {st['failed_launches']}")


@cli.command()
@click.argument("cluster_config_file")
@click.option("--json", "as_json", is_flag=True, default=False)
@_cluster_name
def info(cluster_config_file, as_json, cluster_name):
    """Show cluster summary: resources, runtimes, endpoints."""
    from cloudtik_amd.core import cluster_operator as op
    cfg = _load(cluster_config_file, cluster_name)
    i = op.get_cluster_info(cfg)
    if as_json:
        _echo_json(i)
        return
    click.echo(f"Cluster {i['cluster_name']}: {i['status']}")
    click.echo(f"  head: {i['head_ip']} ({i['head_status']})")
    click.echo(f"  workers: {i['total_workers_ready']}/{i['total_workers']} ready {i['workers_by_status']}")
    click.echo(f"  resources: {i['resources']}")
    click.echo(f"  runtimes: {', '.join(i['runtimes'])}")
    for name, ep in i["endpoints"].items():
        click.echo(f"  {name}: {ep.get('url')}")


@cli.command(name="head-ip")
@click.argument("cluster_config_file")
@_cluster_name
def head_ip(cluster_config_file, cluster_name):
    """Print the head node IP."""
    from cloudtik_amd.core import cluster_operator as op
    click.echo(op.get_head_node_ip(_load(cluster_config_file, cluster_name)))


@cli.command(name="worker-ips")
@click.argument("cluster_config_file")
@click.option("--node-status", default=None)
@_cluster_name
def worker_ips(cluster_config_file, node_status, cluster_name):
    """Print the worker node IPs."""
    from cloudtik_amd.core import cluster_operator as op
    for ip in op.get_worker_node_ips(_load(cluster_config_file, cluster_name), node_status=node_status):
        click.echo(ip)


cli.add_command(head_ip, name="head-host")
cli.add_command(worker_ips, name="worker-hosts")
cli.add_command(head_ip, name="head_ip")
cli.add_command(worker_ips, name="worker_ips")


@cli.command()
@click.argument("cluster_config_file")
@click.option("--lines", type=int, default=100)
@click.option("--follow", "-f", is_flag=True, default=False)
@_cluster_name
def monitor(cluster_config_file, lines, follow, cluster_name):
    """Tail the cluster controller log (and follow every node's logs)."""
    from cloudtik_amd.core import cluster_operator as op
    op.monitor_cluster(cluster_config_file, lines, follow, override_cluster_name=cluster_name)


cli.add_command(monitor, name="logs")


@cli.command(name="kill-node")
@click.argument("cluster_config_file")
@click.option("--node-ip", default=None)
@click.option("--hard", is_flag=True, default=False)
@_yes
@_cluster_name
def kill_node(cluster_config_file, node_ip, hard, yes, cluster_name):
    """Kill a worker node (a random one without --node-ip)."""
    from cloudtik_amd.core import cluster_operator as op
    ip = op.kill_node(cluster_config_file, node_ip, hard, cluster_name)
    click.echo(f"killed {ip}" if ip else "no worker to kill")


@cli.command(name="wait-for-ready")
@click.argument("cluster_config_file")
@click.option("--min-workers", type=int, default=None)
@click.option("--timeout", type=int, default=C.CLOUDTIK_WAIT_FOR_CLUSTER_READY_TIMEOUT_S)
@_cluster_name
def wait_for_ready(cluster_config_file, min_workers, timeout, cluster_name):
    """Wait until the given number of workers are ready."""
    from cloudtik_amd.core import cluster_operator as op
    try:
        n = op.wait_for_ready(cluster_config_file, min_workers, timeout, override_cluster_name=cluster_name)
    except TimeoutError as e:
        _fail(str(e))
    click.echo(f"{n} worker(s) ready")


@cli.command(name="process-status")
@click.argument("cluster_config_file")
@_cluster_name
def process_status(cluster_config_file, cluster_name):
    """Show the CloudTik daemons of every node."""
    from tabulate import tabulate
    from cloudtik_amd.core import cluster_operator as op
    rows = []
    for nid, v in sorted(op.cluster_process_status(_load(cluster_config_file, cluster_name)).items()):
        for name, st in sorted(v.get("processes", {}).items()):
            rows.append([v.get("node_ip"), name, st.get("pid"), "running" if st.get("alive") else "DEAD"])
    click.echo(tabulate(rows, headers=["node", "process", "pid", "state"]))


@cli.command(name="resource-metrics")
@click.argument("cluster_config_file")
@_cluster_name
def resource_metrics(cluster_config_file, cluster_name):
    """Show CPU / memory / GPU load of every node."""
    from tabulate import tabulate
    from cloudtik_amd.core import cluster_operator as op
    rows = []
    for nid, m in sorted(op.cluster_resource_metrics(_load(cluster_config_file, cluster_name)).items()):
        gpus = m.get("gpus") or []
        vram = sum(g.get("vram_used") or 0 for g in gpus) / 2**30
        rows.append([m.get("node_ip"), f"{m.get('cpu_percent', 0):.0f}%",
                     f"{(m.get('memory_used', 0)) / 2**30:.1f}/{m.get('memory_total', 0) / 2**30:.1f} GiB",
                     len(gpus), f"{m.get('gpu_busy_percent_avg') or 0:.0f}%", f"{vram:.1f} GiB"])
    click.echo(tabulate(rows, headers=["node", "cpu", "memory", "gpus", "gpu busy", "vram used"]))


@cli.command(name="debug-status")
@click.argument("cluster_config_file")
@_cluster_name
def debug_status(cluster_config_file, cluster_name):
    """Show the scaler's status: launches, updates, demands, recent events."""
    from cloudtik_amd.core import cluster_operator as op
    _echo_json(op.get_scaling_status(_load(cluster_config_file, cluster_name)) or {})


@cli.command(name="health-check")
@click.argument("cluster_config_file")
@click.option("--with-details", is_flag=True, default=False)
@_cluster_name
def health_check(cluster_config_file, with_details, cluster_name):
    """Check that daemons run and nodes heart-beat."""
    from cloudtik_amd.core import cluster_operator as op
    r = op.health_check(_load(cluster_config_file, cluster_name), with_details)
    if with_details:
        _echo_json(r)
    if r["healthy"]:
        click.secho("Cluster is healthy.", fg="green")
    else:
        for p in r["problems"]:
            click.secho(p, fg="red")
        sys.exit(1)


@cli.command(name="cluster-dump")
@click.argument("cluster_config_file")
@click.option("--output", "-o", default=None)
@click.option("--hosts", default=None, help="Only these nodes (IPs or node ids, comma separated).")
@click.option("--head-only", is_flag=True, default=False)
@_cluster_name
@dump_options
def cluster_dump(cluster_config_file, output, hosts, head_only, cluster_name, params):
    """Collect logs, debug state, packages, processes and GPU state of the cluster's nodes."""
    from cloudtik_amd.core import cluster_operator as op
    click.echo(op.cluster_dump(cluster_config_file, output, override_cluster_name=cluster_name, hosts=hosts,
                               head_only=head_only, params=params))


cli.add_command(cluster_dump, name="cluster_dump")


@cli.command(name="start-proxy")
@click.argument("cluster_config_file")
@click.option("--port", type=int, default=C.DEFAULT_PROXY_PORT)
@_cluster_name
def start_proxy(cluster_config_file, port, cluster_name):
    """Start a SOCKS proxy to the cluster network (SSH dynamic forwarding to the head)."""
    from cloudtik_amd.core import proxy
    click.echo(proxy.start_proxy(_load(cluster_config_file, cluster_name), port))


@cli.command(name="stop-proxy")
@click.argument("cluster_config_file")
@_cluster_name
def stop_proxy(cluster_config_file, cluster_name):
    """Stop the SOCKS proxy of the cluster."""
    from cloudtik_amd.core import proxy
    click.echo(proxy.stop_proxy(_load(cluster_config_file, cluster_name)))


def _register_groups():
    from cloudtik_amd.cli.node import node
    from cloudtik_amd.cli.runtime import runtime
    from cloudtik_amd.cli.workspace import workspace, storage, database
    from cloudtik_amd.cli.head import head
    for g in (node, runtime, workspace, storage, database, head):
        cli.add_command(g)
    _register_runtime_groups()


def _register_runtime_groups():
    """Runtime packages contribute command groups: ``cloudtik_amd.runtime.<name>.cli`` exposing
    a click group called ``<name>`` becomes ``cloudtik <name> ...`` (reference scripts.py:66)."""
    import importlib
    import pkgutil
    import cloudtik_amd.runtime as rt_pkg
    for info in pkgutil.iter_modules(rt_pkg.__path__):
        if not info.ispkg:
            continue
        try:
            mod = importlib.import_module(f"{rt_pkg.__name__}.{info.name}.cli")
        except ImportError:
            continue
        grp = getattr(mod, info.name, None)
        if isinstance(grp, click.Group) and info.name not in cli.commands:
            cli.add_command(grp)


_register_groups()


def main(argv=None):
    return cli.main(args=argv, prog_name="cloudtik")


if __name__ == "__main__":
    main()
