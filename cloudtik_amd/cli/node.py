"""``cloudtik node ...``: commands run ON a cluster node by the merged start/stop commands
(reference scripts/node_scripts.py:48-768: start / stop / resources / nodes / service /
wait-for-port / dump)."""
from __future__ import annotations

import json
import os
import socket
import sys
import time

import click

from cloudtik_amd.cli.dump_options import dump_options

from cloudtik_amd.core import constants as C

DEFAULT_BOOTSTRAP_CONFIG = "~/cloudtik_bootstrap_config.yaml"


def _node_ip(ip):
    if ip:
        return ip
    from cloudtik_amd.core.executor import local_ips
    ips = [i for i in local_ips() if i.count(".") == 3 and not i.startswith("127.")]
    return ips[0] if ips else "127.0.0.1"


def _password():
    return os.environ.get("CLOUDTIK_STATE_PASSWORD") or C.CLOUDTIK_STATE_PASSWORD


@click.group()
def node():
    """Commands run on a cluster node."""


@node.command()
@click.option("--head", is_flag=True, default=False)
@click.option("--node-ip", default=None)
@click.option("--port", type=int, default=C.CLOUDTIK_DEFAULT_PORT, help="State service port (head).")
@click.option("--address", default=None, help="Head state service address (workers).")
@click.option("--state", is_flag=True, default=False, help="Head: start the state service + node agent.")
@click.option("--controller", is_flag=True, default=False, help="Head: start the cluster controller.")
@click.option("--resources", default=None, help="JSON resources override of this node.")
@click.option("--config", "config_file", default=DEFAULT_BOOTSTRAP_CONFIG)
def start(head, node_ip, port, address, state, controller, resources, config_file):
    """Start the CloudTik daemons of this node."""
    from cloudtik_amd.core import services
    node_ip = _node_ip(node_ip)
    pw = _password()
    if head:
        addr = f"{node_ip}:{port}"
        if state or not controller:
            services.start_state_server(node_ip, port, pw)
            services.start_node_monitor(addr, node_ip, True, pw, resources)
            click.echo(f"state service on {addr}")
        if controller or not state:
            cfg = os.path.expanduser(config_file)
            if not os.path.exists(cfg):
                click.secho(f"no bootstrap config at {cfg}; controller not started", fg="yellow")
            else:
                services.start_cluster_controller(addr, cfg, pw)
                click.echo("cluster controller started")
    else:
        if not address:
            raise click.UsageError("workers need --address=HEAD_IP:PORT")
        services.start_node_monitor(address, node_ip, False, pw, resources)
        click.echo(f"node agent reporting to {address}")


@node.command()
@click.option("--controller-only", is_flag=True, default=False)
def stop(controller_only):
    """Stop the CloudTik daemons this node started."""
    from cloudtik_amd.core import services
    if controller_only:
        services.stop_process(C.PROCESS_TYPE_CLUSTER_CONTROLLER)
        return
    stopped = services.stop_all()
    click.echo(f"stopped: {', '.join(stopped) or 'nothing'}")


@node.command()
@click.option("--json", "as_json", is_flag=True, default=True)
def resources(as_json):
    """Print the detected resources of this node (CPU, memory, AMD GPUs)."""
    from cloudtik_amd.core.resources import detect_resources
    click.echo(json.dumps(detect_resources(), indent=2))


@node.command()
@click.option("--address", default=None)
def nodes(address):
    """List the nodes registered in the state service."""
    from cloudtik_amd.core.state.state_client import NODE_TABLE, StateClient
    addr = address or os.environ.get(C.CLOUDTIK_ADDRESS_ENV) or f"127.0.0.1:{C.CLOUDTIK_DEFAULT_PORT}"
    c = StateClient.create(addr, _password())
    now = time.time()
    for nid, n in sorted(c.table_get_all(NODE_TABLE).items()):
        click.echo(f"{nid}\t{n.get('node_ip')}\t{n.get('node_kind')}\t"
                   f"heartbeat {now - n.get('last_heartbeat_time', 0):.1f}s ago\t{n.get('resources')}")


@node.command(name="process-status")
def process_status():
    """Show this node's CloudTik daemons."""
    from cloudtik_amd.core import services
    for name, info in services.list_processes().items():
        click.echo(f"{name}\t{info['pid']}\t{'running' if info['alive'] else 'DEAD'}")


@node.command(name="wait-for-port")
@click.argument("port", type=int)
@click.option("--host", default="127.0.0.1")
@click.option("--timeout", type=int, default=60)
@click.option("--free", is_flag=True, default=False, help="Wait for the port to become free instead.")
def wait_for_port(port, host, timeout, free):
    """Wait until a TCP port is listening (or free)."""
    end = time.time() + timeout
    while time.time() < end:
        try:
            with socket.create_connection((host, port), timeout=1):
                if not free:
                    return
        except OSError:
            if free:
                return
        time.sleep(0.5)
    sys.exit(1)


@node.command()
@click.option("--output", "-o", default=None)
@click.option("--silent", is_flag=True, default=False)
@dump_options
def dump(output, silent, params):
    """Archive this node's logs, debug state, pip packages, processes and GPU state."""
    from cloudtik_amd.core.cluster_dump import collect_local
    out = collect_local(params, output or f"cloudtik-node-dump-{time.strftime('%Y%m%d-%H%M%S')}.tar.gz")
    if not silent:
        click.echo(out)


@node.command(name="service-daemon")
@click.argument("command", type=click.Choice(["start", "stop"]))
@click.argument("identifier")
@click.option("--service-class", default=None, help="ServiceRunner / PullJob class (module.Class).")
@click.option("--pull-script", default=None, help="Script run every --interval seconds.")
@click.option("--interval", type=float, default=None)
@click.argument("service_args", nargs=-1)
def service_daemon(command, identifier, service_class, pull_script, interval, service_args):
    """Start / stop a generic service daemon or periodic pull job on this node."""
    from cloudtik_amd.core.service_daemon import start_service_daemon, stop_service_daemon
    if command == "start":
        pid = start_service_daemon(identifier, service_class, pull_script, interval, list(service_args))
        click.echo(f"service daemon {identifier} started (pid {pid})")
    else:
        ok = stop_service_daemon(identifier)
        click.echo(f"service daemon {identifier} {'stopped' if ok else 'was not running'}")
