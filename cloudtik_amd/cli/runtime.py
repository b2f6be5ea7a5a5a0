"""``cloudtik runtime ...`` (reference scripts/runtime_scripts.py:116-343): run a runtime's
install / configure / services steps on this node, or list the available runtimes."""
from __future__ import annotations

import os

import click
import yaml

DEFAULT_BOOTSTRAP_CONFIG = "~/cloudtik_bootstrap_config.yaml"


def _runtime(name: str):
    from cloudtik_amd.core import runtime_factory as rf
    cfg_path = os.path.expanduser(DEFAULT_BOOTSTRAP_CONFIG)
    rc = {}
    if os.path.exists(cfg_path):
        with open(cfg_path) as f:
            rc = ((yaml.safe_load(f) or {}).get("runtime", {}) or {}).get(name, {}) or {}
    return rf.get_runtime(name, rc)


@click.group()
def runtime():
    """Runtime operations on this node."""


@runtime.command()
@click.argument("name")
@click.option("--head", is_flag=True, default=False)
def install(name, head):
    """Install the runtime on this node."""
    _runtime(name).node_install(head)


@runtime.command()
@click.argument("name")
@click.option("--head", is_flag=True, default=False)
def configure(name, head):
    """Configure the runtime on this node."""
    _runtime(name).node_configure(head)


@runtime.command()
@click.argument("name")
@click.argument("command", type=click.Choice(["start", "stop"]))
@click.option("--head", is_flag=True, default=False)
def services(name, command, head):
    """Start or stop the runtime's services on this node."""
    _runtime(name).node_services(command, head)


@runtime.command(name="list")
def list_runtimes():
    """List the available runtimes."""
    from cloudtik_amd.core import runtime_factory as rf
    for n in rf.list_runtimes():
        cls = rf.get_runtime_cls(n)
        doc = (cls.__doc__ or "").strip().split("\n")[0]
        click.echo(f"{n:16s} {doc}")
