"""``cloudtik workspace|storage|database ...`` (reference scripts/workspace.py, storage.py,
database.py)."""
from __future__ import annotations

import json

import click
import yaml


def _load(path):
    from cloudtik_amd.core.config.loader import load_config_file
    return load_config_file(path)


@click.group()
def workspace():
    """Workspace operations (network / storage / identity shared by clusters)."""


@workspace.command()
@click.argument("workspace_config_file")
@click.option("--yes", "-y", is_flag=True, default=False)
def create(workspace_config_file, yes):
    """Create a workspace."""
    from cloudtik_amd.core import workspace as ws
    cfg = ws.create_workspace(_load(workspace_config_file))
    click.secho(f"workspace {cfg['workspace_name']} created", fg="green")


@workspace.command()
@click.argument("workspace_config_file")
@click.option("--delete-managed-storage", is_flag=True, default=False)
@click.option("--delete-managed-database", is_flag=True, default=False)
@click.option("--yes", "-y", is_flag=True, default=False)
def delete(workspace_config_file, delete_managed_storage, delete_managed_database, yes):
    """Delete a workspace."""
    from cloudtik_amd.core import workspace as ws
    try:
        ws.delete_workspace(_load(workspace_config_file), delete_managed_storage, delete_managed_database,
                            confirm=None if yes else (lambda q: click.confirm(q, default=False)))
    except (ws.WorkspaceInUse, RuntimeError) as e:
        raise click.ClickException(str(e))
    click.echo("workspace deleted")


@workspace.command()
@click.argument("workspace_config_file")
def update(workspace_config_file):
    """Update a workspace."""
    from cloudtik_amd.core import workspace as ws
    ws.update_workspace(_load(workspace_config_file))


@workspace.command()
@click.argument("workspace_config_file")
def info(workspace_config_file):
    """Show workspace status and clusters."""
    from cloudtik_amd.core import workspace as ws
    cfg = _load(workspace_config_file)
    click.echo(f"status: {ws.workspace_status(cfg).name}")
    click.echo(json.dumps(ws.workspace_info(cfg), indent=2, default=str))


@workspace.command(name="list-clusters")
@click.argument("workspace_config_file")
def list_clusters(workspace_config_file):
    """List the clusters of a workspace."""
    from cloudtik_amd.core import workspace as ws
    for name in sorted(ws.list_workspace_clusters(_load(workspace_config_file)) or {}):
        click.echo(name)


def _storage_group(kind: str):
    @click.group(name=kind)
    def group():
        pass
    group.help = f"Managed {kind} operations (cloud providers)."

    def provider(cfg, name):
        from cloudtik_amd.core import provider_factory as pf
        get = pf.get_storage_provider if kind == "storage" else pf.get_database_provider
        return get(cfg["provider"], cfg.get("workspace_name", "default"), name)

    @group.command()
    @click.argument("config_file")
    @click.option("--name", default=None)
    def create(config_file, name):
        cfg = _load(config_file)
        provider(cfg, name or cfg.get(f"{kind}_name", "default")).create(cfg)

    @group.command()
    @click.argument("config_file")
    @click.option("--name", default=None)
    def delete(config_file, name):
        cfg = _load(config_file)
        provider(cfg, name or cfg.get(f"{kind}_name", "default")).delete(cfg)

    @group.command()
    @click.argument("config_file")
    @click.option("--name", default=None)
    def info(config_file, name):
        cfg = _load(config_file)
        click.echo(yaml.safe_dump(provider(cfg, name or cfg.get(f"{kind}_name", "default")).get_info(cfg)))

    return group


storage = _storage_group("storage")
database = _storage_group("database")
