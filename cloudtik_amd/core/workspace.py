"""Workspace lifecycle (reference core/_private/workspace/workspace_operator.py)."""
from __future__ import annotations

import enum
import logging
from typing import Any, Dict

from cloudtik_amd.core.config import loader, schema as jschema
from cloudtik_amd.core.provider_factory import get_workspace_provider

logger = logging.getLogger(__name__)


class Existence(enum.Enum):
    NOT_EXIST = 0
    STORAGE_ONLY = 1
    DATABASE_ONLY = 2
    IN_COMPLETED = 3
    COMPLETED = 4


def prepare_workspace_config(config: Dict[str, Any]) -> Dict[str, Any]:
    cfg = loader.fill_with_defaults(config, object_name="workspace")
    from cloudtik_amd.core.cluster_config import load_schema
    jschema.validate(cfg, load_schema("workspace"))
    return cfg


def create_workspace(config: Dict[str, Any]):
    cfg = prepare_workspace_config(config)
    p = get_workspace_provider(cfg["provider"], cfg["workspace_name"])
    p.create_workspace(cfg)
    return cfg


class WorkspaceInUse(RuntimeError):
    pass


def delete_workspace(config: Dict[str, Any], delete_managed_storage=False, delete_managed_database=False,
                     confirm=None):
    """Delete the workspace, refusing while it still serves something (reference
    workspace_operator.py:58-112): a complete workspace with running clusters, or managed
    databases that are not being deleted with it.  ``confirm(question) -> bool`` is asked
    last (the CLI prompts unless --yes); a refusal aborts."""
    cfg = prepare_workspace_config(config)
    name = cfg["workspace_name"]
    p = get_workspace_provider(cfg["provider"], name)
    existence = p.check_workspace_existence(cfg)
    if existence == Existence.NOT_EXIST:
        raise RuntimeError(f"workspace {name} does not exist")
    if existence == Existence.COMPLETED:
        running = p.list_clusters(cfg) or {}
        if running:
            raise WorkspaceInUse(f"workspace {name} has running clusters ({', '.join(sorted(running))}): "
                                 f"stop them first")
    if cfg.get("managed_cloud_storage"):
        logger.warning("the managed cloud storage of workspace %s %s", name,
                       "and ALL its data will be deleted" if delete_managed_storage else "is kept")
    if cfg.get("managed_cloud_database") and not delete_managed_database:
        try:
            dbs = p.list_databases(cfg) or {}
        except NotImplementedError:
            dbs = {}
        if dbs:
            raise WorkspaceInUse(f"workspace {name} has managed databases ({', '.join(sorted(dbs))}): delete them "
                                 f"first or pass --delete-managed-database")
    if confirm is not None and not confirm(f"Delete workspace {name}?"):
        raise RuntimeError("aborted")
    p.delete_workspace(cfg, delete_managed_storage, delete_managed_database)


def update_workspace(config: Dict[str, Any]):
    cfg = prepare_workspace_config(config)
    get_workspace_provider(cfg["provider"], cfg["workspace_name"]).update_workspace(cfg)


def workspace_status(config: Dict[str, Any]) -> Existence:
    cfg = prepare_workspace_config(config)
    return get_workspace_provider(cfg["provider"], cfg["workspace_name"]).check_workspace_existence(cfg)


def workspace_info(config: Dict[str, Any]) -> Dict[str, Any]:
    cfg = prepare_workspace_config(config)
    return get_workspace_provider(cfg["provider"], cfg["workspace_name"]).get_workspace_info(cfg)


def list_workspace_clusters(config: Dict[str, Any]):
    cfg = prepare_workspace_config(config)
    return get_workspace_provider(cfg["provider"], cfg["workspace_name"]).list_clusters(cfg)
