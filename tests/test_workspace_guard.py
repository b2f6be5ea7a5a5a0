"""Workspace deletion guard (core/workspace.py; reference workspace_operator.py:58-112): a
workspace whose clusters still run is not deleted, the confirmation is asked last, and a
workspace that does not exist is an error."""
import pytest

from cloudtik_amd.core import tags as T


def test_delete_refuses_running_clusters_then_confirms(tmp_path, monkeypatch):
    from cloudtik_amd.core import workspace as ws
    from cloudtik_amd.core.provider_factory import get_node_provider
    from cloudtik_amd.providers.local import workspace_provider as lwp
    from cloudtik_amd.providers.mock.node_provider import MockProvider
    monkeypatch.setattr(lwp, "STATE_DIR", str(tmp_path))
    MockProvider.reset()
    cfg = {"workspace_name": "w", "provider": {"type": "mock"}}
    with pytest.raises(RuntimeError, match="does not exist"):
        ws.delete_workspace(cfg)
    ws.create_workspace(cfg)
    p = get_node_provider({"type": "mock"}, "c1", use_cache=False)
    (head,) = p.create_node({}, {T.CLOUDTIK_TAG_CLUSTER_NAME: "c1", T.CLOUDTIK_TAG_NODE_KIND: "head",
                                 T.CLOUDTIK_TAG_WORKSPACE_NAME: "w"}, 1)
    asked = []
    with pytest.raises(ws.WorkspaceInUse, match="c1"):
        ws.delete_workspace(cfg, confirm=lambda q: asked.append(q) or True)
    assert asked == []                                    # refused before asking
    p.terminate_node(head)
    with pytest.raises(RuntimeError, match="aborted"):
        ws.delete_workspace(cfg, confirm=lambda q: False)
    assert ws.workspace_status(cfg) == ws.Existence.COMPLETED
    ws.delete_workspace(cfg, confirm=lambda q: True)
    assert ws.workspace_status(cfg) == ws.Existence.NOT_EXIST
    MockProvider.reset()
