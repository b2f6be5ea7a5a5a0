"""AI runtime package.  ``_script_aliases_`` names the runnable entry points that
``cloudtik submit <cluster.yaml> <alias> ...`` resolves through the script registry
(reference runtime/ai/__init__.py:5-15).  Targets are module names, run as
``python -m <module>`` on the node, so nothing here is imported eagerly.
"""
_script_aliases_ = {
    "ai.launch": "cloudtik_amd.runner.launch",
    "ai.modeling.graph_sage": "cloudtik_amd.modeling.graph_sage.run",
    "ai.modeling.xgboost": "cloudtik_amd.modeling.gbdt.run",
    "ai.modeling.gbdt": "cloudtik_amd.modeling.gbdt.run",
    "ai.modeling.transfer_learning": "cloudtik_amd.modeling.transfer_learning.run",
}

# in-process fixes for the cloud-storage / tracking libraries the AI runtime drives
# (reference runtime/ai/conf/patches; see patches.py): applied when they get imported
from cloudtik_amd.runtime.ai import patches as _patches  # noqa: E402

_patches.install()
