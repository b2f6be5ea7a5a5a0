"""Library fixes for the cloud storage / tracking stack the AI runtime uses (reference
runtime/ai/conf/patches/*.patch, copied over the installed files by
runtime/ai/scripts/configure.sh:127-234).

Instead of overwriting files inside site-packages, the fixes are applied in-process, and
only in processes that ask for them: ``install()`` (called when ``cloudtik_amd.runtime.ai``
is imported -- the AI runtime API, the data API and the estimators all live there) registers
a meta-path finder that runs a fix right after its target module executes, and fixes the
targets that are already imported.  Fixes:

* Azure managed identity: when ``~/azure_managed_identity.config`` holds a client id,
  ``azure.identity.DefaultAzureCredential`` (sync and aio) uses it unless the caller passed
  one -- this is what adlfs (``abfs://``) and MLflow's Azure Blob / ADLS Gen2 artifact
  repositories construct;
* MLflow: ``abfss://`` artifact URIs go to the ADLS Gen2 repository;
* adlfs: ``put`` of a local directory creates the remote directory instead of failing;
* gcsfs: a listing of ``dir`` no longer contains a file entry named ``dir`` itself.
"""
from __future__ import annotations

import functools
import importlib.abc
import os
import sys
from typing import Callable, Dict, Optional

MANAGED_IDENTITY_CONFIG = "~/azure_managed_identity.config"


def managed_identity_client_id(path: str = MANAGED_IDENTITY_CONFIG) -> Optional[str]:
    p = os.path.expanduser(path)
    if not os.path.isfile(p):
        return None
    with open(p) as f:
        cid = f.readline().strip()
    return cid or None


# ----------------------------------------------------------------------------- fixes
def _wrap_credential_class(cls):
    if getattr(cls, "_cloudtik_mi", False):
        return cls
    orig = cls.__init__

    @functools.wraps(orig)
    def __init__(self, *a, **kw):
        cid = managed_identity_client_id()
        if cid and "managed_identity_client_id" not in kw:
            kw["managed_identity_client_id"] = cid
        orig(self, *a, **kw)

    cls.__init__ = __init__
    cls._cloudtik_mi = True
    return cls


def fix_azure_identity(mod) -> None:
    if hasattr(mod, "DefaultAzureCredential"):
        _wrap_credential_class(mod.DefaultAzureCredential)


def fix_mlflow_registry(mod) -> None:
    reg = getattr(mod, "_artifact_repository_registry", None)
    if reg is None or "abfss" in getattr(reg, "_registry", {}):
        return
    try:
        from mlflow.store.artifact.azure_data_lake_artifact_repo import AzureDataLakeArtifactRepository
    except ImportError:
        return
    reg.register("abfss", AzureDataLakeArtifactRepository)


def fix_adlfs_spec(mod) -> None:
    fs = getattr(mod, "AzureBlobFileSystem", None)
    if fs is None or getattr(fs, "_cloudtik_put", False) or not hasattr(fs, "_put_file"):
        return
    orig = fs._put_file

    @functools.wraps(orig)
    async def _put_file(self, lpath, rpath, *a, **kw):
        if os.path.isdir(lpath):
            return await self._mkdir(rpath, exist_ok=True)
        return await orig(self, lpath, rpath, *a, **kw)

    fs._put_file = _put_file
    fs._cloudtik_put = True


def fix_gcsfs_core(mod) -> None:
    fs = getattr(mod, "GCSFileSystem", None)
    if fs is None or getattr(fs, "_cloudtik_ls", False) or not hasattr(fs, "_list_objects"):
        return
    orig = fs._list_objects

    @functools.wraps(orig)
    async def _list_objects(self, path, *a, **kw):
        out = await orig(self, path, *a, **kw)
        p = path.rstrip("/")
        if isinstance(out, list) and len(out) > 1:
            # a "directory" listing must not contain a file entry named like the directory
            out = [o for o in out if not (isinstance(o, dict) and o.get("type") == "file"
                                          and o.get("name", "").rstrip("/") == p)]
        return out

    fs._list_objects = _list_objects
    fs._cloudtik_ls = True


FIXES: Dict[str, Callable] = {
    "azure.identity": fix_azure_identity,
    "azure.identity.aio": fix_azure_identity,
    "mlflow.store.artifact.artifact_repository_registry": fix_mlflow_registry,
    "adlfs.spec": fix_adlfs_spec,
    "gcsfs.core": fix_gcsfs_core,
}


# ----------------------------------------------------------------------------- import hook
class _FixingLoader(importlib.abc.Loader):
    def __init__(self, inner, fix):
        self.inner, self.fix = inner, fix

    def create_module(self, spec):
        return self.inner.create_module(spec) if hasattr(self.inner, "create_module") else None

    def exec_module(self, module):
        self.inner.exec_module(module)
        try:
            self.fix(module)
        except Exception as e:                    # a fix must never break the import
            print(f"[cloudtik] fix for {module.__name__} skipped: {e}", file=sys.stderr)


class _FixFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path=None, target=None):
        fix = FIXES.get(name)
        if fix is None:
            return None
        for finder in sys.meta_path:
            if finder is self or not hasattr(finder, "find_spec"):
                continue
            spec = finder.find_spec(name, path, target)
            if spec is not None:
                if spec.loader is not None:
                    spec.loader = _FixingLoader(spec.loader, fix)
                return spec
        return None


def install() -> None:
    """Install the in-process import hook (idempotent) and fix already-imported targets."""
    if not any(isinstance(f, _FixFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _FixFinder())
    for name, fix in FIXES.items():
        mod = sys.modules.get(name)
        if mod is not None:
            fix(mod)


def uninstall() -> None:
    sys.meta_path[:] = [f for f in sys.meta_path if not isinstance(f, _FixFinder)]
