"""In-process library fixes of the AI runtime (runtime/ai/patches.py; reference
runtime/ai/conf/patches/*.patch) against stand-in modules of azure.identity, mlflow's artifact
registry, adlfs and gcsfs (the real packages are not installed here): each fix applies at
import time, only after cloudtik_amd.runtime.ai is imported, and twice-installing is harmless."""
import os
import subprocess
import sys
import textwrap

FAKES = {
    "azure/__init__.py": "",
    "azure/identity/__init__.py": """
        class DefaultAzureCredential:
            def __init__(self, **kw):
                self.kw = kw
    """,
    "azure/identity/aio/__init__.py": """
        class DefaultAzureCredential:
            def __init__(self, **kw):
                self.kw = kw
    """,
    "gcsfs/__init__.py": "",
    "gcsfs/core.py": """
        class GCSFileSystem:
            async def _list_objects(self, path, prefix=""):
                return [{"name": "b/dir", "type": "file"}, {"name": "b/dir/x", "type": "file"},
                        {"name": "b/dir/sub", "type": "directory"}]
    """,
    "adlfs/__init__.py": "",
    "adlfs/spec.py": """
        class AzureBlobFileSystem:
            def __init__(self):
                self.calls = []
            async def _mkdir(self, path, exist_ok=False):
                self.calls.append(("mkdir", path))
            async def _put_file(self, lpath, rpath, **kw):
                self.calls.append(("put", lpath, rpath))
    """,
    "mlflow/__init__.py": "",
    "mlflow/store/__init__.py": "",
    "mlflow/store/artifact/__init__.py": "",
    "mlflow/store/artifact/azure_data_lake_artifact_repo.py": """
        class AzureDataLakeArtifactRepository:
            pass
    """,
    "mlflow/store/artifact/artifact_repository_registry.py": """
        class ArtifactRepositoryRegistry:
            def __init__(self):
                self._registry = {}
            def register(self, scheme, repo):
                self._registry[scheme] = repo
        _artifact_repository_registry = ArtifactRepositoryRegistry()
    """,
}

PROBE = """
import asyncio, json, os, sys
import azure.identity                               # imported BEFORE the fixes: fixed by install()
import cloudtik_amd.runtime.ai                      # installs the hooks
from cloudtik_amd.runtime.ai import patches
patches.install()                                   # idempotent
from azure.identity import DefaultAzureCredential
from azure.identity.aio import DefaultAzureCredential as AioCred
import gcsfs.core, adlfs.spec
import mlflow.store.artifact.artifact_repository_registry as reg
out = {}
out["sync"] = DefaultAzureCredential().kw
out["aio"] = AioCred().kw
out["explicit"] = DefaultAzureCredential(managed_identity_client_id="mine").kw
out["ls"] = [o["name"] for o in asyncio.run(gcsfs.core.GCSFileSystem()._list_objects("b/dir/"))]
fs = adlfs.spec.AzureBlobFileSystem()
asyncio.run(fs._put_file(sys.argv[1], "c/d"))
asyncio.run(fs._put_file(__file__, "c/f"))
out["adlfs"] = fs.calls
out["abfss"] = reg._artifact_repository_registry._registry["abfss"].__name__
print(json.dumps(out))
"""


def test_ai_runtime_library_fixes(tmp_path):
    root = tmp_path / "fake"
    for rel, src in FAKES.items():
        p = root / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(textwrap.dedent(src))
    home = tmp_path / "home"
    home.mkdir()
    (home / "azure_managed_identity.config").write_text("client-123\n")
    probe = tmp_path / "probe.py"
    probe.write_text(PROBE)
    env = dict(os.environ, PYTHONPATH=f"{root}:{os.getcwd()}", HOME=str(home))
    r = subprocess.run([sys.executable, str(probe), str(tmp_path)], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["sync"] == {"managed_identity_client_id": "client-123"}
    assert out["aio"] == {"managed_identity_client_id": "client-123"}
    assert out["explicit"] == {"managed_identity_client_id": "mine"}
    assert out["ls"] == ["b/dir/x", "b/dir/sub"]
    assert out["adlfs"] == [["mkdir", "c/d"], ["put", str(probe), "c/f"]]
    assert out["abfss"] == "AzureDataLakeArtifactRepository"


def test_no_managed_identity_config_leaves_credentials_alone(tmp_path):
    from cloudtik_amd.runtime.ai import patches
    assert patches.managed_identity_client_id(str(tmp_path / "missing")) is None

    class Cred:
        def __init__(self, **kw):
            self.kw = kw
    patches._wrap_credential_class(Cred)
    old = os.environ.get("HOME")
    os.environ["HOME"] = str(tmp_path)
    try:
        assert Cred().kw == {}
    finally:
        os.environ["HOME"] = old
