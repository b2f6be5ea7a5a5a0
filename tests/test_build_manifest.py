"""The op library's build manifest: relink on a changed object set, and the stale-build check
that ``cloudtik_amd.ops`` runs at import (ops/build.py ``stale_sources``)."""
import json
import os

import pytest

from cloudtik_amd.ops import build as B


@pytest.fixture
def tree(tmp_path, monkeypatch):
    csrc = tmp_path / "csrc"
    csrc.mkdir()
    (csrc / "a.hip").write_text("kernel a v1\n")
    (csrc / "common.h").write_text("header\n")
    (csrc / "notes.txt").write_text("not a source\n")
    man = tmp_path / "_C.so.objs"
    monkeypatch.setattr(B, "manifest_path", lambda: str(man))
    monkeypatch.setattr(B, "CSRC", str(csrc))
    return csrc, man


def _write_manifest(man, csrc):
    man.write_text(json.dumps({"objs": ["a.hip.x.o"], "sources": B.source_digest(str(csrc))}))


def test_digest_covers_sources_and_headers_only(tree):
    csrc, _ = tree
    d = B.source_digest(str(csrc))
    assert set(d) == {"a.hip", "common.h"}


def test_stale_sources_flags_edits_additions_and_reverts(tree):
    csrc, man = tree
    assert B.stale_sources() is None                         # no manifest: unknown
    _write_manifest(man, csrc)
    assert B.stale_sources() == []
    (csrc / "a.hip").write_text("kernel a v2\n")             # edited after the link
    assert B.stale_sources() == ["a.hip"]
    (csrc / "a.hip").write_text("kernel a v1\n")             # reverted: current again
    assert B.stale_sources() == []
    (csrc / "b.hip").write_text("new kernel\n")              # a source the library lacks
    assert B.stale_sources() == ["b.hip"]


def test_in_tree_library_matches_its_sources():
    """The in-tree library (when built) was linked from the sources in this tree."""
    if not os.path.exists(B.manifest_path()):
        pytest.skip("op library not built in this tree")
    assert B.stale_sources() == []
