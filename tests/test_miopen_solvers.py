"""MIOpen solver-db installation (ops/miopen_solvers.py): never silently skipped.

CPU tests cover the install decisions (private copy, merge into a preset
MIOPEN_USER_DB_PATH, fallback directories, names for another CU count); the GPU test
profiles a ResNet-50 bottleneck fwd + bwd at the benchmark's shapes and fails if MIOpen
ran any naive convolution kernel (the fallback that costs 25-200 ms per call)."""
import os

import pytest
import torch

from cloudtik_amd.ops import miopen_solvers as M


def _records(path):
    return M._read_records(path)


def test_private_copy(monkeypatch, tmp_path):
    monkeypatch.delenv("MIOPEN_USER_DB_PATH", raising=False)
    monkeypatch.setenv("CLOUDTIK_AMD_CACHE", str(tmp_path))
    monkeypatch.setattr(M, "_kfd_cu_counts", lambda: [])
    st = M.install()
    assert st["installed"] and st["mode"] == "private copy"
    assert os.environ["MIOPEN_USER_DB_PATH"] == st["path"] and st["path"].startswith(str(tmp_path))
    for f in M.shipped_files():
        assert _records(os.path.join(st["path"], f)) == _records(os.path.join(M.SRC, f))


def test_merge_into_preset_keeps_other_records(monkeypatch, tmp_path):
    f = [x for x in M.shipped_files() if x.endswith(".ufdb.txt")][0]
    ours = _records(os.path.join(M.SRC, f))
    key = next(iter(ours))
    (tmp_path / f).write_text(f"{key}=ConvDirectNaiveConvFwd:1.0,0,miopenConvolutionFwdAlgoDirect\n"
                              "other-problem-key=SomeSolver:0.5,0,x\n")
    monkeypatch.setenv("MIOPEN_USER_DB_PATH", str(tmp_path))
    monkeypatch.setattr(M, "_kfd_cu_counts", lambda: [])
    st = M.install()
    assert st["installed"] and st["mode"].startswith("merged")
    recs = _records(str(tmp_path / f))
    assert recs[key] == ours[key]                          # the shipped solver list wins
    assert recs["other-problem-key"] == "SomeSolver:0.5,0,x"  # foreign records survive


def test_falls_back_to_a_writable_directory(monkeypatch, tmp_path):
    monkeypatch.delenv("MIOPEN_USER_DB_PATH", raising=False)
    bad = tmp_path / "file-not-dir"
    bad.write_text("x")
    monkeypatch.setenv("CLOUDTIK_AMD_CACHE", str(bad))          # makedirs under a file fails
    monkeypatch.setenv("XDG_CACHE_HOME", str(bad))
    monkeypatch.setenv("HOME", str(bad))
    monkeypatch.setenv("TMPDIR", str(tmp_path / "ok"))
    monkeypatch.setattr(M, "_kfd_cu_counts", lambda: [])
    monkeypatch.setattr(M.tempfile, "gettempdir", lambda: str(tmp_path / "ok"))
    st = M.install()
    assert st["installed"] and st["path"].startswith(str(tmp_path / "ok"))
    assert st["skipped"]                                     # the failures are reported, not swallowed


def test_alternate_cu_count_names(monkeypatch, tmp_path):
    monkeypatch.delenv("MIOPEN_USER_DB_PATH", raising=False)
    monkeypatch.setenv("CLOUDTIK_AMD_CACHE", str(tmp_path))
    monkeypatch.setattr(M, "_kfd_cu_counts", lambda: [240])
    st = M.install()
    names = set(os.listdir(st["path"]))
    for f in M.shipped_files():
        assert f in names
        alt = M._NAME.sub(lambda m: f"{m.group(1)}f0.{m.group(3)}.{m.group(4)}.txt", f)
        assert alt in names, (alt, names)


def test_disabled_is_reported(monkeypatch):
    monkeypatch.setenv("CLOUDTIK_AMD_MIOPEN_DB", "0")
    st = M.install()
    assert not st["installed"] and "disabled" in st["reason"]


@pytest.mark.gpu
def test_bottleneck_runs_no_naive_conv_kernels(cuda):
    from torch.profiler import ProfilerActivity, profile
    from cloudtik_amd.models.resnet import Bottleneck
    assert M.status()["installed"], M.status()
    torch.manual_seed(0)
    # layer1 block 0 of ResNet-50 at the benchmark batch (the shapes the shipped db covers)
    blk = Bottleneck(64, 64, 1, downsample=True, device=cuda, dtype=torch.bfloat16).to(
        memory_format=torch.channels_last)
    x = torch.randn(256, 64, 56, 56, device=cuda, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_()

    def step():
        blk(x).float().square().mean().backward()

    step()                                   # first call: kernel compile / db lookup
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert names, "profiler saw no GPU kernels"
    naive = sorted({n for n in names if "naive" in n.lower()})
    assert not naive, naive
