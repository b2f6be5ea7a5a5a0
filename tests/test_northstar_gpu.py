"""North-star slice on a real MI355X through the control plane (reference
examples/runtime/ai/basics/pytorch/imagenet-resnet50-synthetic-pytorch-distributed.py:241-268):
``cloudtik start`` of a local-provider cluster whose head is this host (state server, node
monitor, controller), ``cloudtik submit`` of the ResNet-50 synthetic example through the AI
runtime's ``cloudtik-run --nproc-per-node 1``, then config #5 at N = 1 (Parquet -> pinned
loader -> ResNet-50).  The rank must have bound the GPU, mapped the framework's HIP library,
and trained to a finite loss.

The CPU twin (``test_northstar_slice_cpu``) runs the same path with the small model on CPU so
the plumbing is covered by the CPU suite too."""
import glob
import json
import math
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "cloudtik")

CONFIG = """
cluster_name: {name}
provider:
    type: local
available_node_types:
    head.default:
        node_config: {{}}
head_node_type: head.default
runtime:
    types: [ai]
    ai: {{with_gpu: {gpu}}}
"""


def _run(env, *args, timeout=600, check=True):
    r = subprocess.run([CLI, *args], env=env, capture_output=True, text=True, timeout=timeout)
    if check and r.returncode != 0:
        raise AssertionError(f"cloudtik {' '.join(args)} failed ({r.returncode}):\n{r.stdout[-3000:]}\n"
                             f"{r.stderr[-3000:]}")
    return r.stdout


def _cluster(tmp_path, gpu):
    name = f"ns{os.getpid() % 10000}"
    cfg = tmp_path / "cluster.yaml"
    cfg.write_text(CONFIG.format(name=name, gpu=str(gpu).lower()))
    env = dict(os.environ, CLOUDTIK_LOCAL_STATE_DIR=str(tmp_path / "state"), CLOUDTIK_UPDATE_INTERVAL_S="1",
               CLOUDTIK_METRIC_PORT="0", CLOUDTIK_CONFIG_CACHE=str(tmp_path / "cache"),
               CLOUDTIK_PYTHON=sys.executable, CLOUDTIK_SESSION_DIR=str(tmp_path / "session"))
    return env, str(cfg)


def _reports(prefix):
    return [json.load(open(p)) for p in sorted(glob.glob(prefix + ".rank*"))]


def _slice(tmp_path, gpu, model_args):
    env, cfg = _cluster(tmp_path, gpu)
    try:
        assert "is up" in _run(env, "start", cfg, "-y")
        report = str(tmp_path / "rn50")
        out = _run(env, "submit", cfg, os.path.join(ROOT, "examples", "ai", "resnet50_synthetic.py"),
                   "--runtime-options", "--nproc-per-node 1", *model_args, "--report-json", report)
        assert "Img/sec per" in out
        (rep,) = _reports(report)
        assert rep["world"] == 1 and rep["local_rank"] == 0
        assert rep["loss"] is not None and math.isfinite(rep["loss"]) and rep["img_per_sec"] > 0
        out5 = _run(env, "submit", cfg, os.path.join(ROOT, "examples", "ai", "spark_parquet_resnet50.py"),
                    "--runtime-options", "--nproc-per-node 1", "--data-path", str(tmp_path / "parquet"),
                    "--etl-engine", "pyarrow", "--epochs", "1", "--warmup", "1", *(
                        ["--batch-size", "32", "--rows", "256"] if gpu else
                        ["--model", "small", "--batch-size", "16", "--image-size", "32", "--rows", "128"]))
        res = json.loads([ln for ln in out5.splitlines() if ln.startswith("{")][-1])
        assert res["n_gpus"] == 1 and math.isfinite(res["final_loss"]) and res["value"] > 0
        return rep, res
    finally:
        _run(env, "stop", cfg, "-y", "--hard", check=False)


@pytest.mark.gpu
def test_northstar_slice_gpu(tmp_path):
    rep, res = _slice(tmp_path, True, ["--batch-size", "64", "--num-warmup-batches", "2", "--num-iters", "2",
                                       "--num-batches-per-iter", "2"])
    assert rep["device"].startswith("cuda") and rep["device_name"]
    assert any(p.startswith("cloudtik_amd/ops/_C") for p in rep["native_libraries"]), rep["native_libraries"]


def test_northstar_slice_cpu(tmp_path, monkeypatch):
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    rep, res = _slice(tmp_path, False, ["--model", "small", "--batch-size", "8", "--num-warmup-batches", "1",
                                        "--num-iters", "1", "--num-batches-per-iter", "1"])
    assert rep["device"] == "cpu"
