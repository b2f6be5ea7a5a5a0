"""Trainer / Checkpointer / MNIST MLP on CPU (north-star config #1 is this path on a local
cluster: see test_cluster_virtual.py for the `cloudtik submit` leg)."""
import json
import os
import socket
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _loaders(n=2000, batch=64):
    from cloudtik_amd.data import NativeLoader
    from cloudtik_amd.models.mlp import synthetic_mnist
    x, y = synthetic_mnist(n, seed=1)
    xt, yt = synthetic_mnist(500, seed=2)
    return (NativeLoader({"x": x, "y": y}, batch, seed=3, device="cpu", drop_last=True),
            NativeLoader({"x": xt, "y": yt}, 250, shuffle=False, device="cpu"))


def test_trainer_learns_mnist_cpu():
    from cloudtik_amd.models.mlp import MLP
    from cloudtik_amd.train.trainer import Trainer
    torch.manual_seed(0)
    tr, te = _loaders()
    t = Trainer(MLP(), "adamw", lr=2e-3, train_loader=tr, eval_loader=te, epochs=2, log_every=0)
    hist = t.fit()
    assert hist[-1]["eval_accuracy"] > 0.9
    assert hist[0]["loss"] > hist[-1]["loss"]


def test_checkpoint_resume_roundtrip(tmp_path):
    from cloudtik_amd.models.mlp import MLP
    from cloudtik_amd.train.trainer import Trainer
    torch.manual_seed(0)
    tr, te = _loaders(1000)
    t1 = Trainer(MLP(), "adamw", lr=1e-3, train_loader=tr, epochs=1, checkpoint_dir=str(tmp_path), log_every=0)
    t1.fit()
    saved = {k: v.clone() for k, v in t1.model.state_dict().items()}
    m_saved = t1.optimizer.exp_avg.clone()
    step = t1.global_step
    torch.manual_seed(123)                       # different init: must be overwritten
    t2 = Trainer(MLP(), "adamw", lr=1e-3, train_loader=tr, epochs=2, checkpoint_dir=str(tmp_path), log_every=0)
    assert t2.global_step == step and t2.start_epoch == 1
    for k, v in t2.model.state_dict().items():
        assert torch.equal(v, saved[k]), k
    assert torch.equal(t2.optimizer.exp_avg, m_saved)
    t2.fit()                                      # continues with epoch 1 only
    assert len(t2.history) == 1 and t2.history[0]["epoch"] == 1
    from cloudtik_amd.train.checkpoint import Checkpointer
    assert Checkpointer(str(tmp_path)).latest_step() == t2.global_step


def test_grad_accumulation_matches_large_batch():
    """SGD on 2 x 32 micro-batches == 1 x 64 batch (same rows, same order)."""
    from cloudtik_amd.models.mlp import MLP
    from cloudtik_amd.train.trainer import Trainer
    x = torch.randn(64, 1, 28, 28)
    y = torch.randint(0, 10, (64,))
    torch.manual_seed(0)
    a = Trainer(MLP(), "sgd", lr=0.1, train_loader=[(x, y)], epochs=1, log_every=0,
                optimizer_kwargs={"momentum": 0.0})
    a.fit()
    torch.manual_seed(0)
    b = Trainer(MLP(), "sgd", lr=0.1, train_loader=[(x[:32], y[:32]), (x[32:], y[32:])], epochs=1, grad_accum=2,
                log_every=0, optimizer_kwargs={"momentum": 0.0})
    b.fit()
    for (k, va), vb in zip(a.model.state_dict().items(), b.model.state_dict().values()):
        torch.testing.assert_close(va, vb, atol=1e-5, rtol=1e-4)


def test_mnist_example_two_ranks_gloo():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([os.path.join(ROOT, "bin", "cloudtik-run"), "--nproc-per-node", "2", "--master-port", str(port),
                        os.path.join(ROOT, "examples", "ai", "mnist_mlp.py"), "--epochs", "2", "--train-size", "4000"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["world"] == 2 and res["final"]["eval_accuracy"] > 0.9
