#!/usr/bin/env python3
"""Data-parallel training with the Horovod API served on RCCL (gloo on CPU) by
``cloudtik_amd.parallel.horovod`` (reference examples/runtime/ai/basics/pytorch/
mnist-pytorch-horovod-run-hyperopt-mlflow.py and imagenet-resnet50-pytorch-horovod-run.py):
hvd.init, a rank shard of the data, broadcast of the initial state, DistributedOptimizer,
metric averaging, and tracking from rank 0.

    cloudtik-run -np 2 examples/ai/basics/digits_horovod.py --epochs 5
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--lr", type=float, default=3e-3)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args(argv)
    import torch
    import torch.nn.functional as F
    from cloudtik_amd.parallel import horovod as hvd
    from cloudtik_amd.models.mlp import MLP
    from cloudtik_amd.runtime.ai.tracking import start_run
    from digits_hyperopt_tracking import load_digits_split

    hvd.init()
    dev = torch.device(f"cuda:{hvd.local_rank()}" if torch.cuda.is_available() else "cpu")
    xtr, ytr, xva, yva = (torch.from_numpy(t).to(dev) for t in load_digits_split())
    xtr, ytr = xtr[hvd.rank()::hvd.size()], ytr[hvd.rank()::hvd.size()]         # this rank's shard
    torch.manual_seed(hvd.rank())                                                # different init ...
    model = MLP(64, (128, 64), 10, device=dev)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)                     # ... made identical
    opt = hvd.DistributedOptimizer(torch.optim.Adam(model.parameters(), lr=a.lr * hvd.size()),
                                   named_parameters=model.named_parameters())
    hvd.broadcast_optimizer_state(opt, root_rank=0)
    with start_run("digits-horovod") as run:                                      # rank 0 logs
        run.log_params({"world": hvd.size(), "lr": a.lr, "batch": a.batch})
        for epoch in range(a.epochs):
            model.train()
            for i in range(0, len(xtr), a.batch):
                loss = F.cross_entropy(model(xtr[i:i + a.batch]), ytr[i:i + a.batch])
                opt.zero_grad()
                loss.backward()
                opt.step()
            model.eval()
            with torch.no_grad():
                acc = (model(xva).argmax(1) == yva).float().mean()
            acc = float(hvd.allreduce(acc.detach(), name="val_acc"))                 # averaged over ranks
            run.log_metric("val_accuracy", acc, step=epoch)
    if hvd.rank() == 0:
        print(json.dumps({"world": hvd.size(), "val_accuracy": acc}), flush=True)
    hvd.shutdown()


if __name__ == "__main__":
    main()
