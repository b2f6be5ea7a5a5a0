#!/usr/bin/env python3
"""MNIST MLP with the cloudtik_amd Trainer (north-star config #1; reference
examples/runtime/ai/basics/pytorch/mnist-pytorch-*.py).

    python examples/ai/mnist_mlp.py                           # 1 process (CPU or GPU)
    cloudtik-run --nproc-per-node 2 examples/ai/mnist_mlp.py  # DP over gloo (CPU) / RCCL (GPU)
    cloudtik submit cluster.yaml examples/ai/mnist_mlp.py --epochs 3

Data: a Parquet directory with ``image`` (784 uint8/float) and ``label`` columns when
``--data`` is given (e.g. written by a Spark job), otherwise synthetic MNIST-shaped data.
"""
import argparse
import json
import logging
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--lr", type=float, default=2e-3)
    ap.add_argument("--train-size", type=int, default=12000)
    ap.add_argument("--data", default=None, help="Parquet directory with image/label columns")
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--optimizer", default="adamw", choices=["adamw", "adam", "sgd", "lamb"])
    args = ap.parse_args()
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(message)s")

    from cloudtik_amd.data import NativeLoader, read_parquet_columns
    from cloudtik_amd.models.mlp import MLP, synthetic_mnist
    from cloudtik_amd.train.trainer import Trainer, setup_distributed

    rank, world, device = setup_distributed()
    if args.data:
        cols = read_parquet_columns(args.data, ["image", "label"], shapes={"image": (1, 28, 28)},
                                    dtypes={"image": "float32", "label": "int64"})
        x, y = torch.from_numpy(cols["image"]), torch.from_numpy(cols["label"])
        if x.max() > 1.5:
            x = x / 255.0
        n_train = int(0.9 * len(y))
        xtr, ytr, xte, yte = x[:n_train], y[:n_train], x[n_train:], y[n_train:]
    else:
        xtr, ytr = synthetic_mnist(args.train_size, seed=1)
        xte, yte = synthetic_mnist(2000, seed=2)
    train = NativeLoader({"x": xtr, "y": ytr}, args.batch, shuffle=True, seed=7, rank=rank, world=world,
                         device=device, drop_last=True)
    test = NativeLoader({"x": xte, "y": yte}, 500, shuffle=False, rank=rank, world=world, device=device)
    model = MLP(device=device)
    trainer = Trainer(model, args.optimizer, lr=args.lr, train_loader=train, eval_loader=test, epochs=args.epochs,
                      checkpoint_dir=args.checkpoint_dir, log_every=50)
    hist = trainer.fit()
    if rank == 0:
        print(json.dumps({"world": world, "device": str(device), "final": hist[-1]}), flush=True)
    trainer.close()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
