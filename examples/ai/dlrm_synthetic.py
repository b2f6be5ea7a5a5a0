#!/usr/bin/env python3
"""DLRM training on synthetic Criteo-shaped data with hybrid parallelism (reference:
applications/ai/quickstart DLRM bench/dlrm_s_criteo_terabyte.sh -- 13 dense features,
26 sparse tables, E=64, bottom 512-256-64, top 1024-1024-512-256-1, global batch 2048).

Tables are sharded across ranks (model parallel, fused sparse SGD in the embedding
backward), MLPs are data parallel (flat-buffer bucketed all-reduce + fused SGD); the two
meet in one all-to-all per step.  Prints samples/s.

    cloudtik-run examples/ai/dlrm_synthetic.py --batch-per-rank 2048 --steps 50
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-per-rank", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--table-rows", type=int, default=1000000, help="rows per sparse table")
    ap.add_argument("--num-tables", type=int, default=26)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--tiny", action="store_true")
    a = ap.parse_args()

    from cloudtik_amd.models.dlrm import DLRM, DLRMConfig, synthetic_batch
    from cloudtik_amd.parallel import GradBucketer
    from cloudtik_amd.train.optim import FlatParamSpace, FusedSGD
    from cloudtik_amd.train.trainer import setup_distributed
    rank, world, device = setup_distributed()
    cfg = DLRMConfig.tiny() if a.tiny else DLRMConfig(table_sizes=[a.table_rows] * a.num_tables)
    cfg.sparse_lr = a.lr if device.type == "cuda" else 0.0
    torch.manual_seed(0)
    model = DLRM(cfg, device=device, rank=rank, world=world)
    dense_named = [(n, p) for n, p in model.named_parameters() if not n.startswith("emb.")]
    space = FlatParamSpace([p for _, p in dense_named], names=[n for n, _ in dense_named])
    opt = FusedSGD(space, lr=a.lr, momentum=0.0)
    ddp = GradBucketer(space, bucket_mb=16)
    opt.grad_scale = 1.0          # per-rank loss is pre-divided by world: sum the shares
    emb_opt = torch.optim.SGD([model.emb.weight], lr=a.lr) if cfg.sparse_lr == 0.0 else None
    B = a.batch_per_rank * world
    batches = [synthetic_batch(cfg, B, s, model.local_tables, device) for s in range(4)]
    sl = slice(rank * a.batch_per_rank, (rank + 1) * a.batch_per_rank)

    def step(i):
        dense, labels, idx, offs = batches[i % len(batches)]
        logits = model(dense[sl], idx, offs, B)
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logits.float(), labels[sl]) / world
        loss.backward()
        ddp.finish()
        opt.step()
        opt.zero_grad()
        if emb_opt is not None:
            emb_opt.step()
            emb_opt.zero_grad()
        return loss

    for i in range(a.warmup):
        step(i)
    if device.type == "cuda":
        torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    if device.type == "cuda":
        torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if rank == 0:
        print(json.dumps({"metric": "dlrm_train_samples_per_sec", "value": round(a.steps * B / dt, 1),
                          "world": world, "global_batch": B, "ms_per_step": round(1000 * dt / a.steps, 3),
                          "tables": len(cfg.table_sizes), "rows_per_table": cfg.table_sizes[0],
                          "loss": round(loss.item() * world, 4)}), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
