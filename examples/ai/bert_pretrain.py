#!/usr/bin/env python3
"""BERT pretraining from pre-tokenised shards -- the quickstart BERT-large workload
(reference: applications/ai/quickstart/bin/bert-large/train-distributed.sh ->
run_ddp_bert_pretrain_phase1.sh -> run_pretrain_mlperf.py).

Same recipe as the reference: ``BertForPreTraining`` (MLM + NSP), LAMB (betas 0.9/0.999,
eps 1e-6, weight decay 0.01 except bias / LayerNorm), linear-warmup + polynomial-decay LR,
gradient accumulation, bf16 compute with fp32 master weights, checkpoint / resume, periodic
evaluation.  MI355X-side: one rank per GPU over RCCL (``cloudtik-run`` / torchrun), flat
parameter space with bucketed all-reduce overlapped with backward, the native pinned-memory
loader, the HIP kernels of ``cloudtik_amd.ops``.

Shards are Parquet files with the MLPerf shard columns (the reference's HDF5 layout):
``input_ids``, ``segment_ids``, ``input_mask`` [seq]; ``masked_lm_positions``,
``masked_lm_ids`` [max_pred] (position 0 = padding slot); ``next_sentence_labels``.

    python examples/ai/bert_pretrain.py --make-shards 4 --data-dir /data/bert_shards --config tiny
    cloudtik-run --nproc_per_node 8 examples/ai/bert_pretrain.py --data-dir /data/bert_shards \\
        --batch 256 --total-steps 7038 --warmup-proportion 0.2843 --ckpt-dir /ckpt/bert
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

COLUMNS = ["input_ids", "segment_ids", "input_mask", "masked_lm_positions", "masked_lm_ids",
           "next_sentence_labels"]


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--data-dir", required=True, help="directory of training shards (*.parquet)")
    ap.add_argument("--eval-dir", default="", help="directory of evaluation shards")
    ap.add_argument("--make-shards", type=int, default=0, help="write N synthetic shards to --data-dir and exit")
    ap.add_argument("--shard-rows", type=int, default=4096)
    ap.add_argument("--config", default="large", choices=["large", "base", "tiny"])
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--max-pred", type=int, default=76)
    ap.add_argument("--batch", type=int, default=32, help="per-rank micro-batch")
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--lr", type=float, default=3.5e-4)
    ap.add_argument("--weight-decay", type=float, default=0.01)
    ap.add_argument("--warmup-proportion", type=float, default=0.0)
    ap.add_argument("--total-steps", type=int, default=13700, help="LR schedule length (optimizer steps)")
    ap.add_argument("--max-steps", type=int, default=0, help="stop after this many optimizer steps")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--ckpt-dir", default="")
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--log-every", type=int, default=10)
    ap.add_argument("--no-dropout", action="store_true")
    ap.add_argument("--seed", type=int, default=42)
    return ap.parse_args(argv)


def make_shards(args, cfg):
    """Synthetic shards in the MLPerf layout (random tokens, sorted masked positions)."""
    rng = np.random.default_rng(args.seed)
    os.makedirs(args.data_dir, exist_ok=True)
    from cloudtik_amd.data.parquet import write_parquet
    n, S, P = args.shard_rows, args.seq, args.max_pred
    for i in range(args.make_shards):
        lens = rng.integers(S // 2, S + 1, n)
        ids = rng.integers(5, cfg.vocab_size, (n, S)).astype(np.int32)
        mask = (np.arange(S)[None, :] < lens[:, None]).astype(np.int8)
        ids *= mask
        seg = ((np.arange(S)[None, :] >= (lens // 2)[:, None]) & (mask > 0)).astype(np.int8)
        npred = np.minimum(P, np.maximum(1, (lens * 0.15).astype(int)))
        pos = np.zeros((n, P), np.int32)
        mids = np.zeros((n, P), np.int32)
        for r in range(n):
            p = np.sort(rng.choice(np.arange(1, lens[r]), npred[r], replace=False))
            pos[r, :npred[r]] = p
            mids[r, :npred[r]] = ids[r, p]
        write_parquet(os.path.join(args.data_dir, f"part-{i:05d}.parquet"),
                      {"input_ids": ids, "segment_ids": seg, "input_mask": mask, "masked_lm_positions": pos,
                       "masked_lm_ids": mids, "next_sentence_labels": rng.integers(0, 2, n).astype(np.int8)})
    print(f"wrote {args.make_shards} shards x {n} rows to {args.data_dir}")


def to_model_batch(b):
    """Shard columns -> BertForPreTraining inputs; padding mask slots (position 0) are
    ignored by the loss, as in the reference's masked_lm_labels construction."""
    pos = b["masked_lm_positions"].long()
    return dict(input_ids=b["input_ids"].long(), token_type_ids=b["segment_ids"].long(),
                attention_mask=b["input_mask"].long(), masked_lm_positions=pos,
                masked_lm_ids=torch.where(pos > 0, b["masked_lm_ids"].long(), torch.full_like(pos, -100)),
                next_sentence_labels=b["next_sentence_labels"].long())


def main(argv=None):
    args = parse(argv)
    from cloudtik_amd.models.bert import BertConfig, BertForPreTraining
    cfg = {"large": BertConfig.large, "base": BertConfig.base, "tiny": BertConfig.tiny}[args.config]()
    if args.make_shards:
        make_shards(args, cfg)
        return {}
    from cloudtik_amd.data.parquet import ParquetDataLoader
    from cloudtik_amd.train.lr_scheduler import LinearWarmupPolyDecayScheduler
    from cloudtik_amd.train.optim import build_optimizer
    from cloudtik_amd.train.trainer import Trainer, setup_distributed

    rank, world, device = setup_distributed()
    if args.no_dropout:
        cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    torch.manual_seed(args.seed)
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    model = BertForPreTraining(cfg, device=device, dtype=dtype)
    opt = build_optimizer("lamb", model, args.lr, args.weight_decay, BertForPreTraining.no_decay,
                          betas=(0.9, 0.999), eps=1e-6)
    sched = LinearWarmupPolyDecayScheduler(opt, start_warmup_steps=0,
                                           warmup_steps=int(args.warmup_proportion * args.total_steps),
                                           total_steps=args.total_steps, end_learning_rate=0.0, degree=1.0)
    files = sorted(glob.glob(os.path.join(args.data_dir, "**", "*.parquet"), recursive=True))
    if not files:
        raise SystemExit(f"no shards under {args.data_dir} (use --make-shards N to write synthetic ones)")
    loader = ParquetDataLoader(files, args.batch, columns=COLUMNS, seed=args.seed, device=device, drop_last=True,
                               rank=rank, world=world)
    eval_loader = None
    if args.eval_dir:
        ef = sorted(glob.glob(os.path.join(args.eval_dir, "**", "*.parquet"), recursive=True))
        eval_loader = ParquetDataLoader(ef, args.batch, columns=COLUMNS, seed=0, device=device, drop_last=True,
                                        rank=rank, world=world, shuffle=False)

    def step(m, b):
        loss = m(**to_model_batch(b))
        return loss, {"loss": loss.detach()}

    trainer = Trainer(model, optimizer=opt, train_loader=loader, eval_loader=eval_loader, step_fn=step,
                      epochs=args.epochs, max_steps=args.max_steps or None, lr_scheduler=sched,
                      grad_accum=args.grad_accum, checkpoint_dir=args.ckpt_dir or None,
                      checkpoint_every=args.ckpt_every, log_every=args.log_every)
    t0 = time.perf_counter()
    start = trainer.global_step
    hist = trainer.fit()
    if device.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = trainer.global_step - start
    result = {"steps": trainer.global_step, "final_loss": hist[-1].get("loss") if hist else None,
              "tokens_per_sec": round(steps * args.batch * args.grad_accum * world * args.seq / max(dt, 1e-9), 1),
              "world": world}
    if eval_loader is not None:
        result["eval"] = trainer.evaluate()
    trainer.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    return result


if __name__ == "__main__":
    main()
