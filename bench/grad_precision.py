#!/usr/bin/env python3
"""bf16 vs fp32 gradient reduction / accumulation: tiny-BERT loss curves on one GPU.

Same seeds, same data, same dropout stream; the only difference is GradBucketer's
``reduce_dtype`` (None = gradients accumulated over the ``--accum`` micro-batches in the
bf16 flat buffer; fp32 = each backward's bf16 gradients added into an fp32 buffer that the
optimizer reads).  Prints both curves' summary and the max |delta loss| as one JSON line.

    python bench/grad_precision.py --steps 300 --accum 4
"""
import argparse
import json
import os
import sys
from contextlib import nullcontext

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(reduce_fp32, args):
    from cloudtik_amd import ops
    from cloudtik_amd.models.bert import BertConfig, BertForPreTraining, synthetic_pretraining_batch
    from cloudtik_amd.parallel import GradBucketer
    from cloudtik_amd.train.optim import FlatParamSpace, FusedLAMB
    from cloudtik_amd.train.lr_scheduler import LinearWarmupPolyDecayScheduler
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ops.manual_seed(0)
    cfg = BertConfig.tiny(vocab_size=2048, hidden_size=256, num_hidden_layers=4, num_attention_heads=4,
                          intermediate_size=1024)
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16).train()
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = FusedLAMB(space, lr=2e-3, weight_decay=0.01, no_decay=BertForPreTraining.no_decay)
    sched = LinearWarmupPolyDecayScheduler(opt, start_warmup_steps=0, warmup_steps=30, total_steps=args.steps,
                                           end_learning_rate=0.0, degree=1.0)
    ddp = GradBucketer(space, reduce_dtype=torch.float32 if reduce_fp32 else None)
    opt.grad_scale = 1.0 / args.accum
    g = torch.Generator().manual_seed(1)
    pool = [synthetic_pretraining_batch(cfg, args.batch, 128, 20, device=dev, generator=g) for _ in range(16)]
    losses = []
    k = 0
    for _ in range(args.steps):
        tot = 0.0
        for i in range(args.accum):
            ctx = ddp.no_sync() if i < args.accum - 1 else nullcontext()
            with ctx:
                loss = model(**pool[k % len(pool)])
                loss.backward()
            k += 1
            tot += loss.detach().float()
        ddp.finish()
        opt.step()
        sched.step()
        opt.zero_grad()
        losses.append(tot / args.accum)
    return [float(v) for v in torch.stack(losses).cpu()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--accum", type=int, default=4)
    ap.add_argument("--batch", type=int, default=32)
    args = ap.parse_args()
    a = run(False, args)
    b = run(True, args)
    d = [abs(x - y) for x, y in zip(a, b)]
    tail = lambda c: sum(c[-20:]) / 20  # noqa: E731
    print(json.dumps({"steps": args.steps, "accum": args.accum, "loss_first": [a[0], b[0]],
                      "loss_last20_mean_bf16": round(tail(a), 4), "loss_last20_mean_fp32": round(tail(b), 4),
                      "max_abs_delta_loss": round(max(d), 4), "mean_abs_delta_loss": round(sum(d) / len(d), 4),
                      "curve_bf16_every25": [round(v, 3) for v in a[::25]],
                      "curve_fp32_every25": [round(v, 3) for v in b[::25]]}))


if __name__ == "__main__":
    main()
