#!/usr/bin/env python3
"""Headline benchmark: BERT-large phase-1 pretraining throughput (tokens/s, whole job).

Metric / config from BASELINE.json ("samples/sec ResNet-50 + tokens/sec BERT-large, whole
node, 1/2/4/8 MI355X").  Default run = BERT-large (24 x 1024, 16 heads, vocab 30522),
seq 128, 76 masked-LM slots per sequence (max_predictions_per_seq of the reference's
run_ddp_bert_pretrain_phase1.sh:72), per-GPU batch 256, LAMB (lr 3.5e-4, wd 0.01, betas 0.9/0.999 --
the reference's run_ddp_bert_pretrain_phase1.sh:63 hyper-parameters), bf16 compute with
fp32 master weights, dropout 0.1, random-init weights, synthetic token data.
Data-parallel over RCCL with one process per GPU (weak scaling: fixed per-GPU batch).
``--model resnet50`` measures the ResNet-50 half of the metric (images/s).

Protocol: W untimed warm-up steps, then EXACTLY K timed steps bracketed by a barrier +
torch.cuda.synchronize() on both sides; the max time over ranks is reported.  Every timed
step is a full forward + backward + gradient all-reduce + optimizer step + LR update.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# no published reference number exists (BASELINE.json "published": {}); vs_baseline = null
BASELINE = {"bert-large": None, "resnet50": None}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="bert-large", choices=["bert-large", "bert-base", "resnet50"])
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default per model)")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--max-pred", type=int, default=76,
                    help="masked-LM slots per sequence (reference phase-1: max_predictions_per_seq=76)")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--no-dropout", action="store_true")
    ap.add_argument("--conv-benchmark", action="store_true",
                    help="ResNet: let MIOpen search convolution solvers (torch.backends.cudnn.benchmark)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--tunableop", default="use", choices=["off", "use", "tune"],
                    help="hipBLASLt solution selection via PyTorch TunableOp (results shipped in-tree)")
    return ap.parse_args()


TUNE_FILE = os.path.join(REPO, "cloudtik_amd", "ops", "tunableop", "gfx950_tunableop.csv")


def setup_tunableop(mode, rank):
    """Library GEMMs: let TunableOp pick the fastest hipBLASLt solution per shape.  The tuned
    table (gfx950) is committed in-tree; `--tunableop tune` regenerates it."""
    if mode == "off":
        return
    import torch.cuda.tunable as tn
    if mode == "use" and not os.path.exists(TUNE_FILE):
        return
    os.makedirs(os.path.dirname(TUNE_FILE), exist_ok=True)
    tn.enable(True)
    tn.set_filename(TUNE_FILE if rank == 0 or mode == "use" else TUNE_FILE + f".rank{rank}")
    tn.tuning_enable(mode == "tune")
    if mode == "tune":
        tn.set_max_tuning_duration(60)
        tn.set_max_tuning_iterations(30)


def finish_tunableop(mode, rank):
    # TunableOp writes the results file itself when the process exits
    return None


def bench_bert(args, rank, world, device):
    from cloudtik_amd.models.bert import BertConfig, BertForPreTraining, synthetic_pretraining_batch
    from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
    from cloudtik_amd.train.optim import FusedLAMB, FlatParamSpace
    from cloudtik_amd.train.lr_scheduler import LinearWarmupPolyDecayScheduler
    from cloudtik_amd import ops

    ops.manual_seed(1234 + rank)
    torch.manual_seed(1234)
    cfg = BertConfig.large() if args.model == "bert-large" else BertConfig.base()
    if args.no_dropout:
        cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    model = BertForPreTraining(cfg, device=device, dtype=torch.bfloat16)
    model.train()
    named = [(n, p) for n, p in model.named_parameters()]
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = FusedLAMB(space, lr=3.5e-4, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01,
                    no_decay=BertForPreTraining.no_decay)
    sched = LinearWarmupPolyDecayScheduler(opt, start_warmup_steps=0, warmup_steps=0,
                                           total_steps=13700, end_learning_rate=0.0, degree=1.0)
    broadcast_flat_params(space)
    ddp = GradBucketer(space, bucket_mb=args.bucket_mb)
    opt.grad_scale = ddp.grad_scale
    B = args.batch or 256
    gen = torch.Generator().manual_seed(42 + rank)
    batch = synthetic_pretraining_batch(cfg, B, args.seq, args.max_pred, device=device, generator=gen)

    def step():
        loss = model(**batch)
        loss.backward()
        ddp.finish()
        opt.step()
        sched.step()
        opt.zero_grad()
        return loss

    info = dict(model="bert-large" if args.model == "bert-large" else "bert-base", per_gpu_batch=B,
                seq_len=args.seq, unit="tokens/s", items_per_step=B * args.seq,
                metric="bert_large_pretrain_tokens_per_sec" if args.model == "bert-large"
                else "bert_base_pretrain_tokens_per_sec")
    return step, info


def bench_resnet(args, rank, world, device):
    from cloudtik_amd.models.resnet import resnet50, ResNetTrainStep
    from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
    from cloudtik_amd.train.optim import FusedSGD, FlatParamSpace

    torch.manual_seed(1234)
    if args.conv_benchmark:
        torch.backends.cudnn.benchmark = True
    model = resnet50(device=device)
    model.train()
    named = [(n, p) for n, p in model.named_parameters()]
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = FusedSGD(space, lr=0.1, momentum=0.9, weight_decay=1e-4,
                   no_decay=lambda n: n.endswith("bias") or ".bn" in n or n.startswith("bn"))
    broadcast_flat_params(space)
    ddp = GradBucketer(space, bucket_mb=args.bucket_mb)
    opt.grad_scale = ddp.grad_scale
    B = args.batch or 256
    g = torch.Generator().manual_seed(7 + rank)
    x = torch.randn(B, 3, 224, 224, generator=g).to(device=device, dtype=torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), generator=g).to(device)
    ts = ResNetTrainStep(model, opt, ddp)

    def step():
        return ts(x, y)

    info = dict(model="resnet50", per_gpu_batch=B, seq_len=None, unit="images/s", items_per_step=B,
                metric="resnet50_train_images_per_sec")
    return step, info


def main():
    args = parse()
    from cloudtik_amd.parallel import init_distributed, barrier, all_reduce_max
    rank, world, local, device = init_distributed()
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.backends.cuda.matmul.allow_tf32 = False
    setup_tunableop(args.tunableop, rank)
    fn = bench_bert if args.model.startswith("bert") else bench_resnet
    step, info = fn(args, rank, world, device)

    tw = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if rank == 0:
        print(f"[bench] warm-up {args.warmup} step(s): {time.perf_counter() - tw:.1f}s", file=sys.stderr)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    elapsed = all_reduce_max(t1 - t0)
    ms = elapsed / args.steps * 1000.0
    total_items = info["items_per_step"] * world * args.steps
    value = total_items / elapsed
    lossv = float(loss.detach().float().item())
    if rank == 0:
        base = BASELINE.get(info["model"])
        cfg = {"model": info["model"], "global_batch": info["per_gpu_batch"] * world,
               "per_gpu_batch": info["per_gpu_batch"], "parallelism": f"dp{world}",
               "optimizer": "fused LAMB (HIP)" if info["model"].startswith("bert") else "fused SGD (HIP)",
               "loss_last_step": round(lossv, 4)}
        if info["seq_len"]:
            cfg["seq_len"] = info["seq_len"]
            cfg["max_pred"] = args.max_pred
            cfg["sentences_per_sec"] = round(value / info["seq_len"], 2)
        out = {"metric": info["metric"], "value": round(value, 2), "unit": info["unit"],
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": (round(value / base, 4) if base else None), "dtype": "bf16",
               "data": "synthetic (random tokens/images, random-init weights)", "config": cfg}
        print(json.dumps(out), flush=True)
    finish_tunableop(args.tunableop, rank)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
