#!/usr/bin/env python3
"""Headline benchmark: BERT-large pretraining tokens/s + ResNet-50 training images/s, whole job.

Metric / config from BASELINE.json ("samples/sec ResNet-50 + tokens/sec BERT-large, whole
node, 1/2/4/8 MI355X").  One invocation measures BOTH halves, one after the other in the
same rank processes:

* BERT-large (24 x 1024, 16 heads, vocab 30522), seq 128, 76 masked-LM slots per sequence
  (max_predictions_per_seq, reference run_ddp_bert_pretrain_phase1.sh:72), per-GPU batch 256,
  LAMB (lr 3.5e-4, wd 0.01, betas 0.9/0.999: run_ddp_bert_pretrain_phase1.sh:63) with fp32
  master weights, bf16 compute, dropout 0.1 -> ``value`` (tokens/s over all ranks);
* ResNet-50 v1.5, 224x224, per-GPU batch 256, SGD momentum 0.9, wd 1e-4, bf16 NHWC
  (reference protocol: examples/runtime/ai/basics/pytorch/
  imagenet-resnet50-synthetic-pytorch-distributed.py:156-210) -> ``resnet50_images_per_sec``.

Random-init weights and synthetic data (one resident batch per rank, re-used every step).
Data parallel over RCCL, one process per GPU, weak scaling (fixed per-GPU batch).

Protocol per model: W untimed warm-up steps, then EXACTLY K timed steps bracketed by a
barrier + torch.cuda.synchronize() on both sides; the max time over ranks is reported.  Each
timed step is forward + backward + bucketed gradient all-reduce + optimizer step (+ LR
schedule for BERT).

Launch:
    python bench.py --gpus N --steps K --warmup W          # spawns N rank processes itself
    torchrun --nproc-per-node N bench.py --gpus N ...       # or ranks from the environment
Options: ``--model bert-large|resnet50`` (one half only), ``--impl eager`` (stock PyTorch
baseline: HF BertForPreTraining + SDPA + DDP + per-tensor LAMB / nn.Conv2d+BatchNorm2d
ResNet-50 + DDP + torch SGD), ``--compare-eager`` (also run the eager baseline and report
the ratio), ``--device cpu --model tiny`` (gloo plumbing check).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# no published reference number exists (BASELINE.json "published": {}): vs_baseline is the ratio
# to the same-config stock PyTorch-ROCm eager step measured in the same run (--baseline-steps)
BASELINE = {"bert-large": None, "resnet50": None}
BASELINE_DESC = ("same-config stock PyTorch-ROCm eager step measured in this run after the native one "
                 "(HF BertForPreTraining + SDPA + per-tensor LAMB / torchvision-style ResNet-50 + torch SGD, "
                 "autocast bf16, stock DDP at world size > 1); BASELINE.json publishes no number")
TUNE_FILE = os.environ.get("CLOUDTIK_BENCH_TUNE_FILE") or os.path.join(REPO, "cloudtik_amd", "ops", "tunableop",
                                                                         "gfx950_tunableop.csv")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="all", choices=["all", "bert-large", "bert-base", "resnet50", "tiny"])
    ap.add_argument("--impl", default="native", choices=["native", "eager"])
    ap.add_argument("--compare-eager", action="store_true",
                    help="also run the stock-PyTorch baseline of the same config for the full K / W steps")
    ap.add_argument("--baseline-steps", type=int, default=-1,
                    help="native runs: after the native halves, time this many steps of the same-config stock "
                         "PyTorch-ROCm eager step (SURVEY.md section 6 item 3; BASELINE.json publishes no "
                         "number) and report native / eager as vs_baseline; 0 = skip; -1 (default) = 5 at "
                         "world size 1, skipped above (a stock-DDP failure on one rank would leave the others "
                         "in a collective: the scaling runs never risk it)")
    ap.add_argument("--baseline-warmup", type=int, default=2)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--batch", type=int, default=0, help="BERT per-GPU batch (default 256)")
    ap.add_argument("--rn-batch", type=int, default=0, help="ResNet-50 per-GPU batch (default 256)")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--max-pred", type=int, default=76,
                    help="masked-LM slots per sequence (reference phase-1: max_predictions_per_seq=76)")
    ap.add_argument("--bucket-mb", default="auto",
                    help="BERT gradient bucket (MiB), or auto: the size measured on this node for this "
                         "world size by bench/comm_bench.py --write-tuning (parallel/comm_tuning.py), "
                         "64 MiB when never measured")
    ap.add_argument("--rn-bucket-mb", default="auto",
                    help="ResNet-50 gradient bucket (MiB) or auto (measured, else 8 MiB): its 51 MB of "
                         "bf16 gradients would be ONE 64 MiB bucket, all-reduced only after the whole "
                         "backward; 8 MiB gives 7 buckets that overlap the backward of the earlier stages")
    ap.add_argument("--grad-dtype", default="auto", choices=["auto", "bf16", "fp32"],
                    help="native path, gradient REDUCTION precision: fp32 = the bf16 per-backward "
                         "gradients are summed across ranks in fp32 (the reference's DDP all-reduces "
                         "fp32 gradients, run_pretrain_mlperf.py:688-691); bf16 = summed in bf16 (half "
                         "the bytes on the wire); auto = fp32 at world size > 1 (at world size 1 nothing "
                         "is reduced and the optimizer reads the bf16 gradients either way)")
    ap.add_argument("--zero", action="store_true",
                    help="ZeRO-1: reduce-scatter gradients, shard optimizer state, all-gather weights")
    ap.add_argument("--no-dropout", action="store_true")
    ap.add_argument("--graph", default="off", choices=["auto", "on", "off"],
                    help="ResNet-50: capture the whole training step into one hipGraph and replay it "
                         "(train/graph_step.py); auto = on at world size 1 (collectives are not captured). "
                         "Off by default: measured 28.9-29.1 ms/step replayed vs 27.2 eager (the eager "
                         "step is GPU-bound and its side-stream overlap survives capture only partly)")
    ap.add_argument("--conv-benchmark", action="store_true",
                    help="ResNet: let MIOpen search convolution solvers (torch.backends.cudnn.benchmark)")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="auto: RCCL on GPU, gloo on CPU; gloo on GPU lets several ranks share "
                         "one GPU (plumbing check of the GPU data-parallel path without RCCL)")
    ap.add_argument("--tunableop", default=os.environ.get("CLOUDTIK_BENCH_TUNABLEOP", "use"),
                    choices=["off", "use", "tune"],
                    help="hipBLASLt solution selection via PyTorch TunableOp (results shipped in-tree)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ rank launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """Start n rank processes of this script (one per GPU) and wait for them.

    Runs before anything touches the GPU in this (parent) process.  If any rank fails, the
    others are terminated (no rank is left blocked in a collective until the RCCL timeout).
    Returns the first non-zero exit code, else 0."""
    port = _free_port()
    cpus = rank_cpus(n)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CLOUDTIK_BENCH_CHILD="1")
        pin = cpus.get(r)
        if pin:
            env["CLOUDTIK_BENCH_CPUS"] = ",".join(map(str, pin))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      preexec_fn=(lambda c=pin: os.sched_setaffinity(0, c)) if pin else None))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
                deadline = time.time() + 30
                for q in live:
                    try:
                        q.wait(max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
        time.sleep(0.2)
    return rc if rc >= 0 else 128 - rc


def rank_cpus(n: int):
    """local rank -> cores of its GPU's NUMA node (runner/affinity.py), restricted to the cores
    this process may use; {} when the topology is unknown or leaves a rank no core."""
    try:
        from cloudtik_amd.runner.affinity import rank_cpu_sets
        allowed = os.sched_getaffinity(0)
        out = {}
        for r, cores in rank_cpu_sets(n).items():
            c = sorted(set(cores) & allowed)
            if not c:
                return {}
            out[r] = c
        return out
    except Exception:  # noqa: BLE001 - affinity is an optimisation, never a failure
        return {}


# ------------------------------------------------------------------ TunableOp
def setup_tunableop(mode, rank):
    """Library GEMMs: let TunableOp pick the fastest hipBLASLt solution per shape.  The tuned
    table (gfx950) is committed in-tree; `--tunableop tune` regenerates it."""
    import torch
    if mode == "off" or not torch.cuda.is_available():
        return
    import torch.cuda.tunable as tn
    if mode == "use" and not os.path.exists(TUNE_FILE):
        return
    tn.enable(True)
    if mode == "use" and os.environ.get("CLOUDTIK_BENCH_TUNE_DIRECT") == "1":
        tn.set_filename(TUNE_FILE)
    elif mode == "use":
        # every rank reads its own private copy: N ranks never rewrite the shared in-tree
        # table at exit (TunableOp writes its results file when the process ends)
        import shutil
        import tempfile
        fd, path = tempfile.mkstemp(prefix=f"tunableop_rank{rank}_", suffix=".csv")
        os.close(fd)
        shutil.copyfile(TUNE_FILE, path)
        tn.set_filename(path)
    else:
        tn.set_filename(TUNE_FILE if rank == 0 else TUNE_FILE + f".rank{rank}")
    tn.tuning_enable(mode == "tune")
    if mode == "tune":
        tn.set_max_tuning_duration(60)
        tn.set_max_tuning_iterations(30)


def resolve_bucket_mb(value, world: int, default: float) -> float:
    """``--bucket-mb`` value: a number, or ``auto`` = the bucket measured for this world size
    (parallel/comm_tuning.py), else ``default``.  ``auto`` reads a per-node file, so the ranks
    AGREE on rank 0's value before any bucket plan is built: ranks with different plans would
    issue all-reduces of different sizes (a hang, or gradients summed across parameters)."""
    if str(value).lower() != "auto":
        return float(value)
    from cloudtik_amd.parallel.comm_tuning import bucket_mb
    mb = float(bucket_mb(world, default))
    import torch.distributed as dist
    if world > 1 and dist.is_initialized():
        vals = [None] * dist.get_world_size()
        dist.all_gather_object(vals, mb)
        if len(set(vals)) > 1 and dist.get_rank() == 0:
            print(f"[bench] note: per-node measured bucket sizes differ {vals}; every rank uses rank 0's "
                  f"{vals[0]} MiB", file=sys.stderr)
        mb = float(vals[0])
    return mb


def reduce_fp32(args, world: int) -> bool:
    """Whether gradients are summed across ranks in fp32 (``--grad-dtype``)."""
    if args.grad_dtype == "auto":
        return world > 1
    return args.grad_dtype == "fp32"


def bucket_plan(ddp):
    """Gradient-bucket plan of a GradBucketer: count, sizes, collective, wire dtype."""
    esize = ddp.space.grad.element_size() if not ddp.fp32 else 4
    sizes = [(hi - lo) * esize for lo, hi, _ in ddp.buckets]
    return {"buckets": len(sizes), "bytes_total": sum(sizes), "bytes_max": max(sizes) if sizes else 0,
            "bytes_min": min(sizes) if sizes else 0,
            "collective": "reduce_scatter+all_gather (ZeRO-1)" if ddp.zero else "all_reduce",
            "overlap_with_backward": bool(ddp.overlap), "p2p_small_buckets": ddp.p2p is not None}


def environment(device, world):
    """Versions and state that decide performance on a fresh box (printed to stderr and
    recorded in the JSON line)."""
    import torch
    import torch.distributed as dist
    env = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None)}
    try:
        from cloudtik_amd import ops
        from cloudtik_amd.ops import miopen_solvers
        env["native_ops"] = ops.native_available()
        env["miopen_db"] = miopen_solvers.status()
    except Exception as e:  # noqa: BLE001
        env["ops_error"] = repr(e)[:200]
    if device.type == "cuda":
        p = torch.cuda.get_device_properties(device)
        env["gpu"] = {"name": p.name, "arch": getattr(p, "gcnArchName", None), "cus": p.multi_processor_count,
                      "hbm_gib": round(p.total_memory / 2 ** 30, 1)}
        try:
            v = torch.cuda.nccl.version()
            env["rccl"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
        except Exception:  # noqa: BLE001
            env["rccl"] = None
    env["nccl_env"] = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_"))}
    if os.environ.get("CLOUDTIK_BENCH_CPUS"):
        env["rank0_cpus"] = os.environ["CLOUDTIK_BENCH_CPUS"]
    if dist.is_initialized():
        # world size as seen by a real collective (not just the launcher's env)
        t = torch.ones(1, device=device)
        dist.all_reduce(t)
        env["world_size_seen_by_collective"] = int(t.item())
        # physical devices behind the ranks (gloo ranks may share one GPU)
        ident = f"{socket.gethostname()}:{device.type}:{device.index if device.type == 'cuda' else os.getpid()}"
        ids = [None] * world
        dist.all_gather_object(ids, ident)
        env["distinct_devices"] = len(set(ids)) if device.type == "cuda" else None
    return env


# ------------------------------------------------------------------ native builders
def build_bert(args, rank, world, device, kind):
    import torch
    from cloudtik_amd.models.bert import BertConfig, BertForPreTraining, synthetic_pretraining_batch
    from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
    from cloudtik_amd.train.optim import FusedLAMB, FlatParamSpace
    from cloudtik_amd.train.lr_scheduler import LinearWarmupPolyDecayScheduler
    from cloudtik_amd import ops

    ops.manual_seed(1234 + rank)
    torch.manual_seed(1234)
    # weight-gradient routing: the model's own (in line: BertForPreTraining), the same at
    # every world size
    cfg = {"bert-large": BertConfig.large, "bert-base": BertConfig.base, "tiny": BertConfig.tiny}[kind]()
    if args.no_dropout:
        cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    model = BertForPreTraining(cfg, device=device, dtype=dtype)
    model.train()
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named],
                           shard=(rank, world) if args.zero and world > 1 else (0, 1))
    opt = FusedLAMB(space, lr=3.5e-4, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01,
                    no_decay=BertForPreTraining.no_decay)
    sched = LinearWarmupPolyDecayScheduler(opt, start_warmup_steps=0, warmup_steps=0,
                                           total_steps=13700, end_learning_rate=0.0, degree=1.0)
    broadcast_flat_params(space)
    ddp = GradBucketer(space, bucket_mb=resolve_bucket_mb(args.bucket_mb, world, 64.0),
                       reduce_dtype=torch.float32 if reduce_fp32(args, world) else None,
                       mode="reduce_scatter" if args.zero and world > 1 else "all_reduce")
    opt.grad_scale = ddp.grad_scale
    B = args.batch or (256 if kind != "tiny" else 4)
    S = args.seq if kind != "tiny" else 32
    P = args.max_pred if kind != "tiny" else 5
    gen = torch.Generator().manual_seed(42 + rank)
    batch = synthetic_pretraining_batch(cfg, B, S, P, device=device, generator=gen)

    def step():
        loss = model(**batch)
        loss.backward()
        ddp.finish()
        opt.step()
        sched.step()
        opt.zero_grad()
        return loss

    def close():
        ddp.remove()

    info = dict(model=kind if kind != "tiny" else "bert-tiny", per_gpu_batch=B, seq_len=S, max_pred=P,
                unit="tokens/s", items_per_step=B * S,
                metric="bert_large_pretrain_tokens_per_sec" if kind in ("bert-large", "tiny")
                else "bert_base_pretrain_tokens_per_sec",
                optimizer="fused LAMB (HIP)", impl="native", plan=bucket_plan(ddp), bucketer=ddp)
    return step, close, info


def build_resnet(args, rank, world, device, kind):
    import torch
    from cloudtik_amd.models.resnet import resnet50, resnet18_like_small, ResNetTrainStep
    from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
    from cloudtik_amd.train.optim import FusedSGD, FlatParamSpace

    torch.manual_seed(1234)
    # weight gradients on the side stream beside the memory-bound backward: the model's own
    # routing (models/resnet.py)
    if args.conv_benchmark:
        torch.backends.cudnn.benchmark = True
    tiny = kind == "tiny"
    model = resnet18_like_small(device=device) if tiny else resnet50(device=device)
    model.train()
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named],
                           shard=(rank, world) if args.zero and world > 1 else (0, 1))
    opt = FusedSGD(space, lr=0.1, momentum=0.9, weight_decay=1e-4,
                   no_decay=lambda n: n.endswith("bias") or ".bn" in n or n.startswith("bn"))
    broadcast_flat_params(space)
    ddp = GradBucketer(space, bucket_mb=resolve_bucket_mb(args.rn_bucket_mb, world, 8.0),
                       reduce_dtype=torch.float32 if reduce_fp32(args, world) else None,
                       mode="reduce_scatter" if args.zero and world > 1 else "all_reduce")
    opt.grad_scale = ddp.grad_scale
    B = args.rn_batch or (256 if not tiny else 4)
    R = 224 if not tiny else 32
    g = torch.Generator().manual_seed(7 + rank)
    x = torch.randn(B, 3, R, R, generator=g).to(device=device, dtype=next(model.parameters()).dtype)
    if device.type == "cuda":
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10 if tiny else 1000, (B,), generator=g).to(device)
    ts = ResNetTrainStep(model, opt, ddp)
    step = lambda: ts(x, y)  # noqa: E731
    graph = device.type == "cuda" and (args.graph == "on" or (args.graph == "auto" and world == 1))
    if graph:
        from cloudtik_amd.train.graph_step import GraphedStep
        step = GraphedStep(step, optimizers=[opt], warmup=min(3, max(0, args.warmup - 1)))

    info = dict(model="resnet50" if not tiny else "resnet-tiny", per_gpu_batch=B, seq_len=None,
                unit="images/s", items_per_step=B, metric="resnet50_train_images_per_sec",
                optimizer="fused SGD (HIP)", impl="native", image_size=R, plan=bucket_plan(ddp),
                hip_graph=bool(graph), bucketer=None if graph else ddp)
    return step, ddp.remove, info


# ------------------------------------------------------------------ eager (stock PyTorch) builders
def _ddp(model, device, world):
    import torch
    if world <= 1:
        return model
    from torch.nn.parallel import DistributedDataParallel as DDP
    return DDP(model, device_ids=[device.index] if device.type == "cuda" else None)


def build_bert_eager(args, rank, world, device, kind):
    import torch
    from cloudtik_amd.benchmarks.eager import (ReferenceLAMB, build_hf_bert, dense_mlm_labels, hf_bert_config,
                                               lamb_param_groups)
    from cloudtik_amd.models.bert import BertConfig, synthetic_pretraining_batch
    tiny = kind == "tiny"
    extra = dict(vocab_size=512, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                 intermediate_size=512, max_position_embeddings=128) if tiny else {}
    if args.no_dropout:
        extra.update(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    hcfg = hf_bert_config(large=kind != "bert-base", **extra)
    model = build_hf_bert(hcfg, device)
    model.train()
    opt = ReferenceLAMB(lamb_param_groups(model, 0.01), lr=3.5e-4, betas=(0.9, 0.999), eps=1e-6)
    dm = _ddp(model, device, world)
    B = args.batch or (256 if not tiny else 4)
    S = args.seq if not tiny else 32
    P = args.max_pred if not tiny else 5
    ours = BertConfig(vocab_size=hcfg.vocab_size)
    gen = torch.Generator().manual_seed(42 + rank)
    b = synthetic_pretraining_batch(ours, B, S, P, device=device, generator=gen)
    labels = dense_mlm_labels(b, S)
    amp = device.type == "cuda"

    def step():
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=amp):
            out = dm(input_ids=b["input_ids"], token_type_ids=b["token_type_ids"],
                     attention_mask=b["attention_mask"], labels=labels, next_sentence_label=b["next_sentence_labels"])
        out.loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return out.loss

    info = dict(model=kind if not tiny else "bert-tiny", per_gpu_batch=B, seq_len=S, max_pred=P, unit="tokens/s",
                items_per_step=B * S, metric="bert_large_pretrain_tokens_per_sec",
                optimizer="per-tensor LAMB (stock PyTorch)", impl="eager")
    return step, (lambda: None), info


def build_resnet_eager(args, rank, world, device, kind):
    import torch
    import torch.nn.functional as F
    from cloudtik_amd.benchmarks.eager import StockResNet50
    tiny = kind == "tiny"
    torch.manual_seed(1234)
    if args.conv_benchmark:
        torch.backends.cudnn.benchmark = True
    model = StockResNet50(num_classes=10 if tiny else 1000).to(device)
    if device.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, foreach=True)
    dm = _ddp(model, device, world)
    B = args.rn_batch or (256 if not tiny else 4)
    R = 224 if not tiny else 32
    g = torch.Generator().manual_seed(7 + rank)
    x = torch.randn(B, 3, R, R, generator=g).to(device)
    if device.type == "cuda":
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10 if tiny else 1000, (B,), generator=g).to(device)
    amp = device.type == "cuda"

    def step():
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=amp):
            loss = F.cross_entropy(dm(x).float(), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    info = dict(model="resnet50" if not tiny else "resnet-tiny", per_gpu_batch=B, seq_len=None, unit="images/s",
                items_per_step=B, metric="resnet50_train_images_per_sec", optimizer="torch.optim.SGD (foreach)",
                impl="eager", image_size=R)
    return step, (lambda: None), info


# ------------------------------------------------------------------ GPU telemetry
class GpuTelemetry:
    """Clock / power / temperature of this rank's GPU (amdgpu sysfs), sampled right before
    and after a timed region and every ``period`` s inside it by a daemon thread (a sysfs
    read costs microseconds and never touches the GPU queue).  An MFMA-bound step's speed
    follows the clock the chip holds under load, so a slow box and a regression can be told
    apart from the JSON line alone."""

    def __init__(self, device, period=0.25):
        self.dev_dir = None
        self.period = period
        self._samples = []
        self._stop = None
        self._thread = None
        if device.type != "cuda":
            return
        try:
            import torch
            from cloudtik_amd.core.node.metrics import pci_device_dir
            p = torch.cuda.get_device_properties(device)
            self.dev_dir = pci_device_dir(getattr(p, "pci_domain_id", 0), p.pci_bus_id, p.pci_device_id)
        except Exception:  # noqa: BLE001 - telemetry is informational
            self.dev_dir = None

    def snapshot(self):
        if self.dev_dir is None:
            return {}
        try:
            from cloudtik_amd.core.node.metrics import gpu_clock_snapshot
            return gpu_clock_snapshot(self.dev_dir)
        except Exception as e:  # noqa: BLE001
            return {"error": repr(e)[:120]}

    def start(self):
        import threading
        self.before = self.snapshot()
        self._samples = []
        if self.dev_dir is None:
            return
        self._stop = threading.Event()

        def loop():
            while not self._stop.wait(self.period):
                self._samples.append(self.snapshot())
        self._thread = threading.Thread(target=loop, daemon=True)
        self._thread.start()

    def stop(self):
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=2)
            self._thread = None
        out = {"before": self.before, "after": self.snapshot()}
        during = {}
        for key in ("sclk_mhz", "mclk_mhz", "power_w", "temp_junction_c", "temp_edge_c", "temp_mem_c"):
            vals = [s[key] for s in self._samples if isinstance(s.get(key), (int, float))]
            if vals:
                during[key] = {"mean": round(sum(vals) / len(vals), 1), "min": min(vals), "max": max(vals)}
        if during:
            during["samples"] = len(self._samples)
            out["during"] = during
        return out


# ------------------------------------------------------------------ timing
def kernel_audit(step, device):
    """One extra UNTIMED step: which path every convolution took (exact: the route counters of
    ops/conv.py -- ``library_conv_calls`` > 0 means a convolution fell back to MIOpen), and how
    many GPU kernels torch.profiler saw.  The profiler count is a LOWER bound on ROCm: roctracer
    drops activity records (169-216 seen per ResNet-50 step against rocprofv3's 568,
    profiles/r5/audit_probe.md), so rocprofv3 is the kernel-count authority.  {} if disabled."""
    import torch
    if device.type != "cuda" or os.environ.get("CLOUDTIK_BENCH_AUDIT", "1") == "0":
        return {}
    from cloudtik_amd.ops import conv as CV
    before = dict(CV.ROUTES)
    out = {}
    try:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            step()
            torch.cuda.synchronize()
        names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
        naive = sorted({n for n in names if "naive" in n.lower()})
        out.update(kernels_seen_by_torch_profiler=len(names),
                   naive_conv_launches_seen=sum("naive" in n.lower() for n in names), naive_conv_kernels=naive[:8])
    except Exception as e:  # noqa: BLE001
        out["profiler_error"] = repr(e)[:200]
    out.update(igemm_conv_calls=CV.ROUTES["igemm"] - before["igemm"],
               library_conv_calls=CV.ROUTES["library"] - before["library"],
               kernel_count_authority="rocprofv3 --kernel-trace (torch.profiler undercounts on ROCm)")
    return out


def bucket_timeline(step, bucketer, device):
    """One extra UNTIMED step with the bucketer's trace on: when each gradient bucket's
    collective was issued relative to the end of backward (ms; negative = overlapped)."""
    import torch
    if bucketer is None or device.type != "cuda" or bucketer.world <= 1:
        return None
    bucketer.trace = True
    try:
        step()
        torch.cuda.synchronize()
        return [{"bucket": b, "bytes": n, "ms_vs_backward_end": t, "done_ms_vs_backward_end": d,
                 "host_wait_ms": w} for b, n, t, d, w in bucketer.timeline_full()]
    finally:
        bucketer.trace = False


def timed(step, args, rank, world, device, audit=False, bucketer=None):
    """W warm-up steps, then K timed steps between barrier+sync brackets.  Returns
    (max elapsed over ranks, per-rank elapsed list, last loss, per-step ms, audit).

    Per-step times come from HIP events recorded between the steps on the compute stream
    (no host synchronisation inside the timed loop); the headline is the host clock around
    all K steps."""
    import torch
    import torch.distributed as dist
    from cloudtik_amd.parallel import barrier

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()

    tw = time.perf_counter()
    for _ in range(args.warmup):
        step()
    sync()
    if rank == 0:
        print(f"[bench] warm-up {args.warmup} step(s): {time.perf_counter() - tw:.1f}s", file=sys.stderr)
    # nothing may sit between warm-up and the timed loop: the profiler-based kernel audit
    # runs AFTER the timed region (round 3: a torch.profiler session placed here left one
    # timed ResNet step blocked ~4.7 s on the host on a fresh box)
    barrier()
    sync()
    cuda = device.type == "cuda"
    events = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if cuda else []
    stamps = []
    tele = GpuTelemetry(device)
    tele.start()
    t0 = time.perf_counter()
    loss = None
    if cuda:
        events[0].record()
    host = []                       # host-side issue time of each step (no sync inside the loop)
    for i in range(args.steps):
        th = time.perf_counter()
        loss = step()
        if cuda:
            events[i + 1].record()
            host.append((time.perf_counter() - th) * 1e3)
        else:
            stamps.append(time.perf_counter())
    barrier()
    sync()
    el = time.perf_counter() - t0
    telemetry = tele.stop()
    if cuda:
        step_ms = [events[i].elapsed_time(events[i + 1]) for i in range(args.steps)]
    else:
        prev = [t0] + stamps[:-1]
        step_ms = [(b - a) * 1e3 for a, b in zip(prev, stamps)]
    per_rank = [el]
    if dist.is_initialized():
        t = torch.tensor([el], dtype=torch.float64, device=device)
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        per_rank = [float(o.item()) for o in out]
    info = {"gpu_telemetry": telemetry} if telemetry.get("before") or telemetry.get("after") else {}
    if host:
        # a host issue time close to the GPU step time means the step is launch / host bound
        # the fastest step's issue time is the host cost of a step whose launches never waited;
        # the mean also holds the steps that blocked on a full launch queue (the host ahead of
        # the GPU)
        info.update(host_issue_ms_mean=round(sum(host) / len(host), 3),
                    host_issue_ms_min=round(min(host), 3), host_ms=[round(h, 3) for h in host])
    if dist.is_initialized() and world > 1:
        # every rank's per-step GPU times (the max over ranks is the headline; a straggler
        # rank or step shows up here)
        t = torch.tensor(step_ms, dtype=torch.float64, device=device)
        outs = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        info["per_rank_step_ms"] = [[round(float(x), 3) for x in o.tolist()] for o in outs]
    loss_v = float(loss.detach().float().item())
    if audit:
        info.update(kernel_audit(step, device))
    tl = bucket_timeline(step, bucketer, device)
    if tl is not None:
        info["bucket_timeline"] = tl
    return max(per_rank), per_rank, loss_v, step_ms, info


def mean_ci(xs):
    """mean and 1.96 sigma (the reference protocol's ± band,
    imagenet-resnet50-synthetic-pytorch-distributed.py:194-210)."""
    import statistics
    if not xs:
        return None, None
    m = statistics.fmean(xs)
    return m, (1.96 * statistics.pstdev(xs) if len(xs) > 1 else 0.0)


def run_one(build, args, rank, world, device, kind):
    import gc
    import torch
    step, close, info = build(args, rank, world, device, kind)
    bucketer = info.pop("bucketer", None)
    prio = None
    if device.type == "cuda" and os.environ.get("CLOUDTIK_AMD_COMPUTE_PRIO", "0") == "1":
        # the step's own stream at the highest priority: the gradient side stream (and RCCL's
        # streams) keep the default one, so their workgroups yield CU slots to the critical path
        lo, hi = torch.cuda.Stream.priority_range()
        prio = torch.cuda.Stream(device=device, priority=min(lo, hi))
        prio.wait_stream(torch.cuda.current_stream())
    with (torch.cuda.stream(prio) if prio is not None else contextlib.nullcontext()):
        elapsed, per_rank, loss, step_ms, audit = timed(step, args, rank, world, device,
                                                        audit=info["unit"] == "images/s", bucketer=bucketer)
    if prio is not None:
        torch.cuda.current_stream().wait_stream(prio)
    del bucketer
    host_ms = audit.pop("host_issue_ms_mean", None) if audit else None
    info["host_issue_ms_min"] = audit.pop("host_issue_ms_min", None) if audit else None
    host_arr = audit.pop("host_ms", None) if audit else None
    info["per_rank_step_ms"] = audit.pop("per_rank_step_ms", None) if audit else None
    info["bucket_timeline"] = audit.pop("bucket_timeline", None) if audit else None
    info["gpu_telemetry"] = audit.pop("gpu_telemetry", None) if audit else None
    if audit and rank == 0:
        print(f"[bench] {info['model']} kernel audit (one untimed step): {json.dumps(audit)}", file=sys.stderr)
    plan = info.pop("plan", None)
    info["host_issue_ms"] = host_ms
    info["host_ms"] = host_arr
    close()
    del step
    gc.collect()
    if device.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    m, ci = mean_ci(step_ms)
    # per-step throughput of the whole job (reference: mean img/s ± 1.96 sigma)
    rates = [info["items_per_step"] * world / (t / 1e3) for t in step_ms if t > 0]
    rm, rci = mean_ci(rates)
    info.update(elapsed=elapsed, ms=elapsed / args.steps * 1e3,
                per_rank_ms=[round(e / args.steps * 1e3, 3) for e in per_rank],
                value=info["items_per_step"] * world * args.steps / elapsed, loss=loss,
                step_ms=[round(t, 3) for t in step_ms], step_ms_mean=round(m, 3) if m else None,
                step_ms_ci95=round(ci, 3) if ci is not None else None,
                rate_mean=round(rm, 2) if rm else None, rate_ci95=round(rci, 2) if rci is not None else None,
                audit=audit, plan=plan)
    return info


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist
    from cloudtik_amd.parallel import init_distributed
    backend = "gloo" if args.device == "cpu" else (None if args.dist_backend == "auto" else args.dist_backend)
    rank, world, local, device = init_distributed(backend=backend, gpu=args.device == "cuda")
    if args.device == "cpu":
        device = torch.device("cpu")
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.backends.cuda.matmul.allow_tf32 = False
    if args.impl == "native" or args.compare_eager:
        setup_tunableop(args.tunableop, rank)

    if args.model == "all":
        kinds = [("bert", "bert-large"), ("resnet", "resnet50")]
    elif args.model == "tiny":
        kinds = [("bert", "tiny"), ("resnet", "tiny")]
    elif args.model == "resnet50":
        kinds = [("resnet", "resnet50")]
    else:
        kinds = [("bert", args.model)]
    builders = {("bert", "native"): build_bert, ("resnet", "native"): build_resnet,
                ("bert", "eager"): build_bert_eager, ("resnet", "eager"): build_resnet_eager}
    results = []
    for fam, kind in kinds:
        r = run_one(builders[(fam, args.impl)], args, rank, world, device, kind)
        results.append(r)
    # the stock-PyTorch baseline AFTER every native half (the native numbers are taken on a
    # chip that has not yet run anything else); short unless --compare-eager
    base_steps = args.baseline_steps if args.baseline_steps >= 0 else (5 if world == 1 else 0)
    if args.impl == "native" and (args.compare_eager or base_steps > 0):
        import copy
        eargs = copy.copy(args)
        if not args.compare_eager:
            eargs.steps, eargs.warmup = base_steps, args.baseline_warmup
        for (fam, kind), r in zip(kinds, results):
            try:
                e = run_one(builders[(fam, "eager")], eargs, rank, world, device, kind)
                r["eager_value"], r["eager_ms"], r["eager_steps"] = e["value"], e["ms"], eargs.steps
            except Exception as ex:  # noqa: BLE001 - the baseline never costs the headline
                r["eager_error"] = repr(ex)[:300]
                if rank == 0:
                    print(f"[bench] eager baseline of {kind} failed: {ex!r}", file=sys.stderr)
                break

    envinfo = environment(device, world)
    if device.type == "cuda" and args.tunableop != "off":
        import torch.cuda.tunable as tn
        envinfo["tunableop"] = {"solutions": len(tn.get_results() or []), "file": tn.get_filename()}
    if rank == 0:
        print(f"[bench] environment: {json.dumps(envinfo)}", file=sys.stderr)
    n_dev = envinfo.get("distinct_devices") or (world if device.type == "cuda" else 0)
    if rank == 0:
        head = results[0]
        base = BASELINE.get(head["model"])
        cfg = {"model": head["model"], "global_batch": head["per_gpu_batch"] * world,
               "per_gpu_batch": head["per_gpu_batch"], "parallelism": f"dp{world}",
               "optimizer": head["optimizer"], "impl": head["impl"], "loss_last_step": round(head["loss"], 4),
               "grad_dtype": ("bf16 grads, " + ("fp32" if reduce_fp32(args, world) else "bf16") + " cross-rank sum"
                              if world > 1 else "bf16 (nothing reduced at world size 1)")
               if head["impl"] == "native" else "fp32 (autocast)",
               "zero1": bool(args.zero and world > 1)}
        if "hip_graph" in head:
            cfg["hip_graph"] = head["hip_graph"]
        if head["seq_len"]:
            cfg.update(seq_len=head["seq_len"], max_pred=head["max_pred"],
                       sentences_per_sec=round(head["value"] / head["seq_len"], 2))
        out = {"metric": head["metric"], "value": round(head["value"], 2), "unit": head["unit"],
               "n_gpus": n_dev, "world_size": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(head["ms"], 3), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": (round(head["value"] / base, 4) if base else
                               round(head["value"] / head["eager_value"], 4) if head.get("eager_value") else None),
               "baseline": (BASELINE_DESC if (not base and head.get("eager_value")) else None),
               "dtype": "bf16" if device.type == "cuda" else "fp32",
               "data": "synthetic (one resident random batch per rank, re-used every step; random-init weights)",
               "config": cfg,
               "world_size_seen_by_rccl": envinfo.get("world_size_seen_by_collective", 1)
               if (dist.is_initialized() and dist.get_backend() == "nccl") else (1 if world == 1 else None),
               "backend": dist.get_backend() if dist.is_initialized() else None,
               "per_rank_ms_per_step": head["per_rank_ms"],
               "step_ms_mean": head["step_ms_mean"], "step_ms_ci95": head["step_ms_ci95"],
               "value_mean_per_step": head["rate_mean"], "value_ci95": head["rate_ci95"],
               "bucket_plan": head["plan"],
               "host_issue_ms_per_step": head.get("host_issue_ms"),
               "host_issue_ms_min_per_step": head.get("host_issue_ms_min"),
               "step_ms": head["step_ms"], "host_ms": head.get("host_ms"),
               "per_rank_step_ms": head.get("per_rank_step_ms"), "bucket_timeline": head.get("bucket_timeline"),
               "gpu_telemetry": head.get("gpu_telemetry"),
               "env": {k: envinfo.get(k) for k in ("gpu", "rccl", "nccl_env", "rank0_cpus", "tunableop",
                                                   "distinct_devices", "world_size_seen_by_collective")
                       if envinfo.get(k) is not None},
               "miopen_db": (envinfo.get("miopen_db") or {}).get("mode") if (envinfo.get("miopen_db") or {}).get(
                   "installed") else "NOT INSTALLED"}
        if device.type == "cuda" and n_dev != world:
            out["note"] = f"{world} ranks shared {n_dev} GPU(s): plumbing check, not a scaling point"
        if "eager_value" in head:
            out["eager_value"] = round(head["eager_value"], 2)
            out["eager_ms_per_step"] = round(head["eager_ms"], 3)
            out["eager_steps"] = head["eager_steps"]
            out["speedup_vs_eager"] = round(head["value"] / head["eager_value"], 3)
        if "eager_error" in head:
            out["eager_error"] = head["eager_error"]
        for r in results[1:]:
            key = "resnet50" if r["model"].startswith("resnet") else r["model"].replace("-", "_")
            out[f"{key}_images_per_sec" if r["unit"] == "images/s" else f"{key}_value"] = round(r["value"], 2)
            out[f"{key}_ms_per_step"] = round(r["ms"], 3)
            out[f"{key}_per_gpu_batch"] = r["per_gpu_batch"]
            out[f"{key}_per_rank_ms_per_step"] = r["per_rank_ms"]
            out[f"{key}_loss_last_step"] = round(r["loss"], 4)
            out[f"{key}_step_ms_mean"], out[f"{key}_step_ms_ci95"] = r["step_ms_mean"], r["step_ms_ci95"]
            out[f"{key}_value_mean_per_step"], out[f"{key}_value_ci95"] = r["rate_mean"], r["rate_ci95"]
            out[f"{key}_bucket_plan"] = r["plan"]
            out[f"{key}_host_issue_ms_per_step"] = r.get("host_issue_ms")
            out[f"{key}_host_issue_ms_min_per_step"] = r.get("host_issue_ms_min")
            out[f"{key}_step_ms"], out[f"{key}_host_ms"] = r["step_ms"], r.get("host_ms")
            if r.get("per_rank_step_ms"):
                out[f"{key}_per_rank_step_ms"] = r["per_rank_step_ms"]
            if r.get("bucket_timeline"):
                out[f"{key}_bucket_timeline"] = r["bucket_timeline"]
            if r.get("gpu_telemetry"):
                out[f"{key}_gpu_telemetry"] = r["gpu_telemetry"]
            if "hip_graph" in r:
                out[f"{key}_hip_graph"] = r["hip_graph"]
            if r.get("audit"):
                out[f"{key}_kernel_audit"] = {k: v for k, v in r["audit"].items() if k != "naive_conv_kernels"}
            if "eager_value" in r:
                out[f"{key}_eager_value"] = round(r["eager_value"], 2)
                out[f"{key}_eager_ms_per_step"] = round(r["eager_ms"], 3)
                out[f"{key}_speedup_vs_eager"] = round(r["value"] / r["eager_value"], 3)
                out[f"{key}_vs_baseline"] = round(r["value"] / r["eager_value"], 4)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
