#!/usr/bin/env python3
"""ResNet-50 synthetic-data training benchmark, reference protocol
(examples/runtime/ai/basics/pytorch/imagenet-resnet50-synthetic-pytorch-distributed.py:15-24,
194-210 and its ``-horovod-run.py`` twin): ``--batch-size`` 32 per worker by default,
``--num-warmup-batches`` 10, then ``--num-iters`` x ``--num-batches-per-iter`` timed
batches; prints "Img/sec per device: mean +- 1.96 sigma" and the total over all devices.

MI355X path: NHWC bf16 ResNet-50 with fused BN(+add)+ReLU HIP kernels, fused SGD over a
flat parameter space, and either the built-in bucketed all-reduce (default) or the
Horovod-compatible DistributedOptimizer (``--horovod``, optional ``--fp16-allreduce`` /
``--use-adasum``), one process per GPU:

    cloudtik-run examples/ai/resnet50_synthetic.py --batch-size 256
    cloudtik-run --launcher horovod examples/ai/resnet50_synthetic.py --horovod
"""
import argparse
import os
import sys
import timeit

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def native_libraries():
    """The framework's native shared objects mapped into this process (/proc/self/maps)."""
    import cloudtik_amd
    root = os.path.dirname(os.path.dirname(os.path.abspath(cloudtik_amd.__file__)))
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.split()[-1] if len(line.split()) >= 6 else ""
                if path.endswith(".so") and "cloudtik_amd" in path and os.path.realpath(path).startswith(
                        os.path.realpath(root)):
                    out.add(os.path.relpath(os.path.realpath(path), os.path.realpath(root)))
    except OSError:
        pass
    return sorted(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--num-warmup-batches", type=int, default=10)
    ap.add_argument("--num-batches-per-iter", type=int, default=10)
    ap.add_argument("--num-iters", type=int, default=10)
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "small"])
    ap.add_argument("--horovod", action="store_true")
    ap.add_argument("--fp16-allreduce", action="store_true")
    ap.add_argument("--use-adasum", action="store_true")
    ap.add_argument("--report-json", default=None,
                    help="each rank writes <path>.rank<R>: its device binding, the native HIP libraries "
                         "mapped into the process, the last loss and its img/s (end-to-end checks)")
    args = ap.parse_args()

    from cloudtik_amd.models.resnet import resnet18_like_small, resnet50
    from cloudtik_amd.train.trainer import setup_distributed
    rank, world, device = setup_distributed()
    gpu = device.type == "cuda"
    torch.manual_seed(0)
    if args.model == "resnet50":
        model = resnet50(device=device, dtype=torch.bfloat16 if gpu else torch.float32)
        shape, classes = (3, 224, 224), 1000
    else:
        model = resnet18_like_small(num_classes=10, device=device)
        shape, classes = (3, 32, 32), 10
    dtype = next(model.parameters()).dtype
    data = torch.randn(args.batch_size, *shape, device=device, dtype=dtype).contiguous(
        memory_format=torch.channels_last)
    target = torch.randint(0, classes, (args.batch_size,), device=device)

    if args.horovod:
        import cloudtik_amd.parallel.horovod as hvd
        hvd.init()
        lr_scaler = hvd.size() if not args.use_adasum else 1
        opt = torch.optim.SGD(model.parameters(), lr=0.01 * lr_scaler, momentum=0.9)
        compression = hvd.Compression.bf16 if args.fp16_allreduce else hvd.Compression.none
        opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=compression,
                                       op=hvd.Adasum if args.use_adasum else hvd.Average)
        hvd.broadcast_parameters(model.state_dict(), root_rank=0)
        hvd.broadcast_optimizer_state(opt, root_rank=0)

        def step():
            opt.zero_grad()
            F.cross_entropy(model(data).float(), target).backward()
            opt.step()
    else:
        from cloudtik_amd.models.resnet import ResNetTrainStep
        from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
        from cloudtik_amd.train.optim import FlatParamSpace, FusedSGD
        named = list(model.named_parameters())
        space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
        opt = FusedSGD(space, lr=0.01, momentum=0.9, weight_decay=1e-4)
        broadcast_flat_params(space)
        ddp = GradBucketer(space, bucket_mb=25)
        opt.grad_scale = ddp.grad_scale
        ts = ResNetTrainStep(model, opt, ddp)

        def step():
            return ts(data, target)

    def log(s):
        if rank == 0:
            print(s, flush=True)

    last = {}

    def benchmark_step():
        last["loss"] = step()
        if gpu:
            torch.cuda.synchronize()

    log(f"Model: {args.model}  Batch size: {args.batch_size}  Number of {'GPU' if gpu else 'CPU'}s: {world}")
    log("Running warmup...")
    timeit.timeit(benchmark_step, number=args.num_warmup_batches)
    log("Running benchmark...")
    img_secs = []
    for x in range(args.num_iters):
        t = timeit.timeit(benchmark_step, number=args.num_batches_per_iter)
        img_sec = args.batch_size * args.num_batches_per_iter / t
        log(f"Iter #{x}: {img_sec:.1f} img/sec per {'GPU' if gpu else 'CPU'}")
        img_secs.append(img_sec)
    mean, conf = np.mean(img_secs), 1.96 * np.std(img_secs)
    log(f"Img/sec per {'GPU' if gpu else 'CPU'}: {mean:.1f} +-{conf:.1f}")
    log(f"Total img/sec on {world} {'GPU' if gpu else 'CPU'}(s): {world * mean:.1f} +-{world * conf:.1f}")
    if args.report_json:
        import json
        loss = last.get("loss")
        with open(f"{args.report_json}.rank{rank}", "w") as f:
            json.dump({"rank": rank, "world": world, "local_rank": int(os.environ.get("LOCAL_RANK", 0)),
                       "device": str(device), "device_name": torch.cuda.get_device_name(device) if gpu else None,
                       "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES"),
                       "native_libraries": native_libraries(), "img_per_sec": float(mean),
                       "loss": float(loss.detach().float()) if torch.is_tensor(loss) else None}, f)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
