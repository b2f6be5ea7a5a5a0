#!/usr/bin/env python3
"""ResNet-50 training on an ImageNet-style folder -- the quickstart ResNet-50 workload
(reference: applications/ai/quickstart/bin/resnet50/train-distributed.sh ->
models/image_recognition/pytorch/common/main.py).

Reference recipe: torchvision resnet50, SGD (momentum 0.9, weight decay 1e-4), step LR decay
(x0.1 every 30 epochs), RandomResizedCrop(224) + flip for training, Resize(256) +
CenterCrop(224) for validation, top-1 / top-5 accuracy, checkpoint per epoch, DDP.  Here:
NHWC bf16 ResNet-50 with the fused BN(+add)+ReLU HIP kernels, fused SGD over a flat
parameter space with bucketed RCCL all-reduce, and the PIL process-pool + GPU ingest
pipeline of ``data/imagefolder.py``; one rank per GPU (``cloudtik-run`` / torchrun).

    python examples/ai/resnet50_train.py --data /data/imagenet --epochs 90 --batch 256 --lr 0.1 \\
        --ckpt-dir /ckpt/rn50
    python examples/ai/resnet50_train.py --make-folder 4x8 --data /tmp/tiny   # synthetic folder
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--data", required=True, help="root with train/ and val/ class folders")
    ap.add_argument("--make-folder", default="", help="CxN: write C classes x N random JPEGs per split and exit")
    ap.add_argument("--arch", default="resnet50", choices=["resnet50", "resnet34", "resnet101", "resnext50_32x4d"])
    ap.add_argument("--epochs", type=int, default=90)
    ap.add_argument("--max-steps", type=int, default=0)
    ap.add_argument("--batch", type=int, default=256, help="per-rank batch")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--lr", type=float, default=0.1, help="per 256 images (scaled by the global batch)")
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--weight-decay", type=float, default=1e-4)
    ap.add_argument("--lr-step-epochs", type=int, default=30)
    ap.add_argument("--warmup-epochs", type=int, default=0)
    ap.add_argument("--label-smoothing", type=float, default=0.0)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--ckpt-dir", default="")
    ap.add_argument("--log-every", type=int, default=50)
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args(argv)


def make_folder(root: str, spec: str, seed: int = 0):
    from PIL import Image
    classes, per = (int(v) for v in spec.lower().split("x"))
    rng = np.random.default_rng(seed)
    for split in ("train", "val"):
        for c in range(classes):
            d = os.path.join(root, split, f"n{c:08d}")
            os.makedirs(d, exist_ok=True)
            for i in range(per):
                h, w = int(rng.integers(160, 320)), int(rng.integers(160, 320))
                # class-dependent mean colour so a model can actually learn the toy task
                img = np.clip(rng.normal(40 + 60 * (c % 4), 30, (h, w, 3)), 0, 255).astype(np.uint8)
                Image.fromarray(img).save(os.path.join(d, f"{i:05d}.jpg"), quality=90)
    print(f"wrote {classes} classes x {per} images per split under {root}")


def main(argv=None):
    args = parse(argv)
    if args.make_folder:
        make_folder(args.data, args.make_folder, args.seed)
        return {}
    from cloudtik_amd.data.imagefolder import ImageFolderLoader, scan_image_folder
    from cloudtik_amd.models import resnet as R
    from cloudtik_amd.train.lr_scheduler import StepDecayScheduler
    from cloudtik_amd.train.optim import build_optimizer
    from cloudtik_amd.train.trainer import Trainer, setup_distributed

    rank, world, device = setup_distributed()
    torch.manual_seed(args.seed)
    train_samples, classes = scan_image_folder(os.path.join(args.data, "train"))
    val_dir = os.path.join(args.data, "val")
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    model = getattr(R, args.arch)(num_classes=len(classes), device=device, dtype=dtype)
    train = ImageFolderLoader(os.path.join(args.data, "train"), args.batch, train=True, image_size=args.image_size,
                              rank=rank, world=world, seed=args.seed, workers=args.workers, device=device,
                              samples=train_samples)
    val = ImageFolderLoader(val_dir, args.batch, train=False, image_size=args.image_size, rank=rank, world=world,
                            workers=args.workers, device=device, drop_last=False) if os.path.isdir(val_dir) else None
    lr = args.lr * args.batch * world / 256
    opt = build_optimizer("sgd", model, lr, args.weight_decay,
                          lambda n: n.endswith("bias") or ".bn" in n or n.startswith("bn"), momentum=args.momentum)
    steps_per_epoch = max(1, len(train))
    sched = StepDecayScheduler(opt, step_size=args.lr_step_epochs * steps_per_epoch, gamma=0.1,
                               warmup_steps=args.warmup_epochs * steps_per_epoch)

    def step(m, batch):
        x, y = batch
        logits = m(x).float()
        loss = F.cross_entropy(logits, y, label_smoothing=args.label_smoothing)
        top5 = logits.topk(min(5, logits.shape[1]), dim=1).indices
        hit = top5 == y[:, None]
        return loss, {"loss": loss.detach(), "top1": hit[:, 0].float().mean(), "top5": hit.any(1).float().mean()}

    trainer = Trainer(model, optimizer=opt, train_loader=train, eval_loader=val, step_fn=step, epochs=args.epochs,
                      max_steps=args.max_steps or None, lr_scheduler=sched, checkpoint_dir=args.ckpt_dir or None,
                      log_every=args.log_every)
    t0 = time.perf_counter()
    s0 = trainer.global_step
    hist = trainer.fit()
    if device.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    trainer.close()
    train.close()
    if val is not None:
        val.close()
    last = hist[-1] if hist else {}
    result = {"steps": trainer.global_step, "loss": last.get("loss"), "val_top1": last.get("eval_top1"),
              "val_top5": last.get("eval_top5"),
              "images_per_sec": round((trainer.global_step - s0) * args.batch * world / max(dt, 1e-9), 1)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    return result


if __name__ == "__main__":
    main()
