#!/usr/bin/env python3
"""Mask R-CNN / Faster R-CNN training and COCO box-AP evaluation on COCO-format data -- the
quickstart Mask R-CNN workload (reference: applications/ai/quickstart/bin/maskrcnn/* ->
maskrcnn_benchmark tools/train_net.py with the e2e_mask_rcnn_R_50_FPN_1x config; SURVEY.md
§2.12).

Reference recipe (1x schedule): SGD momentum 0.9, weight decay 1e-4, base LR 0.02 for 16
images (scaled linearly with the global batch), linear warm-up over 500 iterations from 1/3,
x0.1 at 60k and 80k of 90k iterations, shorter side 800 / longer side <= 1333, horizontal
flip.  Here: NHWC bf16 ResNet-50-FPN with the HIP detection ops (segmented NMS, multi-level
NHWC ROIAlign, fixed-size sync-free RoI sampling), fused SGD + bucketed RCCL all-reduce,
COCO JSON + PIL process-pool loader (``data/coco.py``), one rank per GPU.

    python examples/ai/maskrcnn_train.py --make-coco 16 --coco-root /tmp/coco   # synthetic set
    cloudtik-run --nproc_per_node 8 examples/ai/maskrcnn_train.py --coco-root /data/coco \\
        --train-ann annotations/instances_train2017.json --train-images train2017 \\
        --val-ann annotations/instances_val2017.json --val-images val2017 --batch 2
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


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--coco-root", required=True)
    ap.add_argument("--train-ann", default="annotations/instances_train.json")
    ap.add_argument("--train-images", default="train")
    ap.add_argument("--val-ann", default="annotations/instances_val.json")
    ap.add_argument("--val-images", default="val")
    ap.add_argument("--make-coco", type=int, default=0, help="write N synthetic images per split and exit")
    ap.add_argument("--model", default="maskrcnn", choices=["maskrcnn", "fasterrcnn"])
    ap.add_argument("--batch", type=int, default=2, help="images per rank")
    ap.add_argument("--min-size", type=int, default=800)
    ap.add_argument("--max-size", type=int, default=1333)
    ap.add_argument("--lr", type=float, default=0.02, help="for 16 images (scaled by the global batch)")
    ap.add_argument("--max-iter", type=int, default=90000)
    ap.add_argument("--steps", type=int, nargs="*", default=[60000, 80000])
    ap.add_argument("--warmup-iters", type=int, default=500)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--no-fixed-canvas", action="store_true",
                    help="pad each batch to its own size instead of one canvas per orientation")
    ap.add_argument("--ckpt-dir", default="")
    ap.add_argument("--ckpt-every", type=int, default=2500)
    ap.add_argument("--log-every", type=int, default=20)
    ap.add_argument("--eval-only", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args(argv)


def make_coco(root: str, n: int, seed: int = 0):
    """Synthetic COCO-format split pair: coloured rectangles / triangles with polygon outlines."""
    from PIL import Image, ImageDraw
    rng = np.random.default_rng(seed)
    cats = [{"id": 3, "name": "rect"}, {"id": 7, "name": "tri"}]
    for split in ("train", "val"):
        os.makedirs(os.path.join(root, split), exist_ok=True)
        images, anns = [], []
        for i in range(n):
            w, h = int(rng.integers(320, 480)), int(rng.integers(240, 400))
            im = Image.fromarray(rng.integers(0, 60, (h, w, 3), dtype=np.uint8))
            d = ImageDraw.Draw(im)
            for _ in range(int(rng.integers(1, 4))):
                bw, bh = int(rng.integers(40, w // 2)), int(rng.integers(40, h // 2))
                x, y = int(rng.integers(0, w - bw)), int(rng.integers(0, h - bh))
                if rng.random() < 0.5:
                    poly, cat, col = [x, y, x + bw, y, x + bw, y + bh, x, y + bh], 3, (220, 40, 40)
                else:
                    poly, cat, col = [x, y + bh, x + bw // 2, y, x + bw, y + bh], 7, (40, 220, 40)
                d.polygon([(poly[j], poly[j + 1]) for j in range(0, len(poly), 2)], fill=col)
                anns.append({"id": len(anns) + 1, "image_id": i + 1, "category_id": cat, "iscrowd": 0,
                             "bbox": [x, y, bw, bh], "area": float(bw * bh), "segmentation": [poly]})
            fn = f"{i:06d}.jpg"
            im.save(os.path.join(root, split, fn), quality=92)
            images.append({"id": i + 1, "file_name": fn, "width": w, "height": h})
        os.makedirs(os.path.join(root, "annotations"), exist_ok=True)
        with open(os.path.join(root, "annotations", f"instances_{split}.json"), "w") as f:
            json.dump({"images": images, "annotations": anns, "categories": cats}, f)
    print(f"wrote {n} images per split under {root}")


@torch.no_grad()
def evaluate(model, loader, ds, rank, world, device):
    """COCO box AP over the validation split (detections gathered to every rank)."""
    from cloudtik_amd.data.coco import evaluate_bbox
    model.eval()
    dets = {}
    for imgs, _, sizes, ids, scales in loader:
        out = model(imgs, image_sizes=sizes)
        for r, iid, s in zip(out, ids, scales):
            dets[int(iid)] = {"boxes": (r["boxes"].float() / s).cpu().numpy(), "scores": r["scores"].float().cpu().numpy(),
                              "labels": r["labels"].cpu().numpy()}
    if world > 1:
        import torch.distributed as dist
        parts = [None] * world
        dist.all_gather_object(parts, dets)
        dets = {k: v for p in parts for k, v in p.items()}
    model.train()
    return evaluate_bbox(dets, ds.ground_truth())


def main(argv=None):
    args = parse(argv)
    if args.make_coco:
        make_coco(args.coco_root, args.make_coco, args.seed)
        return {}
    from cloudtik_amd.data.coco import CocoDetection, CocoLoader
    from cloudtik_amd.models.detection import faster_rcnn_resnet50_fpn, mask_rcnn_resnet50_fpn
    from cloudtik_amd.train.lr_scheduler import WarmupMultiStepScheduler
    from cloudtik_amd.train.optim import build_optimizer
    from cloudtik_amd.train.trainer import Trainer, setup_distributed

    rank, world, device = setup_distributed()
    import logging
    logging.basicConfig(level=logging.INFO if rank == 0 else logging.WARNING, format="%(asctime)s %(message)s")
    torch.manual_seed(args.seed)
    with_masks = args.model == "maskrcnn"
    root = args.coco_root
    train_ds = CocoDetection(os.path.join(root, args.train_images), os.path.join(root, args.train_ann), train=True,
                             with_masks=with_masks)
    val_ds = CocoDetection(os.path.join(root, args.val_images), os.path.join(root, args.val_ann), train=False,
                           with_masks=False)
    build = mask_rcnn_resnet50_fpn if with_masks else faster_rcnn_resnet50_fpn
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    model = build(train_ds.num_classes, device=device, dtype=dtype)
    train = CocoLoader(train_ds, args.batch, args.min_size, args.max_size, rank=rank, world=world, seed=args.seed,
                       workers=args.workers, device=device, fixed_canvas=not args.no_fixed_canvas)
    val = CocoLoader(val_ds, args.batch, args.min_size, args.max_size, rank=rank, world=world, workers=args.workers,
                     device=device, drop_last=False, fixed_canvas=not args.no_fixed_canvas)
    result = {}
    if not args.eval_only:
        lr = args.lr * args.batch * world / 16
        opt = build_optimizer("sgd", model, lr, 1e-4, lambda n: n.endswith("bias") or ".bn" in n, momentum=0.9)
        sched = WarmupMultiStepScheduler(opt, args.steps, 0.1, 1.0 / 3, args.warmup_iters)

        def step(m, batch):
            imgs, targets, sizes, _, _ = batch
            losses = m(imgs, targets, sizes)
            loss = sum(losses.values())
            return loss, {k: v.detach().float() for k, v in losses.items()}

        epochs = -(-args.max_iter // max(1, len(train)))
        trainer = Trainer(model, optimizer=opt, train_loader=train, step_fn=step, epochs=epochs,
                          max_steps=args.max_iter, lr_scheduler=sched, checkpoint_dir=args.ckpt_dir or None,
                          checkpoint_every=args.ckpt_every, log_every=args.log_every)
        t0, s0 = time.perf_counter(), trainer.global_step
        hist = trainer.fit()
        if device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        trainer.close()
        result.update(steps=trainer.global_step, images_per_sec=round(
            (trainer.global_step - s0) * args.batch * world / max(dt, 1e-9), 2),
            losses={k: v for k, v in (hist[-1] if hist else {}).items() if k.startswith("loss")})
    result["bbox"] = evaluate(model, val, val_ds, rank, world, device)
    train.close()
    val.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    return result


if __name__ == "__main__":
    main()
