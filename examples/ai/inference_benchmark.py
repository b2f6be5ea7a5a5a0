#!/usr/bin/env python3
"""Inference (and detection-training) throughput of the reference's quickstart workloads on
MI355X (ResNet50v1.5 / ResNeXt101-32x16d classification, Faster / Mask
R-CNN and RetinaNet, SSD-ResNet34 and SSD-MobileNet, YOLOv4 inference; Mask R-CNN and
SSD-ResNet34 training).

Protocol of the quickstart ``--benchmark`` runs: W untimed warm-up batches, then K timed
batches bracketed by ``torch.cuda.synchronize()``; prints one JSON line per model with
images/s.  bf16 weights/activations (NHWC), random-init weights, synthetic images.
Detection inference includes the post-processing (decode + HIP NMS, masks).

    python examples/ai/inference_benchmark.py --models resnet50,maskrcnn --batch 32
    python examples/ai/inference_benchmark.py --models maskrcnn --train --batch 4
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402

MODELS = {
    # name: (input size, default batch)
    "resnet50": (224, 128),
    "resnext101_32x16d": (224, 64),
    "maskrcnn": (800, 4),
    "fasterrcnn": (800, 4),
    "retinanet": (800, 4),
    "ssd_resnet34": (1200, 8),
    "ssd_resnet34_300": (300, 32),
    "ssd_mobilenet": (300, 64),
    "yolov4": (608, 16),
    "rnnt": (0, 32),            # MLPerf RNN-T, 400 feature frames, 60 labels
    "t5_base": (0, 16),         # T5-base, 128 source tokens, 32 generated
    "transnetv2": (0, 8),       # 100-frame 48x27 windows
}


def build(name, dev, num_classes=81):
    from cloudtik_amd.models import resnet as R
    from cloudtik_amd.models import detection as D
    from cloudtik_amd.models.detection.retinanet import retinanet_resnet50_fpn
    from cloudtik_amd.models.detection.ssd import ssd300_mobilenet_v1, ssd300_resnet34
    from cloudtik_amd.models.detection.yolo import yolov4
    if name == "resnet50":
        return R.resnet50(device=dev)
    if name == "resnext101_32x16d":
        return R.resnext101_32x16d(device=dev)
    if name == "maskrcnn":
        return D.mask_rcnn_resnet50_fpn(num_classes, device=dev)
    if name == "fasterrcnn":
        return D.faster_rcnn_resnet50_fpn(num_classes, device=dev)
    if name == "retinanet":
        return retinanet_resnet50_fpn(num_classes - 1, device=dev)
    if name.startswith("ssd_resnet34"):
        return ssd300_resnet34(num_classes, device=dev)
    if name == "ssd_mobilenet":
        return ssd300_mobilenet_v1(91, device=dev)
    if name == "yolov4":
        return yolov4(80, device=dev)
    if name == "rnnt":
        from cloudtik_amd.models.rnnt import rnnt_mlperf
        m = rnnt_mlperf(device=dev)
        with torch.no_grad():
            # random init argmaxes to a non-blank label almost every joint step (blank is 1
            # of 29 classes); a trained transducer mostly predicts blank.  Bias the blank
            # logit so greedy decoding emits at a speech-like rate instead of 30 labels per frame.
            m.joint_out.bias[m.cfg.blank] += 6.0
        return m
    if name == "t5_base":
        from cloudtik_amd.models.t5 import T5Config, T5ForConditionalGeneration
        return T5ForConditionalGeneration(T5Config.base(), device=dev)
    if name == "transnetv2":
        from cloudtik_amd.models.transnetv2 import TransNetV2
        return TransNetV2(device=dev)
    raise ValueError(name)


def infer_fn(name, model, size):
    if name in ("resnet50", "resnext101_32x16d", "maskrcnn", "fasterrcnn", "retinanet"):
        return model
    if name.startswith("ssd"):
        def f(x):
            loc, conf = model(x)
            return model.postprocess(loc, conf, size)
        return f
    if name == "yolov4":
        return lambda x: model.postprocess(model(x), (size, size))
    if name == "rnnt":
        return lambda x: model.greedy_decode(*x)
    if name == "t5_base":
        return lambda x: model.generate(x, max_new_tokens=32)
    if name == "transnetv2":
        return model.predict_transitions
    raise ValueError(name)


def make_input(name, batch, size, dev):
    """Synthetic input of the model's shape (images unless the model says otherwise)."""
    if name == "rnnt":
        from cloudtik_amd.models.rnnt import synthetic_speech_batch
        f, fl, _, _ = synthetic_speech_batch(batch, T=400, U=60, device=dev)
        return f, fl
    if name == "t5_base":
        return torch.randint(2, 32128, (batch, 128), device=dev)
    if name == "transnetv2":
        return torch.randint(0, 256, (batch, 100, 27, 48, 3), dtype=torch.uint8, device=dev)
    return torch.randn(batch, 3, size, size, device=dev)


def run(name, args, dev):
    size, batch = MODELS[name]
    size = args.size or size
    batch = args.batch or batch
    torch.manual_seed(0)
    model = build(name, dev)
    x = make_input(name, batch, size, dev)
    if name in ("resnet50", "resnext101_32x16d"):
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    if args.train:
        from cloudtik_amd.models.detection import synthetic_detection_batch
        from cloudtik_amd.train.optim import build_optimizer
        model.train()
        opt = build_optimizer("sgd", model, 0.01, 1e-4, momentum=0.9)
        if name == "rnnt":
            from cloudtik_amd.models.rnnt import synthetic_speech_batch
            sb = synthetic_speech_batch(batch, T=400, U=60, device=dev)

            def step():
                loss = model(*sb)
                loss.backward()
                opt.step()
                opt.zero_grad()
        elif name == "t5_base":
            y = torch.randint(2, 32128, (batch, 32), device=dev)

            def step():
                loss = model(x, y)
                loss.backward()
                opt.step()
                opt.zero_grad()
        elif name in ("resnet50", "resnext101_32x16d"):
            y = torch.randint(0, 1000, (batch,), device=dev)

            def step():
                loss = torch.nn.functional.cross_entropy(model(x).float(), y)
                loss.backward()
                opt.step()
                opt.zero_grad()
        else:
            imgs, tg = synthetic_detection_batch(batch, size, 81, 8, with_masks=(name == "maskrcnn"), device=dev)

            def step():
                out = model(imgs, tg)
                loss = sum(out.values())
                loss.backward()
                opt.step()
                opt.zero_grad()
    else:
        model.eval()
        f = infer_fn(name, model, size)

        def step():
            with torch.no_grad():
                return f(x)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    unit = {"rnnt": "utterances_per_sec", "t5_base": "sequences_per_sec",
            "transnetv2": "windows_per_sec"}.get(name, "images_per_sec")
    out = {"model": name, "mode": "train" if args.train else "inference", "batch": batch, "size": size,
           unit: round(batch * args.steps / dt, 2), "ms_per_batch": round(dt / args.steps * 1000, 3),
           "dtype": "bf16", "data": "synthetic, random-init weights"}
    print(json.dumps(out), flush=True)
    del model
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,resnext101_32x16d,maskrcnn,retinanet,ssd_resnet34_300,"
                                        "ssd_mobilenet,yolov4")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--size", type=int, default=0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--train", action="store_true")
    ap.add_argument("--conv-benchmark", action="store_true")
    args = ap.parse_args()
    if args.conv_benchmark:
        torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    for name in args.models.split(","):
        run(name.strip(), args, dev)


if __name__ == "__main__":
    main()
