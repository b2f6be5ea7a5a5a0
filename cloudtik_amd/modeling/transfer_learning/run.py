"""``ai.modeling.transfer_learning``: fine-tune an image or text classifier and export it
(reference transfer-learning workflow scripts; distributed with ``cloudtik-run -np N``)."""
from __future__ import annotations

import argparse
import json
import os
import sys


def parse_args(argv=None):
    ap = argparse.ArgumentParser("ai.modeling.transfer_learning", description=__doc__)
    a = ap.add_argument
    a("--framework", default="pytorch")
    a("--use-case", "--use_case", default="image_classification",
      choices=["image_classification", "text_classification"])
    a("--model", "--model-name", "--model_name", dest="model", default="resnet50")
    a("--dataset-dir", "--dataset_dir", help="image folder root (class sub-directories)")
    a("--dataset-file", "--dataset_file", help="CSV with text and label columns")
    a("--text-col", "--text_col", default="text")
    a("--label-col", "--label_col", default="label")
    a("--synthetic", type=int, default=0, help="use N synthetic samples")
    a("--num-classes", "--num_classes", type=int, default=0)
    a("--image-size", "--image_size", type=int, default=224)
    a("--max-seq-length", "--max_seq_length", type=int, default=128)
    a("--pretrained", default=None, help="local safetensors / torch weights")
    a("--no-freeze", "--no_freeze", action="store_true", help="fine-tune the whole backbone")
    a("--epochs", type=int, default=1)
    a("--batch-size", "--batch_size", type=int, default=32)
    a("--lr", "--learning-rate", type=float, default=None)
    a("--val-split", "--val_split", type=float, default=0.1)
    a("--output-dir", "--output_dir", default="./output")
    a("--max-steps", "--max_steps", type=int, default=None)
    a("--device", default=None)
    return ap.parse_args(argv)


def run(args):
    import torch
    from torch.utils.data import random_split
    from cloudtik_amd.modeling.transfer_learning import (HashTokenizer, ImageFolderDataset,
                                                         TextClassificationDataset, get_model,
                                                         synthetic_image_dataset)
    from cloudtik_amd.train.trainer import setup_distributed
    rank, _, _ = setup_distributed()
    if args.use_case == "image_classification":
        if args.dataset_dir:
            ds = ImageFolderDataset(args.dataset_dir, args.image_size)
        else:
            ds = synthetic_image_dataset(args.synthetic or 256, args.num_classes or 4, args.image_size)
        kw = {"freeze_backbone": not args.no_freeze}
        lr = args.lr or 1e-3
    else:
        tok = HashTokenizer(max_length=args.max_seq_length)
        if not args.dataset_file:
            raise SystemExit("--dataset-file is required for text classification")
        ds = TextClassificationDataset.from_csv(args.dataset_file, args.text_col, args.label_col, tok)
        kw = {}
        lr = args.lr or 2e-5
    classes = getattr(ds, "classes", None)
    n_cls = args.num_classes or len(classes)
    n_val = int(len(ds) * args.val_split)
    gen = torch.Generator().manual_seed(0)
    train_ds, val_ds = random_split(ds, [len(ds) - n_val, n_val], generator=gen) if n_val else (ds, None)
    model = get_model(args.model, args.framework, args.use_case, num_classes=n_cls, pretrained_path=args.pretrained,
                      device=args.device, classes=classes, **kw)
    hist = model.train(train_ds, epochs=args.epochs, batch_size=args.batch_size, lr=lr, eval_dataset=val_ds,
                       max_steps=args.max_steps, log_every=0)
    result = {"history": hist}
    if rank == 0:
        result["export"] = model.export(args.output_dir)
        print(json.dumps(result, default=float), flush=True)
    return result


def main(argv=None):
    return run(parse_args(argv))


if __name__ == "__main__":
    sys.exit(0 if main() is not None else 1)
