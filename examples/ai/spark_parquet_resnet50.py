#!/usr/bin/env python3
"""Spark + AI runtime pipeline (north-star config 5): ETL writes ImageNet-shaped Parquet, then
ResNet-50 trains from it with the pinned-memory hipMemcpyAsync loader, one rank per GPU.

    # ETL + training on every GPU of the node
    cloudtik-run examples/ai/spark_parquet_resnet50.py --data-path /data/imagenet_parquet
    # or on a cluster: cloudtik submit cluster.yaml examples/ai/spark_parquet_resnet50.py ...

Stage 1 (rank 0, skipped when the part files exist): Spark (if pyspark is installed) or a
pyarrow process pool writes ``--parts`` Parquet files of uint8 224x224x3 images + labels
(synthetic content; no dataset can be downloaded here).  Stage 2: every rank reads its own
part files (ParquetImageLoader: row groups streamed with bounded host memory -> pinned
slots -> side-stream async H2D of uint8 -> fused normalise/flip kernel -> bf16
channels-last; ``--resident`` loads the parts into RAM for the native loader instead), and trains ResNet-50 with fused SGD
and bucketed RCCL all-reduce.  Prints one JSON line with images/s of the whole job and the
pipeline efficiency (throughput relative to the same steps on one GPU-resident batch).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data-path", default="/tmp/cloudtik_imagenet_parquet")
    ap.add_argument("--rows", type=int, default=0, help="total rows to generate (default 16 batches per rank)")
    ap.add_argument("--parts", type=int, default=0, help="part files (default 4 per rank)")
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "small"])
    ap.add_argument("--etl-engine", default="auto", choices=["auto", "spark", "pyarrow"])
    ap.add_argument("--resident", action="store_true",
                    help="load the rank's parts into host RAM first (default: stream row groups)")
    ap.add_argument("--window", type=int, default=4, help="streaming shuffle window (row groups)")
    ap.add_argument("--workers", type=int, default=4, help="row-group decode threads")
    args = ap.parse_args()

    from cloudtik_amd.data.pipeline import ParquetImageLoader, rank_parts, write_image_shards
    from cloudtik_amd.models.resnet import ResNetTrainStep, resnet18_like_small, resnet50
    from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
    from cloudtik_amd.train.optim import FlatParamSpace, FusedSGD
    from cloudtik_amd.train.trainer import setup_distributed

    rank, world, device = setup_distributed()
    gpu = device.type == "cuda"
    parts = args.parts or 4 * world
    rows = args.rows or 16 * args.batch_size * world
    t0 = time.time()
    etl_s = 0.0
    if rank == 0 and len([f for f in os.listdir(args.data_path)] if os.path.isdir(args.data_path) else []) < parts:
        write_image_shards(args.data_path, rows, parts, args.image_size, 1000 if args.model == "resnet50" else 10,
                           engine=args.etl_engine)
        etl_s = time.time() - t0
    if world > 1:
        dist.barrier()

    loader = ParquetImageLoader(rank_parts(args.data_path, rank, world), args.batch_size, args.image_size,
                                seed=rank, device=device, streaming=not args.resident, window=args.window,
                                num_workers=args.workers)
    if args.model == "resnet50":
        model = resnet50(device=device, dtype=torch.bfloat16 if gpu else torch.float32)
    else:
        model = resnet18_like_small(num_classes=10, device=device)
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = FusedSGD(space, lr=0.01, momentum=0.9, weight_decay=1e-4)
    broadcast_flat_params(space)
    ddp = GradBucketer(space, bucket_mb=25)
    opt.grad_scale = ddp.grad_scale
    step = ResNetTrainStep(model, opt, ddp)
    dtype = next(model.parameters()).dtype

    def sync():
        if gpu:
            torch.cuda.synchronize()

    # pipeline throughput: loader -> ingest kernel -> train step, no per-step host syncs so
    # the side-stream copies overlap the previous step's compute
    n_img, steps, t_start, loss = 0, 0, None, None
    for epoch in range(args.epochs):
        loader.set_epoch(epoch)
        for x, y in loader:
            if steps == args.warmup:
                sync()
                t_start = time.time()
            loss = step(x.to(dtype), y)
            steps += 1
            if t_start is not None:
                n_img += x.shape[0]
    sync()
    pipe_s = time.time() - t_start if t_start else 0.0
    # the same steps on one resident batch: the ceiling the input pipeline is measured against
    x_res, y_res = x.to(dtype).clone(), y.clone()
    n_res = max(1, min(20, steps - args.warmup))
    sync()
    t1 = time.time()
    for _ in range(n_res):
        step(x_res, y_res)
    sync()
    res_s = (time.time() - t1) / n_res
    stats = torch.tensor([n_img, pipe_s, res_s], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(stats)
    if rank == 0:
        n_img, pipe_s, res_s = stats.tolist()
        pipe_s, res_s = pipe_s / world, res_s / world
        ips = n_img / pipe_s if pipe_s else None
        resident_ips = args.batch_size * world / res_s
        print(json.dumps({"metric": "resnet50_parquet_pipeline_images_per_sec", "model": args.model,
                          "value": round(ips, 1) if ips else None, "resident_batch_images_per_sec": round(resident_ips, 1),
                          "pipeline_efficiency": round(ips / resident_ips, 4) if ips else None, "n_gpus": world,
                          "batch_per_gpu": args.batch_size, "etl_seconds": round(etl_s, 2), "rows": rows,
                          "parts": parts, "final_loss": float(loss.detach()), "data": "synthetic parquet",
                          "loader": "resident" if args.resident else "streaming"}), flush=True)
    loader.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
