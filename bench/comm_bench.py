#!/usr/bin/env python3
"""Collective microbenchmark: RCCL all-reduce / reduce-scatter / all-gather bus bandwidth over
xGMI, plus the one-shot P2P all-reduce kernel (parallel/p2p.py), and the gradient-bucket size
the two curves imply.

Why: the data-parallel step hands its gradients to RCCL in buckets (parallel/ddp.py;
bench.py --bucket-mb / --rn-bucket-mb).  On one MI355X node every GPU has 7 point-to-point
xGMI links, so a ring collective is per-link bound and only reaches its plateau above some
message size; below it the latency terms (2 (n-1) steps) dominate and the one-shot P2P kernel
(every peer read at once) wins.  The bucket size should sit at the knee of the RCCL curve, and
the P2P path should take every bucket below the crossover.  This script measures both on the
node instead of assuming them (reference: DDP bucket_cap_mb=8192 for BERT,
run_pretrain_mlperf.py:688-691; 25 MB default buckets for ResNet).

Launch (one process per GPU, like bench.py):
    python bench/comm_bench.py --gpus 8                     # spawns 8 ranks itself
    torchrun --nproc-per-node 8 bench/comm_bench.py ...     # or ranks from the environment
    python bench/comm_bench.py --device cpu --gpus 2        # gloo plumbing check (CPU)

Bus bandwidth follows the nccl-tests convention: algbw = bytes / t; busbw = algbw x
2 (n-1)/n for all-reduce, x (n-1)/n for reduce-scatter and all-gather (bytes = the full
buffer).  At n = 1 there is no traffic; the table still runs end to end (latency floor).
Rank 0 prints one markdown table on stderr and one JSON line on stdout.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

MiB = 1 << 20


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--min-bytes", type=int, default=1 * MiB)
    ap.add_argument("--max-bytes", type=int, default=256 * MiB)
    ap.add_argument("--p2p-min-bytes", type=int, default=16 << 10,
                    help="smallest size of the small-message sweep (P2P vs RCCL all-reduce)")
    ap.add_argument("--p2p-max-bytes", type=int, default=4 * MiB,
                    help="largest message the one-shot P2P kernel takes (its staging buffer)")
    ap.add_argument("--dtypes", default="bf16,fp32")
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-p2p", action="store_true")
    ap.add_argument("--write-tuning", nargs="?", const="", default=None, metavar="PATH",
                    help="store the recommended bucket and P2P crossover for this world size in the "
                         "tuning file the data-parallel path reads (parallel/comm_tuning.py; default "
                         "path when given without a value)")
    ap.add_argument("--plateau", type=float, default=0.8,
                    help="recommended bucket = smallest size reaching this fraction of the peak busbw")
    return ap.parse_args(argv)


def sizes(lo, hi):
    out, s = [], lo
    while s <= hi:
        out.append(s)
        s *= 2
    return out


def spawn(n: int) -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        rc = rc or c
    return rc


def bus_factor(op: str, n: int) -> float:
    if n <= 1:
        return 0.0
    return 2.0 * (n - 1) / n if op == "all_reduce" else (n - 1) / n


def recommend_bucket(rows, plateau: float):
    """Smallest message size whose all-reduce busbw reaches ``plateau`` x the peak of the
    sweep (None when there is no traffic, n = 1)."""
    ar = sorted((r for r in rows if r["op"] == "all_reduce" and r["busbw_gbs"] > 0), key=lambda r: r["bytes"])
    if not ar:
        return None
    peak = max(r["busbw_gbs"] for r in ar)
    for r in ar:
        if r["busbw_gbs"] >= plateau * peak:
            return r["bytes"]
    return ar[-1]["bytes"]


def crossover(small):
    """Largest size at which the P2P one-shot all-reduce still beats RCCL (None if never)."""
    best = None
    for r in sorted(small, key=lambda r: r["bytes"]):
        if r.get("p2p_us") is not None and r["p2p_us"] < r["rccl_us"]:
            best = r["bytes"]
    return best


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args.gpus))

    import torch
    import torch.distributed as dist
    from cloudtik_amd.parallel import barrier, init_distributed

    cuda = args.device == "cuda"
    rank, world, local, device = init_distributed(backend=None if cuda else "gloo", gpu=cuda)
    if not cuda:
        device = torch.device("cpu")
    if not dist.is_initialized():
        # one rank: still a real (1-member) RCCL / gloo communicator, so the table measures the
        # collective's launch + copy floor end to end
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        kw = {"device_id": device} if cuda else {}
        dist.init_process_group("nccl" if cuda else "gloo", init_method=f"tcp://127.0.0.1:{port}",
                                rank=0, world_size=1, **kw)
    dts = {"bf16": torch.bfloat16, "fp32": torch.float32}

    def sync():
        if cuda:
            torch.cuda.synchronize()

    def timeit(fn, iters, warmup):
        for _ in range(warmup):
            fn()
        sync()
        barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        sync()
        el = (time.perf_counter() - t0) / iters
        if dist.is_initialized():
            t = torch.tensor([el], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    rows = []
    for dname in args.dtypes.split(","):
        dt = dts[dname]
        es = torch.empty((), dtype=dt).element_size()
        for nbytes in sizes(args.min_bytes, args.max_bytes):
            n = nbytes // es
            n -= n % max(1, world)
            buf = torch.ones(n, dtype=dt, device=device)
            chunk = torch.empty(n // max(1, world), dtype=dt, device=device)
            for op in args.ops.split(","):
                if op == "all_reduce":
                    fn = lambda: dist.all_reduce(buf)  # noqa: E731
                elif op == "reduce_scatter":
                    fn = lambda: dist.reduce_scatter_tensor(chunk, buf)  # noqa: E731
                elif op == "all_gather":
                    fn = lambda: dist.all_gather_into_tensor(buf, chunk)  # noqa: E731
                else:
                    raise SystemExit(f"unknown op {op}")
                t = timeit(fn, args.iters, args.warmup)
                alg = n * es / t / 1e9
                rows.append({"op": op, "dtype": dname, "bytes": n * es, "us": round(t * 1e6, 2),
                             "algbw_gbs": round(alg, 2), "busbw_gbs": round(alg * bus_factor(op, world), 2)})
            del buf, chunk

    # small messages: RCCL all-reduce vs the one-shot P2P kernel
    small = []
    p2p = None
    if cuda and not args.no_p2p:
        try:
            from cloudtik_amd.parallel.p2p import P2PAllReducer
            p2p = P2PAllReducer(max_bytes=args.p2p_max_bytes)
        except Exception as e:  # noqa: BLE001 - no native library / IPC: RCCL-only table
            if rank == 0:
                print(f"[comm_bench] P2P all-reduce unavailable: {e!r}"[:300], file=sys.stderr)
    for nbytes in sizes(args.p2p_min_bytes, args.p2p_max_bytes):
        for dname in args.dtypes.split(","):
            dt = dts[dname]
            n = nbytes // torch.empty((), dtype=dt).element_size()
            buf = torch.ones(n, dtype=dt, device=device)
            r = {"dtype": dname, "bytes": nbytes,
                 "rccl_us": round(timeit(lambda: dist.all_reduce(buf), args.iters, args.warmup) * 1e6, 2)}
            if p2p is not None and p2p.supports(buf):
                r["p2p_us"] = round(timeit(lambda: p2p.all_reduce(buf), args.iters, args.warmup) * 1e6, 2)
                p2p.check()
            small.append(r)
    if p2p is not None:
        p2p.close()

    if rank == 0:
        hdr = "| op | dtype | MiB | us | algbw GB/s | busbw GB/s |\n|---|---|---:|---:|---:|---:|"
        lines = [hdr] + [f"| {r['op']} | {r['dtype']} | {r['bytes'] / MiB:.2f} | {r['us']} | {r['algbw_gbs']} | "
                         f"{r['busbw_gbs']} |" for r in rows]
        lines += ["", "| dtype | KiB | RCCL all-reduce us | P2P one-shot us |", "|---|---:|---:|---:|"]
        lines += [f"| {r['dtype']} | {r['bytes'] >> 10} | {r['rccl_us']} | {r.get('p2p_us', '-')} |" for r in small]
        print("\n".join(lines), file=sys.stderr)
        env = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_", "HSA_"))}
        out = {"world_size": world, "device": args.device,
               "backend": dist.get_backend() if dist.is_initialized() else None,
               "rccl": None, "env": env, "rows": rows, "small": small,
               "recommended_bucket_bytes": recommend_bucket(rows, args.plateau),
               "p2p_crossover_bytes": crossover(small)}
        if cuda:
            try:
                v = torch.cuda.nccl.version()
                out["rccl"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
            except Exception:  # noqa: BLE001
                pass
        if args.write_tuning is not None and cuda:
            from cloudtik_amd.parallel import comm_tuning
            gpu = torch.cuda.get_device_properties(device).name
            comm_tuning.record(world, out["recommended_bucket_bytes"], out["p2p_crossover_bytes"],
                               p=args.write_tuning or None, rccl=out["rccl"], gpu=gpu)
            out["tuning_written"] = args.write_tuning or comm_tuning.path()
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
