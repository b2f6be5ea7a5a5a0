"""Distributed runtime: one process per GPU, torch.distributed over RCCL (xGMI) on GPUs and
gloo on CPU; rendezvous is env:// (MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE /
LOCAL_RANK) as set by ``cloudtik-run`` or torchrun."""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from .ddp import GradBucketer, broadcast_flat_params  # noqa: F401


def env_rank_info():
    """(rank, world, local_rank) from the launcher environment (torch/PMI/OMPI/Horovod
    conventions, mirroring runtime/ai/runner/util/env.py:22-71 of the reference)."""
    def first(*names, default=None):
        for n in names:
            v = os.environ.get(n)
            if v not in (None, ""):
                return int(v)
        return default
    rank = first("RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK", "HOROVOD_RANK", default=0)
    world = first("WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "HOROVOD_SIZE", default=1)
    local = first("LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK",
                  "HOROVOD_LOCAL_RANK", default=0)
    return rank, world, local


def init_distributed(backend: str = None, timeout_s: int = 1800):
    """Initialise the default process group if WORLD_SIZE > 1 and bind this rank's GPU.

    Returns (rank, world, local_rank, device)."""
    rank, world, local = env_rank_info()
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        os.environ["RANK"], os.environ["WORLD_SIZE"] = str(rank), str(world)
        be = backend or ("nccl" if use_gpu else "gloo")
        kw = dict(backend=be, init_method="env://", rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return rank, world, local, device


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(x: float) -> float:
    if not dist.is_initialized():
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
from .sequence import ring_attention, ulysses_attention  # noqa: F401,E402
