"""Distributed runtime: one process per GPU, torch.distributed over RCCL (xGMI) on GPUs and
gloo on CPU; rendezvous is env:// (MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE /
LOCAL_RANK) as set by ``cloudtik-run`` or torchrun."""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from .ddp import GradBucketer, broadcast_flat_params  # noqa: F401


# launcher families: (rank, size, local rank, local size) variables.  Rank and size are
# taken from ONE family (reference runner/util/env.py:22-45 does the same pairing); the
# torch/cloudtik-run family comes first because it is the innermost launcher when several
# are nested (torchrun under an mpirun allocation), then Horovod, OpenMPI, MPICH/PMI.
_FAMILIES = (("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"),
             ("HOROVOD_RANK", "HOROVOD_SIZE", "HOROVOD_LOCAL_RANK", "HOROVOD_LOCAL_SIZE"),
             ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK",
              "OMPI_COMM_WORLD_LOCAL_SIZE"),
             ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID", "MPI_LOCALNRANKS"))


def env_rank_info():
    """(rank, world, local_rank) from the launcher environment -- the ONE implementation used
    by bench.py, the Trainer and the Horovod-compatible API."""
    env = os.environ
    for rk, sz, lr, _ in _FAMILIES:
        r, w = env.get(rk), env.get(sz)
        if r not in (None, "") and w not in (None, ""):
            local = env.get(lr)
            if local in (None, ""):
                local = next((env[f[2]] for f in _FAMILIES if env.get(f[2]) not in (None, "")), 0)
            return int(r), int(w), int(local)
        if (r not in (None, "")) != (w not in (None, "")):
            raise RuntimeError(f"only one of {rk} / {sz} is set: cannot determine rank and world size")
    return 0, 1, 0


def env_local_world() -> int:
    env = os.environ
    for f in _FAMILIES:
        v = env.get(f[3])
        if v not in (None, ""):
            return int(v)
    return 1


def init_distributed(backend: str = None, timeout_s: int = 1800, gpu: bool = None):
    """Initialise the default process group if WORLD_SIZE > 1 and bind this rank's GPU.

    ``gpu`` (default: a GPU is present and the backend is not gloo) binds a GPU even under
    gloo -- ranks that share one GPU exercise the GPU data-parallel path (bucketer, gradient
    side stream, ZeRO-1) with gloo moving the CUDA tensors instead of RCCL.

    Returns (rank, world, local_rank, device)."""
    rank, world, local = env_rank_info()
    if gpu is None:
        gpu = backend != "gloo"
    use_gpu = torch.cuda.is_available() and gpu
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
