"""Horovod-compatible API on torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).

The reference installs Horovod 0.27 (built against NCCL/MPI/oneCCL) and its examples use
``hvd.DistributedOptimizer`` with fp16 compression and Adasum, ``broadcast_parameters`` and
``broadcast_optimizer_state`` (examples/runtime/ai/basics/pytorch/
imagenet-resnet50-synthetic-pytorch-horovod-run.py:159-169).  Scripts
written for ``import horovod.torch as hvd`` run unchanged against
``import cloudtik_amd.parallel.horovod as hvd``:

* ranks come from ``cloudtik-run --launcher horovod`` (HOROVOD_* / torch env);
* ``DistributedOptimizer`` does Horovod-style tensor fusion: gradients are packed into
  fusion buffers (``HOROVOD_FUSION_THRESHOLD``, default 64 MiB) in ready order with ONE
  multi-tensor HIP launch (ops.multi_tensor, optional bf16/fp16 compression and
  pre-scaling), all-reduced asynchronously while backward continues, and unpacked (with
  averaging) in ``step()`` / ``synchronize()``;
* ``op=Adasum`` combines gradients with the Adasum rule
  ``a (+) b = (1 - a.b / 2|a|^2) a + (1 - a.b / 2|b|^2) b`` over a binary tree of ranks.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist

Average, Sum, Adasum, Min, Max, Product = "average", "sum", "adasum", "min", "max", "product"


# ---------------------------------------------------------------------- process group
def init(comm=None, backend: Optional[str] = None):
    if dist.is_initialized():
        return
    from cloudtik_amd.train.trainer import setup_distributed
    rank, world, device = setup_distributed(backend)
    if world == 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29400 + os.getpid() % 1000))
        be = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(be, rank=0, world_size=1)


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()


def is_initialized() -> bool:
    return dist.is_initialized()


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", os.environ.get("HOROVOD_LOCAL_RANK", 0)))


def local_size() -> int:
    return int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("HOROVOD_LOCAL_SIZE", 1)))


def cross_rank() -> int:
    return rank() // max(1, local_size())


def cross_size() -> int:
    return max(1, size() // max(1, local_size()))


def nccl_built() -> bool:          # RCCL is the "nccl" backend on ROCm
    return dist.is_nccl_available()


def gloo_built() -> bool:
    return dist.is_gloo_available()


def mpi_built() -> bool:
    return dist.is_mpi_available()


def barrier():
    if size() > 1:
        dist.barrier()


def join(device=-1) -> int:
    barrier()
    return size() - 1


# ---------------------------------------------------------------------- compression
class _NoneCompressor:
    @staticmethod
    def compress(t):
        return t, None

    @staticmethod
    def decompress(t, ctx):
        return t

    dtype = None


class _CastCompressor:
    dtype = torch.float16

    @classmethod
    def compress(cls, t):
        if t.dtype.is_floating_point and t.dtype != cls.dtype:
            return t.to(cls.dtype), t.dtype
        return t, None

    @staticmethod
    def decompress(t, ctx):
        return t.to(ctx) if ctx is not None else t


class _FP16Compressor(_CastCompressor):
    dtype = torch.float16


class _BF16Compressor(_CastCompressor):
    dtype = torch.bfloat16


class Compression:
    none = _NoneCompressor
    fp16 = _FP16Compressor
    bf16 = _BF16Compressor


def _red_op(op):
    return {Sum: dist.ReduceOp.SUM, Average: dist.ReduceOp.SUM, Min: dist.ReduceOp.MIN, Max: dist.ReduceOp.MAX,
            Product: dist.ReduceOp.PRODUCT}[op]


def _resolve_op(average, op):
    if op is None:
        return Average if (average is None or average) else Sum
    return op


# ---------------------------------------------------------------------- collectives
class _Handle:
    def __init__(self, work, result, post=None):
        self.work, self.result, self.post = work, result, post

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
            if self.post is not None:
                self.result = self.post(self.result)
        return self.result


def allreduce_async_(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0,
                     compression=Compression.none):
    op = _resolve_op(average, op)
    if op == Adasum:
        adasum_allreduce_(tensor)
        return _Handle(None, tensor)
    t, ctx = compression.compress(tensor)
    if prescale_factor != 1.0:
        t.mul_(prescale_factor)
    work = dist.all_reduce(t, op=_red_op(op), async_op=True) if size() > 1 else None
    scale = postscale_factor / (size() if op == Average else 1)

    def post(res):
        r = compression.decompress(res, ctx)
        if scale != 1.0:
            r.mul_(scale)
        if r is not tensor:
            tensor.copy_(r)
        return tensor

    if work is None:
        return _Handle(None, post(t))
    return _Handle(work, t, post)


def allreduce_(tensor, average=None, name=None, op=None, **kw):
    return allreduce_async_(tensor, average, name, op, **kw).wait()


def allreduce(tensor, average=None, name=None, compression=Compression.none, op=None, **kw):
    return allreduce_(tensor.clone(), average, name, op, compression=compression, **kw)


def allreduce_async(tensor, average=None, name=None, op=None, **kw):
    return allreduce_async_(tensor.clone(), average, name, op, **kw)


def grouped_allreduce(tensors: List[torch.Tensor], average=None, name=None, op=None, compression=Compression.none):
    return [allreduce(t, average, name, compression, op) for t in tensors]


def synchronize(handle: _Handle):
    return handle.wait()


def poll(handle: _Handle) -> bool:
    return handle.work is None or handle.work.is_completed()


def allgather(tensor: torch.Tensor, name=None) -> torch.Tensor:
    """Concatenate every rank's tensor along dim 0 (first dims may differ)."""
    if size() == 1:
        return tensor.clone()
    n = torch.tensor([tensor.shape[0]], device=tensor.device)
    sizes = [torch.zeros_like(n) for _ in range(size())]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(tensor.shape[1:]), dtype=tensor.dtype, device=tensor.device)
    pad[:tensor.shape[0]] = tensor
    outs = [torch.empty_like(pad) for _ in range(size())]
    dist.all_gather(outs, pad)
    return torch.cat([o[:s] for o, s in zip(outs, sizes)])


def broadcast_(tensor, root_rank: int, name=None):
    if size() > 1:
        dist.broadcast(tensor, root_rank)
    return tensor


def broadcast(tensor, root_rank: int, name=None):
    return broadcast_(tensor.clone(), root_rank)


def broadcast_object(obj: Any, root_rank: int = 0, name=None):
    if size() == 1:
        return obj
    lst = [obj if rank() == root_rank else None]
    dist.broadcast_object_list(lst, root_rank)
    return lst[0]


def allgather_object(obj: Any, name=None) -> List[Any]:
    if size() == 1:
        return [obj]
    out = [None] * size()
    dist.all_gather_object(out, obj)
    return out


def alltoall(tensor: torch.Tensor, splits: Optional[List[int]] = None, name=None):
    if size() == 1:
        return tensor.clone()
    if splits is None:
        splits = [tensor.shape[0] // size()] * size()
    send = torch.tensor(splits, device=tensor.device)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    recv_splits = recv.tolist()
    out = torch.empty((sum(recv_splits),) + tuple(tensor.shape[1:]), dtype=tensor.dtype, device=tensor.device)
    dist.all_to_all_single(out, tensor.contiguous(), recv_splits, list(splits))
    return out


def broadcast_parameters(params, root_rank: int = 0):
    """params: a state_dict, or an iterable of (name, tensor) / tensors."""
    if isinstance(params, dict):
        items = sorted(params.items())
    else:
        items = list(params)
        items = [(str(i), p) if isinstance(p, torch.Tensor) else p for i, p in enumerate(items)]
    for _, p in items:
        if isinstance(p, torch.Tensor):
            broadcast_(p.data if hasattr(p, "data") else p, root_rank)


def broadcast_optimizer_state(optimizer, root_rank: int = 0):
    """Broadcast the optimizer's tensor state + hyper-parameters from root."""
    sd = optimizer.state_dict()
    # hyper-parameters (lr, momentum, ...) as an object; tensors by broadcast
    groups = broadcast_object([{k: v for k, v in g.items() if k != "params"} for g in sd["param_groups"]], root_rank)
    for g, src in zip(optimizer.param_groups, groups):
        g.update(src)
    for p_state in optimizer.state.values():
        for k, v in p_state.items():
            if isinstance(v, torch.Tensor):
                broadcast_(v, root_rank)
    flat = getattr(optimizer, "_flat_state", None)
    if callable(flat):
        for v in flat().values():
            broadcast_(v, root_rank)


# ---------------------------------------------------------------------- Adasum
def _adasum_pair(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    af, bf = a.double(), b.double()
    dot = (af * bf).sum()
    na, nb = (af * af).sum(), (bf * bf).sum()
    ca = 1.0 - dot / (2.0 * na) if na > 0 else torch.tensor(1.0, dtype=torch.float64, device=a.device)
    cb = 1.0 - dot / (2.0 * nb) if nb > 0 else torch.tensor(1.0, dtype=torch.float64, device=a.device)
    return (ca * af + cb * bf).to(a.dtype)


def adasum_allreduce_(tensor: torch.Tensor) -> torch.Tensor:
    """Adasum over all ranks (binary tree over the gathered vectors; identical result on
    every rank).  Memory: world x tensor -- meant for gradient buckets, not whole models
    on huge worlds."""
    w = size()
    if w == 1:
        return tensor
    flat = tensor.reshape(-1)
    outs = [torch.empty_like(flat) for _ in range(w)]
    dist.all_gather(outs, flat.contiguous())
    vecs = outs
    while len(vecs) > 1:
        nxt = [_adasum_pair(vecs[i], vecs[i + 1]) for i in range(0, len(vecs) - 1, 2)]
        if len(vecs) % 2:
            nxt.append(vecs[-1])
        vecs = nxt
    tensor.copy_(vecs[0].view_as(tensor))
    return tensor


# ---------------------------------------------------------------------- DistributedOptimizer
class _DistributedOptimizer:
    """Wraps a torch optimizer: fused, overlapped gradient all-reduce before ``step()``."""

    def __init__(self, optimizer, named_parameters=None, compression=Compression.none,
                 backward_passes_per_step: int = 1, op=Average, gradient_predivide_factor: float = 1.0,
                 fusion_threshold: Optional[int] = None):
        self._opt = optimizer
        self.compression = compression
        self.op = op
        self.backward_passes_per_step = max(1, backward_passes_per_step)
        self.predivide = gradient_predivide_factor
        params = [p for g in optimizer.param_groups for p in g["params"] if p.requires_grad]
        if named_parameters is not None:
            names = {id(p): n for n, p in named_parameters}
        else:
            names = {id(p): f"param.{i}" for i, p in enumerate(params)}
        self._names = names
        self._params = params
        thr = fusion_threshold if fusion_threshold is not None else int(
            os.environ.get("HOROVOD_FUSION_THRESHOLD", 64 * 1024 * 1024))
        # static buckets in reverse registration order (≈ backward order), split by dtype
        self._buckets: List[List[torch.nn.Parameter]] = []
        cur, cur_bytes, cur_dtype = [], 0, None
        for p in reversed(params):
            nb = p.numel() * p.element_size()
            if cur and (cur_bytes + nb > thr or p.dtype != cur_dtype):
                self._buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nb
            cur_dtype = p.dtype
        if cur:
            self._buckets.append(cur)
        self._bucket_of = {id(p): i for i, b in enumerate(self._buckets) for p in b}
        self._pending = [0] * len(self._buckets)
        self._counts: Dict[int, int] = {}
        self._handles: Dict[int, Tuple[_Handle, torch.Tensor]] = {}
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params] if size() > 1 else []
        self._skip = False

    def __getattr__(self, item):
        return getattr(self._opt, item)

    @property
    def param_groups(self):
        return self._opt.param_groups

    def _on_grad(self, p):
        if self._skip:
            return
        pid = id(p)
        self._counts[pid] = self._counts.get(pid, 0) + 1
        if self._counts[pid] % self.backward_passes_per_step:
            return
        b = self._bucket_of[pid]
        self._pending[b] += 1
        if self._pending[b] == len(self._buckets[b]):
            self._launch(b)

    def _launch(self, b):
        from cloudtik_amd.ops.multi_tensor import pack
        ps = self._buckets[b]
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in ps]
        cdt = self.compression.dtype if (self.compression.dtype is not None and grads[0].dtype.is_floating_point) \
            else grads[0].dtype
        pre = 1.0 / self.predivide if self.predivide != 1.0 else 1.0
        pre = pre / self.backward_passes_per_step
        flat = pack(grads, scale=pre, dtype=cdt)
        if self.op == Adasum:
            adasum_allreduce_(flat)
            self._handles[b] = (_Handle(None, flat), flat)
            return
        work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True)
        self._handles[b] = (_Handle(work, flat), flat)

    def synchronize(self):
        from cloudtik_amd.ops.multi_tensor import unpack
        if size() == 1:
            return
        for b in range(len(self._buckets)):
            if b not in self._handles and self._pending[b] < len(self._buckets[b]):
                self._launch(b)          # params without gradients this step
        post = self.predivide / (size() if self.op == Average else 1)
        if self.op == Adasum:
            post = self.predivide
        for b, (h, flat) in sorted(self._handles.items()):
            h.wait()
            ps = self._buckets[b]
            for p in ps:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            unpack(flat, [p.grad for p in ps], scale=post)
        self._handles.clear()
        self._pending = [0] * len(self._buckets)

    def step(self, closure=None):
        self.synchronize()
        return self._opt.step(closure)

    def zero_grad(self, set_to_none: bool = True):
        return self._opt.zero_grad(set_to_none=set_to_none)

    class _SkipSync:
        def __init__(self, o):
            self.o = o

        def __enter__(self):
            self.o._skip = True

        def __exit__(self, *a):
            self.o._skip = False

    def skip_synchronize(self):
        return _DistributedOptimizer._SkipSync(self)

    def state_dict(self):
        return self._opt.state_dict()

    def load_state_dict(self, sd):
        return self._opt.load_state_dict(sd)


def DistributedOptimizer(optimizer, named_parameters: Optional[Iterable] = None, compression=Compression.none,
                         backward_passes_per_step: int = 1, op=Average, gradient_predivide_factor: float = 1.0,
                         num_groups: int = 0, groups=None, sparse_as_dense: bool = False,
                         fusion_threshold: Optional[int] = None):
    return _DistributedOptimizer(optimizer, named_parameters, compression, backward_passes_per_step, op,
                                 gradient_predivide_factor, fusion_threshold)
