"""Multi-tensor flatten / unflatten in one HIP launch (bucket pack with scale + optional
bf16 compression; csrc/elementwise.hip mt_copy_kernel).  Reference: SSD
distributed.py:13-48 (flatten per dtype -> all_reduce -> /world -> unflatten) and Horovod
tensor fusion with fp16 compression."""
from __future__ import annotations

from typing import List, Optional

import torch


def _kernel_dtypes(*ts) -> bool:
    return all(t.dtype in (torch.float32, torch.bfloat16) for t in ts)


def pack(tensors: List[torch.Tensor], out: Optional[torch.Tensor] = None, scale: float = 1.0,
         dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    n = sum(t.numel() for t in tensors)
    dtype = dtype or tensors[0].dtype
    if out is None:
        out = torch.empty(n, dtype=dtype, device=tensors[0].device)
    from cloudtik_amd import ops
    if out.is_cuda and ops._use_native(out) and _kernel_dtypes(out, tensors[0]):
        ops.require_native().mt_copy([t.contiguous() for t in tensors], out, float(scale), False)
        return out
    off = 0
    for t in tensors:
        out[off:off + t.numel()].copy_(t.reshape(-1) * scale)
        off += t.numel()
    return out


def unpack(flat: torch.Tensor, tensors: List[torch.Tensor], scale: float = 1.0) -> None:
    from cloudtik_amd import ops
    if flat.is_cuda and ops._use_native(flat) and _kernel_dtypes(flat, tensors[0]) and \
            all(t.is_contiguous() for t in tensors):
        ops.require_native().mt_copy(list(tensors), flat, float(scale), True)
        return
    off = 0
    for t in tensors:
        t.copy_((flat[off:off + t.numel()].to(t.dtype) * scale).view_as(t))
        off += t.numel()
