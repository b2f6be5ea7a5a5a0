"""Prefetching batch loader over columnar host data, backed by the native loader
(ops/csrc/loader.hip): worker threads gather shuffled rows into pinned host slots and each
``next()`` issues ``hipMemcpyAsync`` per column on a side stream that the consumer's
stream waits on -- no host<->device synchronisation on the training loop's critical path.

    loader = NativeLoader({"image": images_uint8, "label": labels}, batch_size=256,
                          rank=rank, world=world, device="cuda")
    for epoch in range(E):
        loader.set_epoch(epoch)
        for batch in loader:          # dict of device tensors, [B, ...] per column
            ...

Every DP rank reads a disjoint set of batches of the same per-epoch permutation.
On a CPU device (tests, CPU-only jobs) the same pipeline runs with plain host buffers.
"""
from __future__ import annotations

from typing import Dict, Iterator, Optional

import numpy as np
import torch


def _as_host_tensor(a) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        t = a.detach()
        if t.is_cuda:
            raise ValueError("loader columns must live in host memory")
        return t.contiguous()
    arr = np.ascontiguousarray(a)
    if not arr.flags.writeable:        # e.g. zero-copy Arrow buffers
        arr = arr.copy()
    return torch.from_numpy(arr)


class NativeLoader:
    def __init__(self, columns: Dict[str, object], batch_size: int, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False, num_workers: int = 4, prefetch: int = 4, rank: int = 0, world: int = 1,
                 device=None):
        from cloudtik_amd import ops
        self._C = ops.require_native() if torch.cuda.is_available() else ops._C
        if self._C is None:
            raise RuntimeError("the native op library is not built (python -m cloudtik_amd.ops.build)")
        self.names = list(columns)
        self.cols = [_as_host_tensor(columns[n]) for n in self.names]
        n = self.cols[0].shape[0]
        for name, c in zip(self.names, self.cols):
            if c.shape[0] != n:
                raise ValueError(f"column {name} has {c.shape[0]} rows, expected {n}")
        self.num_rows = n
        self.batch_size = batch_size
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.on_gpu = self.device.type == "cuda"
        self._h = self._C.loader_create(self.cols, batch_size, shuffle, seed, drop_last, num_workers,
                                        max(2, prefetch), rank, world, self.on_gpu)
        self._copy_stream = torch.cuda.Stream(device=self.device) if self.on_gpu else None
        self.epoch = 0

    def __len__(self) -> int:
        return int(self._C.loader_num_batches(self._h))

    def set_epoch(self, epoch: int):
        self.epoch = epoch
        self._C.loader_set_epoch(self._h, epoch)

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        for _ in range(len(self)):
            b = self.next()
            if b is None:
                return
            yield b
        # rearm the same epoch for a second iteration unless set_epoch is called
        self._C.loader_set_epoch(self._h, self.epoch)

    def next(self) -> Optional[Dict[str, torch.Tensor]]:
        shapes = [(self.batch_size,) + tuple(c.shape[1:]) for c in self.cols]
        if self.on_gpu:
            # allocate on the copy stream: the allocator then only hands out blocks whose
            # previous users on that stream are done, so the async copy never races compute
            with torch.cuda.stream(self._copy_stream):
                outs = [torch.empty(s, dtype=c.dtype, device=self.device) for s, c in zip(shapes, self.cols)]
            rows = self._C.loader_next_device(self._h, outs, self._copy_stream.cuda_stream)
            cur = torch.cuda.current_stream(self.device)
            for t in outs:                 # consumed on the compute stream
                t.record_stream(cur)
        else:
            outs = [torch.empty(s, dtype=c.dtype) for s, c in zip(shapes, self.cols)]
            rows = self._C.loader_next_host(self._h, outs)
        if rows == 0:
            return None
        if rows < self.batch_size:
            outs = [t[:rows] for t in outs]
        return dict(zip(self.names, outs))

    def close(self):
        if getattr(self, "_h", None):
            if self.on_gpu:
                torch.cuda.current_stream(self.device).synchronize()
            self._C.loader_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
