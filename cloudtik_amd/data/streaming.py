"""Bounded-memory streaming of Parquet row groups into pinned, GPU-bound batches.

The Spark -> AI hand-off (north-star config 5) at ImageNet scale: a rank's part files are
far larger than what should sit in host RAM (~190 GB of uint8 224x224 images per node), so
nothing is loaded up front.  Per epoch:

* the rank's (file, row group) units are shuffled with the epoch seed (metadata only);
* ``num_workers`` threads decode row groups ahead of the consumer, at most ``read_ahead``
  in flight (pyarrow releases the GIL while decoding);
* decoded row groups enter a shuffle pool of ``window`` row groups; full batches are drawn
  from a random permutation of the pool and the remainder carries over;
* each batch is copied into one of ``prefetch`` pinned host slots and sent to the GPU with a
  non-blocking copy on a side stream; a slot is rewritten only after the event recorded
  behind its previous copy has completed.

Host memory is therefore bounded by ``(window + read_ahead) x row-group bytes + prefetch x
batch bytes`` whatever the dataset size.  Every rank yields the same number of batches per
epoch (the minimum over ranks, agreed once through the process group), so collectives stay
in lockstep.  Reference flow: Petastorm readers over the Horovod Store's Parquet
(examples/runtime/ai/basics/pytorch/mnist-pytorch-spark-horovod-hyperopt-mlflow.py:159-214).
"""
from __future__ import annotations

import collections
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch


def _open(path: str, **kw):
    import pyarrow.parquet as pq
    if "://" in path:
        import pyarrow.fs as pafs
        fs, p = pafs.FileSystem.from_uri(path)
        return pq.ParquetFile(fs.open_input_file(p), **kw)
    return pq.ParquetFile(path, **kw)


class ParquetRowGroupStream:
    """Shuffled, batched numpy columns streamed from Parquet row groups."""

    def __init__(self, paths: Sequence[str], batch_size: int, columns: Sequence[str],
                 shapes: Optional[Dict[str, Tuple[int, ...]]] = None, shuffle: bool = True, seed: int = 0,
                 window: int = 4, read_ahead: int = 2, num_workers: int = 2, drop_last: bool = True):
        from cloudtik_amd.data.parquet import _expand
        self.paths = _expand(list(paths))
        self.batch_size = int(batch_size)
        self.columns = list(columns)
        self.shapes = dict(shapes or {})
        self.shuffle, self.seed = shuffle, seed
        self.window, self.read_ahead = max(1, window), max(1, read_ahead)
        self.num_workers = max(1, num_workers)
        self.drop_last = drop_last
        self.units: List[Tuple[str, int, int]] = []
        for p in self.paths:
            md = _open(p).metadata
            for g in range(md.num_row_groups):
                self.units.append((p, g, md.row_group(g).num_rows))
        if not self.units:
            raise FileNotFoundError(f"no parquet row groups in {paths}")
        self.num_rows = sum(u[2] for u in self.units)
        self.max_batches: Optional[int] = None
        self.epoch = 0

    def __len__(self) -> int:
        n = self.num_rows // self.batch_size if self.drop_last else -(-self.num_rows // self.batch_size)
        return min(n, self.max_batches) if self.max_batches is not None else n

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def _read(self, unit) -> Dict[str, np.ndarray]:
        from cloudtik_amd.data.parquet import _column_to_numpy
        path, g, _ = unit
        # a fresh reader per row group, closed right away: a cached ParquetFile keeps the
        # buffers of every row group it has read alive (measured: the whole part file)
        f = _open(path, pre_buffer=False)
        try:
            t = f.read_row_group(g, columns=self.columns)
        finally:
            f.close()
        out = {}
        for name in self.columns:
            # own copies: numpy views would pin the Arrow buffers until the pool drains
            a = np.array(_column_to_numpy(t.column(name)), copy=True)
            if name in self.shapes:
                a = a.reshape((a.shape[0],) + tuple(self.shapes[name]))
            out[name] = a
        del t
        return out

    def __iter__(self) -> Iterator[Dict[str, np.ndarray]]:
        rng = np.random.default_rng(self.seed + 7919 * self.epoch)
        order = list(range(len(self.units)))
        if self.shuffle:
            rng.shuffle(order)
        limit = len(self)
        emitted = 0
        pool: List[Dict[str, np.ndarray]] = []
        pool_rows = 0
        B = self.batch_size
        with ThreadPoolExecutor(self.num_workers) as ex:
            pending = collections.deque()
            it = iter(order)

            def refill():
                while len(pending) < self.read_ahead:
                    i = next(it, None)
                    if i is None:
                        return
                    pending.append(ex.submit(self._read, self.units[i]))
            refill()
            while True:
                exhausted = not pending
                if not exhausted:
                    rg = pending.popleft().result()
                    refill()
                    pool.append(rg)
                    pool_rows += len(rg[self.columns[0]])
                    if len(pool) < self.window:
                        continue                      # keep filling the shuffle window
                elif not pool_rows:
                    return
                merged = {n: np.concatenate([r[n] for r in pool]) if len(pool) > 1 else pool[0][n]
                          for n in self.columns}
                perm = rng.permutation(pool_rows) if self.shuffle else np.arange(pool_rows)
                nb = pool_rows // B
                for b in range(nb):
                    if emitted >= limit:
                        return
                    idx = perm[b * B:(b + 1) * B]
                    yield {n: merged[n][idx] for n in self.columns}
                    emitted += 1
                rest = perm[nb * B:]
                pool = [{n: merged[n][rest] for n in self.columns}] if len(rest) else []
                pool_rows = len(rest)
                del merged
                if exhausted:
                    if pool_rows and not self.drop_last and emitted < limit:
                        yield pool[0]
                    return


class PinnedStager:
    """numpy batch -> pinned host slot -> device, asynchronously on a side stream."""

    def __init__(self, device, prefetch: int = 4):
        self.device = torch.device(device)
        self.on_gpu = self.device.type == "cuda"
        self.prefetch = max(2, prefetch)
        self.slots: List[Optional[Dict[str, torch.Tensor]]] = [None] * self.prefetch
        self.events: List[Optional[torch.cuda.Event]] = [None] * self.prefetch
        self.i = 0
        self.stream = torch.cuda.Stream(device=self.device) if self.on_gpu else None

    def __call__(self, batch: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
        if not self.on_gpu:
            return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in batch.items()}
        i = self.i = (self.i + 1) % self.prefetch
        ev = self.events[i]
        if ev is not None:
            ev.synchronize()                   # the copy that last read this slot has finished
        slot = self.slots[i]
        if slot is None or any(slot[k].shape != v.shape or slot[k].dtype != torch.from_numpy(v[:0]).dtype
                               for k, v in batch.items()):
            slot = self.slots[i] = {k: torch.empty(v.shape, dtype=torch.from_numpy(v[:0]).dtype, pin_memory=True)
                                    for k, v in batch.items()}
        for k, v in batch.items():
            slot[k].numpy()[...] = v
        cur = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self.stream):
            out = {k: t.to(self.device, non_blocking=True) for k, t in slot.items()}
            if ev is None:
                ev = self.events[i] = torch.cuda.Event()
            ev.record(self.stream)
        cur.wait_stream(self.stream)
        for t in out.values():
            t.record_stream(cur)
        return out


def agree_min_batches(n: int) -> int:
    """Minimum of ``n`` over the default process group (equal batch counts on every rank)."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return n
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([n], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())
