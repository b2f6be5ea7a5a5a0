"""Bounded-memory streaming of Parquet row groups into pinned, GPU-bound batches.

The Spark -> AI hand-off (north-star config 5) at ImageNet scale: a rank's part files are
far larger than what should sit in host RAM (~190 GB of uint8 224x224 images per node), so
nothing is loaded up front.  Per epoch:

* the rank's (file, row group) units are shuffled with the epoch seed (metadata only);
* ``num_workers`` threads decode row groups ahead of the consumer, at most ``read_ahead``
  in flight (pyarrow releases the GIL while decoding);
* decoded row groups enter a shuffle pool of ``window`` row groups; full batches are drawn
  from a random permutation of the pool and the remainder carries over;
* a background producer gathers each batch's rows straight from the decoded row groups
  into one of ``prefetch`` pinned host slots (one copy per byte, no pool concatenation);
  the consumer sends the slot to the GPU with a non-blocking copy on a side stream, and a
  slot is rewritten only after the event recorded behind its previous copy has completed.

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
            a = _column_to_numpy(t.column(name))
            if name in self.shapes:
                a = a.reshape((a.shape[0],) + tuple(self.shapes[name]))
            out[name] = a
        del t
        return out

    def __iter__(self) -> Iterator[Dict[str, np.ndarray]]:
        return self.iter_into(None)

    def iter_into(self, alloc=None) -> Iterator[Dict[str, np.ndarray]]:
        """Yield batches; ``alloc(B, like)`` may supply the output arrays (e.g. pinned host
        slots) -- rows are gathered straight from the decoded row groups into them, grouped
        by row group (order inside a batch carries no meaning), one copy per byte."""
        rng = np.random.default_rng(self.seed + 7919 * self.epoch)
        order = list(range(len(self.units)))
        if self.shuffle:
            rng.shuffle(order)
        limit = len(self)
        emitted = 0
        B = self.batch_size
        pool: Dict[int, Dict[str, np.ndarray]] = {}
        carry_rg = np.empty(0, np.int64)
        carry_row = np.empty(0, np.int64)
        new_rg: List[np.ndarray] = []
        new_row: List[np.ndarray] = []
        uid = 0

        def gather(rg_ids, rows, n_out):
            srt = np.argsort(rg_ids, kind="stable")
            rg_ids, rows = rg_ids[srt], rows[srt]
            cuts = np.flatnonzero(np.diff(rg_ids)) + 1
            starts = np.concatenate([[0], cuts])
            ends = np.concatenate([cuts, [n_out]])
            like = pool[int(rg_ids[0])]
            out = alloc(n_out, like) if alloc is not None else \
                {c: np.empty((n_out,) + like[c].shape[1:], like[c].dtype) for c in self.columns}
            for s0, e0 in zip(starts, ends):
                src = pool[int(rg_ids[s0])]
                for c in self.columns:
                    np.take(src[c], rows[s0:e0], axis=0, out=out[c][s0:e0])
            return out

        with ThreadPoolExecutor(self.num_workers) as ex:
            pending = collections.deque()
            it = iter(order)

            def refill():
                while len(pending) < self.read_ahead:
                    k = next(it, None)
                    if k is None:
                        return
                    pending.append(ex.submit(self._read, self.units[k]))
            refill()
            while True:
                exhausted = not pending
                if not exhausted:
                    arrays = pending.popleft().result()
                    refill()
                    n = len(arrays[self.columns[0]])
                    pool[uid] = arrays
                    new_rg.append(np.full(n, uid, np.int64))
                    new_row.append(np.arange(n, dtype=np.int64))
                    uid += 1
                    if len(new_rg) < self.window:
                        continue                      # keep filling the shuffle window
                rg_ids = np.concatenate([carry_rg] + new_rg)
                rows = np.concatenate([carry_row] + new_row)
                new_rg, new_row = [], []
                if not len(rg_ids):
                    return
                if self.shuffle:
                    perm = rng.permutation(len(rg_ids))
                    rg_ids, rows = rg_ids[perm], rows[perm]
                nb = len(rg_ids) // B
                for b in range(nb):
                    if emitted >= limit:
                        return
                    yield gather(rg_ids[b * B:(b + 1) * B], rows[b * B:(b + 1) * B], B)
                    emitted += 1
                carry_rg, carry_row = rg_ids[nb * B:], rows[nb * B:]
                live = set(np.unique(carry_rg).tolist())
                for k in [k for k in pool if k not in live]:
                    del pool[k]                        # row group fully consumed
                if exhausted:
                    if len(carry_rg) and not self.drop_last and emitted < limit:
                        yield gather(carry_rg, carry_row, len(carry_rg))
                    return


class PinnedBatchLoader:
    """Background producer: gathers each batch straight into one of ``prefetch`` pinned
    host slots; the consumer issues the H2D copy on a side stream, records an event, and
    the producer reuses the slot only once that event has completed."""

    def __init__(self, stream: ParquetRowGroupStream, device, prefetch: int = 4):
        self.stream = stream
        self.device = torch.device(device)
        self.on_gpu = self.device.type == "cuda"
        self.prefetch = max(2, prefetch)
        self.slots: List[Optional[Dict[str, torch.Tensor]]] = [None] * self.prefetch
        self.events: List[Optional[object]] = [None] * self.prefetch
        self.copy_stream = torch.cuda.Stream(device=self.device) if self.on_gpu else None

    def __len__(self):
        return len(self.stream)

    def _slot(self, i, B, like):
        slot = self.slots[i]
        if slot is None or slot[self.stream.columns[0]].shape[0] != B:
            slot = self.slots[i] = {c: torch.empty((B,) + like[c].shape[1:],
                                                   dtype=torch.from_numpy(np.empty(0, like[c].dtype)).dtype,
                                                   pin_memory=self.on_gpu)
                                    for c in self.stream.columns}
        return {c: t.numpy() for c, t in slot.items()}

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        import queue
        import threading
        ready: "queue.Queue" = queue.Queue()
        free: "queue.Queue" = queue.Queue()
        for i in range(self.prefetch):
            free.put(i)
        stop = threading.Event()
        current = [None]

        def alloc(B, like):
            i = free.get()
            while i is None:
                i = free.get()
            ev = self.events[i]
            if ev is not None:
                ev.synchronize()               # the H2D copy that last read this slot is done
            current[0] = i
            return self._slot(i, B, like)

        def produce():
            try:
                for batch in self.stream.iter_into(alloc):
                    if stop.is_set():
                        return
                    ready.put((current[0], batch))
                ready.put(None)
            except BaseException as e:  # noqa: BLE001 - surfaced in the consumer
                ready.put(e)

        th = threading.Thread(target=produce, daemon=True, name="parquet-batch-producer")
        th.start()
        try:
            while True:
                item = ready.get()
                if item is None:
                    return
                if isinstance(item, BaseException):
                    raise item
                i, batch = item
                if not self.on_gpu:
                    out = {c: torch.from_numpy(a.copy()) for c, a in batch.items()}
                    free.put(i)
                    yield out
                    continue
                cur = torch.cuda.current_stream(self.device)
                with torch.cuda.stream(self.copy_stream):
                    out = {c: self.slots[i][c].to(self.device, non_blocking=True) for c in batch}
                    if self.events[i] is None:
                        self.events[i] = torch.cuda.Event()
                    self.events[i].record(self.copy_stream)
                free.put(i)
                cur.wait_stream(self.copy_stream)
                for t in out.values():
                    t.record_stream(cur)
                yield out
        finally:
            stop.set()
            for _ in range(self.prefetch):
                free.put(None)                 # wake a producer blocked on a slot
            th.join(timeout=30)


def agree_min_batches(n: int) -> int:
    """Minimum of ``n`` over the default process group (equal batch counts on every rank)."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return n
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([n], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())
