"""A whole training step -- forward, backward, gradient side stream, optimizer -- captured
once into a hipGraph and replayed (the MI355X answer to a tracing compiler: the kernels stay
the hand-written ones, only their launch goes away).

A ResNet-50 step is ~650 kernel launches; issued one by one from Python the device idles in
the gaps between dependent launches (the serial profile shows 89 % busy,
profiles/r3/steady_resnet50_serial.md).  Replaying the captured graph issues the same kernels
back to back with no host work per kernel.

Rules the captured step must follow (all hold for the bench steps of models/resnet.py):
* static inputs: the step reads the same input tensors every time (copy new data into them);
* no host synchronisation inside (no ``.item()``, no host-side branches on device values);
* per-step optimizer scalars travel through the optimizer's graph slot
  (``graph_step_prepare`` before every replay -- train/optim.py);
* kernels that draw dropout masks get their seed / offset as kernel arguments, so a captured
  step with dropout would replay the SAME mask: ``GraphedStep`` refuses when told the step
  uses dropout (``uses_rng=True``);
* data-parallel collectives are not captured: use it at world size 1 (bench.py --graph).

Measured (scripts/gpu_graph_ab.sh, ResNet-50 batch 256, 1x MI355X): 27.19 / 27.16 ms per step
eager vs 29.12 / 28.94 replayed -- the eager step is already GPU-bound (its weight gradients
overlap the backward chain on a side stream, and the replayed graph keeps less of that
overlap), so the bench leaves capture off; it pays where launches dominate (small batches,
small models).

Warm-up iterations run eagerly on a side stream first (lazy handles, allocator, tuning),
then one capture; every later call is a replay.  The return value is the step output of the
capture (a static tensor refreshed by each replay)."""
from __future__ import annotations

from typing import Any, Callable, Optional, Sequence

import torch


class GraphedStep:
    def __init__(self, fn: Callable[[], Any], optimizers: Sequence[Any] = (), warmup: int = 3,
                 uses_rng: bool = False):
        if uses_rng:
            raise ValueError("graph capture would freeze the dropout masks of this step")
        self.fn = fn
        self.optimizers = list(optimizers)
        self.warmup = int(warmup)
        self.calls = 0
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None

    def _capture(self):
        for o in self.optimizers:
            o.graph_capture_begin()
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            self.out = self.fn()
        torch.cuda.synchronize()
        self.graph = g

    def __call__(self):
        if self.graph is None:
            self.calls += 1
            if self.calls <= self.warmup:
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    out = self.fn()
                torch.cuda.current_stream().wait_stream(side)
                return out
            self._capture()
        for o in self.optimizers:
            o.graph_step_prepare()
        self.graph.replay()
        for o in self.optimizers:
            o.graph_step_done()
        return self.out
