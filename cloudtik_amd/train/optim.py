"""Fused multi-tensor optimizers over a flat parameter space.

``FlatParamSpace`` re-homes every parameter of a model into ONE contiguous buffer per
role -- bf16 model weights, fp32 master weights, gradients -- and points each
``nn.Parameter.data`` / ``.grad`` at a view of it.  Consequences that matter on MI355X:

* the optimizer step is one (LAMB: two) kernel launch(es) for the whole model
  (csrc/optim.hip) instead of ~400 per-tensor launches;
* the gradient buffer IS the data-parallel communication buffer: buckets are plain
  slices, so RCCL all-reduces / reduce-scatters need no pack/unpack copies
  (cloudtik_amd.parallel.ddp);
* with ``shard=(rank, world)`` and ``GradBucketer(mode="reduce_scatter")`` each rank owns
  1/world of the flat space (ZeRO-1): chunk ``rank`` of every gradient bucket, packed into
  shard-local buffers.  Optimizer state and fp32 master weights exist only for the shard,
  gradients are reduce-scattered bucket by bucket during backward, the updated weights are
  all-gathered after the step -- the same bytes on the wire as an all-reduce, 1/world of the
  optimizer HBM traffic and state memory.  Checkpoints hold the state in the global layout.

Reference optimizers reproduced: LAMB (bert_large/training/lamb.py:61-139 -- bf16 params
with fp32 master copy, no bias correction, trust ratio only where weight_decay != 0),
Adam/AdamW (transfer-learning Trainer, GraphSAGE), SGD+momentum (ResNet-50 main.py:317,
DLRM split-SGD).  On CPU the identical math runs in PyTorch.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Callable, Iterable, List, Optional, Sequence, Tuple

import torch

SEG = 8192
ALIGN = 64
_DYN_SLOTS = 8


def _sync_grads():
    """Order the optimizer after weight-gradient GEMMs issued on the gradient side stream."""
    if torch.cuda.is_available():
        from cloudtik_amd.ops.linear import sync_grad_stream
        sync_grad_stream()


def _memory_order(t: torch.Tensor) -> torch.Tensor:
    """``t`` permuted so that its logical order is its memory order (dense tensors)."""
    if t.is_contiguous():
        return t
    perm = sorted(range(t.dim()), key=lambda d: (-t.stride(d), d))
    return t.permute(perm)


def _flat_view(flat: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    """A view of the 1-D slice ``flat`` with ``like``'s shape and strides (same layout)."""
    if like.is_contiguous():
        return flat.view(like.shape)
    return flat.as_strided(like.shape, like.stride())


def _same_order(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same shape and the same strides on every dim of size > 1 (``b`` dense => ``a`` dense
    with the same element order)."""
    return a.shape == b.shape and all(sa == sb for sa, sb, n in zip(a.stride(), b.stride(), a.shape) if n > 1)


class FlatParamSpace:
    def __init__(self, params: Sequence[torch.nn.Parameter], names: Optional[Sequence[str]] = None,
                 grad_dtype: Optional[torch.dtype] = None, shard: Tuple[int, int] = (0, 1),
                 align: int = ALIGN, reverse: bool = True, defer_conv_grads: Optional[bool] = None):
        params = [p for p in params if p.requires_grad]
        assert params, "no trainable parameters"
        names = list(names) if names is not None else [f"p{i}" for i in range(len(params))]
        if reverse:  # backward produces late-layer grads first: put them first in the buffer
            params, names = params[::-1], names[::-1]
        self.params: List[torch.nn.Parameter] = params
        self.names = names
        self.dtype = params[0].dtype
        self.device = params[0].device
        for p in params:
            assert p.dtype == self.dtype and p.device == self.device, "mixed dtype/device params"
        self.grad_dtype = grad_dtype or self.dtype
        self.offsets, self.numels = [], []
        off = 0
        for p in params:
            self.offsets.append(off)
            self.numels.append(p.numel())
            off += ((p.numel() + align - 1) // align) * align
        self.used = off                  # world-size independent: the parameters' extent
        rank, world = shard
        self.rank, self.world = rank, world
        # pad total so every shard is an aligned equal slice
        unit = align * world
        self.total = ((off + unit - 1) // unit) * unit
        self.shard_size = self.total // world
        self.shard_lo = rank * self.shard_size
        self.shard_hi = self.shard_lo + self.shard_size

        dev = self.device
        self.model = torch.zeros(self.total, dtype=self.dtype, device=dev)
        self.grad = torch.zeros(self.total, dtype=self.grad_dtype, device=dev)
        # Deferred conv-weight gradients: autograd's AccumulateGrad adds every conv weight
        # gradient into a preset .grad with its own small kernel (53 launch-bound adds per
        # ResNet-50 step).  Instead these parameters keep .grad unset, so AccumulateGrad just
        # takes MIOpen's output tensor; a post-accumulate hook records the parameter and
        # flush_grads() adds all recorded gradients into the flat buffer with ONE multi-tensor
        # kernel (ops mt_add_) before anything reads the buffer (bucket launch, finish,
        # optimizer step).
        if defer_conv_grads is None:
            import os
            defer_conv_grads = os.environ.get("CLOUDTIK_AMD_DEFER_CONV_GRADS", "1") == "1"
        self._deferred: "OrderedDict[int, torch.nn.Parameter]" = OrderedDict()
        self._hooks = []
        with torch.no_grad():
            for p, o, n in zip(params, self.offsets, self.numels):
                # keep each parameter's memory layout: a channels_last conv weight stays
                # channels_last as a view of the flat buffer (MIOpen's NHWC solvers need
                # input, weight and gradients in the same layout; an NCHW weight next to
                # NHWC activations sends the backward pass to the naive fallback kernels)
                self.model[o:o + n].copy_(_memory_order(p.data).reshape(-1))
                p.data = _flat_view(self.model[o:o + n], p)
                view = _flat_view(self.grad[o:o + n], p)
                if defer_conv_grads and dev.type == "cuda" and p.dim() == 4 and self.grad_dtype == self.dtype:
                    p.grad = None
                    p._ct_flat_view = view
                    p._ct_flat_grad = False
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._on_deferred))
                else:
                    p.grad = view
                    p._ct_flat_grad = True   # ops.linear may accumulate dW straight into it
        # fp32 gradient the optimizer reads instead of ``grad`` when a bucketer reduces /
        # accumulates in fp32 (parallel.GradBucketer(reduce_dtype=torch.float32))
        self.main_grad: Optional[torch.Tensor] = None
        # the shard as (global lo, global hi, shard-local offset) pieces: one contiguous slice
        # by default; set_shard_pieces() switches to ZeRO-1's bucket-interleaved layout
        self.pieces: List[Tuple[int, int, int]] = [(self.shard_lo, self.shard_hi, 0)]
        self.local_grad: Optional[torch.Tensor] = None    # reduce-scatter output (ZeRO-1)
        self.local_model: Optional[torch.Tensor] = None   # this rank's updated weights (ZeRO-1)
        self.norm_allreduce: Optional[Callable[[torch.Tensor], None]] = None
        self.gather_fn: Optional[Callable[[torch.Tensor, torch.Tensor], None]] = None
        self._after_step: Optional[Callable[[], None]] = None
        # fp32 master copy of THIS rank's shard only
        self.master = self.model[self.shard_lo:self.shard_hi].float().clone() \
            if self.dtype != torch.float32 else None
        self._build_segments()

    def set_shard_pieces(self, pieces: Sequence[Tuple[int, int, int]], grad_dtype: torch.dtype,
                         norm_allreduce: Callable[[torch.Tensor], None],
                         gather_fn: Callable[[torch.Tensor, torch.Tensor], None],
                         after_step: Callable[[], None]):
        """ZeRO-1 layout: this rank owns ``pieces`` (global ranges, packed back to back in
        shard-local buffers).  ``gather_fn(local, full)`` rebuilds a global-layout tensor from
        every rank's shard-local one; ``after_step`` all-gathers the updated weights."""
        assert sum(h - l for l, h, _ in pieces) == self.shard_size, "pieces must cover one shard"
        self.pieces = list(pieces)
        self.local_model = self.local_of(self.model)
        self.local_grad = torch.zeros(self.shard_size, dtype=grad_dtype, device=self.device)
        self.master = self.local_model.float().clone() if self.dtype != torch.float32 else None
        self.norm_allreduce, self.gather_fn, self._after_step = norm_allreduce, gather_fn, after_step
        self._build_segments()

    @property
    def sharded(self) -> bool:
        return self.local_model is not None

    def local_of(self, full: torch.Tensor) -> torch.Tensor:
        """This rank's pieces of a global-layout flat tensor, packed."""
        if len(self.pieces) == 1:
            lo, hi, _ = self.pieces[0]
            return full[lo:hi].clone()
        return torch.cat([full[lo:hi] for lo, hi, _ in self.pieces])

    def full_of(self, local: torch.Tensor) -> torch.Tensor:
        """Global-layout tensor assembled from every rank's shard-local ``local``."""
        if self.gather_fn is None:
            return local
        full = torch.zeros(self.total, dtype=local.dtype, device=local.device)
        self.gather_fn(local, full)
        return full

    def after_step(self):
        if self._after_step is not None:
            self._after_step()

    # ------------------------------------------------------------------ segments
    def _build_segments(self):
        seg_tensor, seg_start, seg_len, first = [], [], [], []
        for t, (o, n) in enumerate(zip(self.offsets, self.numels)):
            first.append(len(seg_tensor))
            padded = ((n + ALIGN - 1) // ALIGN) * ALIGN
            for lo, hi, loc in self.pieces:      # a tensor may span several pieces
                a, b = max(o, lo), min(o + padded, hi)
                s = a
                while s < b:
                    e = min(s + SEG, b)
                    seg_tensor.append(t)
                    seg_start.append(loc + s - lo)      # shard-local
                    seg_len.append(e - s)
                    s = e
        first.append(len(seg_tensor))
        dev = self.device
        self.nseg = len(seg_tensor)
        self.seg_tensor = torch.tensor(seg_tensor or [0], dtype=torch.int32, device=dev)
        self.seg_start = torch.tensor(seg_start or [0], dtype=torch.int64, device=dev)
        self.seg_len = torch.tensor(seg_len or [0], dtype=torch.int32, device=dev)
        self.tensor_first_seg = torch.tensor(first, dtype=torch.int32, device=dev)
        self._seg_cpu = (seg_tensor, seg_start, seg_len)

    # ------------------------------------------------------------------ views
    @property
    def shard_params(self) -> torch.Tensor:
        """fp32 weights owned by this rank (master copy, or the model buffer if fp32)."""
        return self.master if self.master is not None else self.shard_model

    @property
    def shard_model(self) -> torch.Tensor:
        if self.local_model is not None:
            return self.local_model
        return self.model[self.shard_lo:self.shard_hi]

    @property
    def reduced_grad(self) -> torch.Tensor:
        """The gradient the optimizer consumes: the fp32 reduction buffer if one is attached,
        else the (model-dtype) gradient buffer itself."""
        return self.main_grad if self.main_grad is not None else self.grad

    @property
    def shard_grad(self) -> torch.Tensor:
        if self.local_grad is not None:
            return self.local_grad
        return self.reduced_grad[self.shard_lo:self.shard_hi]

    # ------------------------------------------------------------------ deferred grads
    def _on_deferred(self, p):
        self._deferred[id(p)] = p

    def flush_grads(self):
        """Add the recorded conv-weight gradients into the flat buffer (one launch) and
        release them; a no-op when nothing is pending."""
        if not self._deferred:
            return
        ps = [p for p in self._deferred.values() if p.grad is not None]
        self._deferred.clear()
        srcs, dsts = [], []
        for p in ps:
            g, v = p.grad, p._ct_flat_view
            # same memory order (strides of size-1 dims do not matter: a 1x1 conv weight's
            # gradient may come back NCHW-strided while the channels_last view is not)
            if g.dtype == v.dtype and _same_order(g, v):
                srcs.append(g)
                dsts.append(v)
            else:
                v.add_(g)
        if srcs:
            from cloudtik_amd import ops
            ops.require_native().mt_add_(srcs, dsts)
        for p in ps:
            p.grad = None

    def zero_grad(self):
        for p in self._deferred.values():
            p.grad = None
        self._deferred.clear()
        self.grad.zero_()
        if self.main_grad is not None:
            self.main_grad.zero_()
        if self.local_grad is not None:
            self.local_grad.zero_()

    def tensor_wd(self, wd_fn: Callable[[str, torch.nn.Parameter], float]) -> torch.Tensor:
        return torch.tensor([float(wd_fn(n, p)) for n, p in zip(self.names, self.params)],
                            dtype=torch.float32, device=self.device)

    def sync_master_from_model(self):
        if self.local_model is not None:
            self.local_model.copy_(self.local_of(self.model))
        if self.master is not None:
            self.master.copy_(self.shard_model.float())


def _is_native(t: torch.Tensor) -> bool:
    if not t.is_cuda:
        return False
    from cloudtik_amd import ops
    ops.require_native()
    return True


class _FlatOptimizer(torch.optim.Optimizer):
    """Base: keeps torch.optim.Optimizer's param_groups (so LR schedulers work) but steps
    the whole flat space with one fused kernel."""

    def __init__(self, params, defaults, space: Optional[FlatParamSpace] = None,
                 no_decay: Optional[Callable[[str], bool]] = None, names=None):
        if isinstance(params, FlatParamSpace):
            space, params = params, params.params
        params = list(params)
        if params and isinstance(params[0], dict):
            groups = params
        else:
            groups = [{"params": params}]
        super().__init__(groups, defaults)
        if space is None:
            flat = [p for g in self.param_groups for p in g["params"]]
            space = FlatParamSpace(flat, names=names)
        self.space = space
        # per-tensor weight decay from the group each param belongs to
        gwd = {}
        for g in self.param_groups:
            for p in g["params"]:
                gwd[id(p)] = g.get("weight_decay", 0.0)
        self._wd = torch.tensor(
            [0.0 if (no_decay is not None and no_decay(n)) else gwd.get(id(p), defaults.get("weight_decay", 0.0))
             for n, p in zip(space.names, space.params)], dtype=torch.float32, device=space.device)
        self.dyn = torch.zeros(4, dtype=torch.float32, device=space.device)
        # per-step scalars (lr, grad scale, bias corrections) reach the device through a RING of
        # pinned host slots: an async H2D copy reads host memory when it EXECUTES, so a single
        # reused slot would let a CPU that runs ahead overwrite step k's values with step k+1's
        # before the copy ran.  A slot is rewritten only after the event recorded behind its
        # previous copy has completed (blocks only if the CPU is _DYN_SLOTS steps ahead).
        pinned = space.device.type == "cuda"
        self._dyn_ring = [torch.zeros(4, dtype=torch.float32, pin_memory=pinned) for _ in range(_DYN_SLOTS)]
        self._dyn_events = [None] * _DYN_SLOTS
        self._dyn_slot = 0
        self.grad_scale = 1.0
        self.step_count = 0

    def zero_grad(self, set_to_none: bool = False):  # grads live in the flat buffer
        self.space.zero_grad()

    def _lr(self):
        lrs = {g["lr"] for g in self.param_groups}
        if len(lrs) != 1:
            raise ValueError("fused flat optimizers need one learning rate across groups")
        return float(next(iter(lrs)))

    def _dyn_values(self, b1, b2):
        t = self.step_count
        bc1 = 1.0 / (1.0 - b1 ** t) if b1 is not None else 1.0
        bc2 = 1.0 / (1.0 - b2 ** t) if b2 is not None else 1.0
        return [self._lr(), self.grad_scale, bc1, bc2]

    def _push_dyn(self, b1=None, b2=None):
        if self.dyn.is_cuda and torch.cuda.is_current_stream_capturing():
            # hipGraph capture (train.graph_step): the captured copy node re-reads ONE fixed
            # pinned slot at every replay; graph_step_prepare() rewrites it between replays
            if getattr(self, "_graph_host", None) is None:
                raise RuntimeError("call graph_capture_begin() before capturing an optimizer step "
                                   "(pinned memory cannot be allocated while a stream captures)")
            self._graph_betas = (b1, b2)
            self._graph_replays = 0
            self._graph_host.copy_(torch.tensor(self._dyn_values(b1, b2), dtype=torch.float32))
            self.dyn.copy_(self._graph_host, non_blocking=True)
            return
        i = self._dyn_slot = (self._dyn_slot + 1) % _DYN_SLOTS
        host, ev = self._dyn_ring[i], self._dyn_events[i]
        if ev is not None:
            ev.synchronize()
        host.copy_(torch.tensor(self._dyn_values(b1, b2), dtype=torch.float32))
        if self.dyn.is_cuda:
            self.dyn.copy_(host, non_blocking=True)
            if ev is None:
                ev = self._dyn_events[i] = torch.cuda.Event()
            ev.record()
        else:
            self.dyn.copy_(host)

    def graph_capture_begin(self):
        """Allocate the pinned scalar slot a captured step's copy node reads (before capture)."""
        if self.dyn.is_cuda and getattr(self, "_graph_host", None) is None:
            self._graph_host = torch.zeros(4, dtype=torch.float32, pin_memory=True)
            self._graph_done = torch.cuda.Event()

    def graph_step_prepare(self):
        """Before replaying a captured training step (the capture itself ran no kernels): count
        the step and put its scalars (lr, grad scale, bias corrections) where the graph's copy
        node reads them.  The slot is only rewritten -- after the previous replay finished with
        it -- when a value changes (never for a constant-lr SGD)."""
        if getattr(self, "_graph_host", None) is None:
            return
        if self._graph_replays > 0:
            self.step_count += 1
        self._graph_replays += 1
        vals = torch.tensor(self._dyn_values(*self._graph_betas), dtype=torch.float32)
        if not torch.equal(vals, self._graph_host):
            self._graph_done.synchronize()
            self._graph_host.copy_(vals)

    def graph_step_done(self):
        """After a replay was launched: mark where the host slot is free again."""
        if getattr(self, "_graph_host", None) is not None:
            self._graph_done.record()

    def state_dict(self):
        """Flat optimizer state in the GLOBAL layout (ZeRO-1 shards are gathered).

        Parameter offsets inside the flat space depend only on the parameter list and the
        alignment, never on the world size (only the tail padding of ``total`` does), so a
        global-layout state restores onto any sharding / world size: ``load_state_dict``
        re-pads it to the current ``total`` and cuts this rank's pieces out of it.  The
        parameter table is stored with it and checked on load."""
        sd = super().state_dict()
        sp = self.space
        flat = dict(self._flat_state())
        if sp.master is not None:      # fp32 master shard (the bf16 model alone loses bits)
            flat["master"] = sp.master
        if sp.sharded or sp.world == 1:
            sd["flat"] = {k: (sp.full_of(v) if sp.sharded else v) for k, v in flat.items()}
            sd["flat_layout"] = "global"
        else:                          # a contiguous shard that no gather function can rebuild
            sd["flat"] = flat
            sd["flat_layout"] = "shard"
        sd["flat_params"] = {"offsets": list(sp.offsets), "numels": list(sp.numels),
                             "used": sp.used, "world": sp.world}
        sd["step_count"] = self.step_count
        return sd

    def load_state_dict(self, sd):
        """Restore the flat state.  The weights themselves come from the MODEL's state dict
        (parameters are views of ``space.model``), loaded before this: the shard-local copies
        derived from it (ZeRO-1 ``local_model``, the fp32 ``master``) are refreshed here
        first, then the saved fp32 master (if any) overrides the bf16-rounded refresh."""
        sd = dict(sd)
        flat = sd.pop("flat", {})
        layout = sd.pop("flat_layout", "shard")
        table = sd.pop("flat_params", None)
        self.step_count = sd.pop("step_count", 0)
        super().load_state_dict(sd)
        sp = self.space
        if table is not None and (list(table["offsets"]) != list(sp.offsets)
                                  or list(table["numels"]) != list(sp.numels)):
            raise ValueError("optimizer state was saved for a different parameter list")
        if layout == "shard" and table is not None and table["world"] != sp.world:
            raise ValueError(f"shard-layout optimizer state of world size {table['world']} cannot be "
                             f"restored at world size {sp.world}")
        sp.sync_master_from_model()
        for k, v in flat.items():
            dst = sp.master if k == "master" else getattr(self, k)
            v = v.to(dst.device)
            if layout == "global":
                if v.numel() != sp.total:          # saved at another world size: re-pad the tail
                    full = torch.zeros(sp.total, dtype=v.dtype, device=v.device)
                    n = min(sp.used, v.numel())
                    full[:n].copy_(v[:n])
                    v = full
                if dst.numel() != sp.total:
                    v = sp.local_of(v)
            dst.copy_(v)

    def _flat_state(self):
        return {}


class FusedLAMB(_FlatOptimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01,
                 bias_correction=False, trust_all=False, max_grad_norm=None, space=None,
                 no_decay=None, names=None):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay),
                         space, no_decay, names)
        sp = self.space
        n = sp.shard_size
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=sp.device)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=sp.device)
        self.betas, self.eps = betas, eps
        self.bias_correction, self.trust_all = bias_correction, trust_all
        self.max_grad_norm = max_grad_norm
        self.seg_part = torch.zeros(max(1, 2 * sp.nseg), dtype=torch.float32, device=sp.device)
        self.tensor_part = torch.zeros(2 * len(sp.params), dtype=torch.float32, device=sp.device)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=sp.device)
        # per-tensor norm all-reduce over the data-parallel group; ZeRO-1 (space.sharded) sets
        # one on the space, an explicit one here takes precedence
        self.norm_allreduce: Optional[Callable[[torch.Tensor], None]] = None

    def _flat_state(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}

    @torch.no_grad()
    def step(self, closure=None):
        _sync_grads()
        loss = closure() if closure is not None else None
        self.space.flush_grads()
        self.step_count += 1
        sp = self.space
        b1, b2 = self.betas
        self._push_dyn(b1 if self.bias_correction else None, b2 if self.bias_correction else None)
        g = sp.shard_grad
        if self.seg_part.numel() < 2 * sp.nseg:      # segments rebuilt by a ZeRO-1 layout
            self.seg_part = torch.zeros(2 * sp.nseg, dtype=torch.float32, device=sp.device)
        if _is_native(g):
            from cloudtik_amd import ops
            C = ops.require_native()
            nar = self.norm_allreduce or sp.norm_allreduce
            if self.max_grad_norm:
                self._sumsq.zero_()
                C.sumsq_into(g, self._sumsq)
                if nar is not None:
                    nar(self._sumsq)
                C.clip_coef(self._sumsq, self.dyn, float(self.grad_scale), float(self.max_grad_norm))
            wm = sp.shard_model if sp.master is not None else None
            C.lamb_step(g, self.exp_avg, self.exp_avg_sq, sp.shard_params, wm, sp.seg_tensor,
                        sp.seg_start, sp.seg_len, sp.tensor_first_seg, self._wd, self.dyn, b1, b2,
                        self.eps, self.bias_correction, self.trust_all, self.seg_part, self.tensor_part, 1)
            if nar is not None:
                nar(self.tensor_part)
            C.lamb_step(g, self.exp_avg, self.exp_avg_sq, sp.shard_params, wm, sp.seg_tensor,
                        sp.seg_start, sp.seg_len, sp.tensor_first_seg, self._wd, self.dyn, b1, b2,
                        self.eps, self.bias_correction, self.trust_all, self.seg_part, self.tensor_part, 2)
        else:
            self._step_torch(g)
        sp.after_step()
        return loss

    def _step_torch(self, g):
        sp = self.space
        b1, b2 = self.betas
        lr, gs = self._lr(), self.grad_scale
        t = self.step_count
        bc1 = 1.0 / (1.0 - b1 ** t) if self.bias_correction else 1.0
        bc2 = 1.0 / (1.0 - b2 ** t) if self.bias_correction else 1.0
        gf = g.float() * gs
        nar = self.norm_allreduce or sp.norm_allreduce
        if self.max_grad_norm:
            nrm = gf.pow(2).sum()
            if nar is not None:
                buf = nrm.reshape(1).clone()
                nar(buf)
                nrm = buf[0]
            coef = torch.clamp(self.max_grad_norm / (nrm.sqrt() + 1e-6), max=1.0)
            gf = gf * coef
        m, v, w = self.exp_avg, self.exp_avg_sq, sp.shard_params
        m.mul_(b1).add_(gf, alpha=1 - b1)
        v.mul_(b2).addcmul_(gf, gf, value=1 - b2)
        wd = self._per_elem(self._wd)
        u = (m * bc1) / ((v * bc2).sqrt() + self.eps) + wd * w
        T = len(sp.params)
        tid = self._per_elem(torch.arange(T, dtype=torch.float32, device=w.device)).long()
        valid = self._valid_mask()
        tp = torch.zeros(2 * T, dtype=torch.float32, device=w.device)
        tp[0::2].index_add_(0, tid[valid], (w * w)[valid])
        tp[1::2].index_add_(0, tid[valid], (u * u)[valid])
        if nar is not None:
            nar(tp)
        wn, un = tp[0::2].sqrt(), tp[1::2].sqrt()
        ratio = torch.where((wn > 0) & (un > 0), wn / un.clamp_min(1e-30), torch.ones_like(wn))
        if not self.trust_all:
            ratio = torch.where(self._wd != 0, ratio, torch.ones_like(ratio))
        w.sub_(lr * self._per_elem(ratio) * u)
        if sp.master is not None:
            sp.shard_model.copy_(w)

    def _per_elem(self, per_tensor: torch.Tensor) -> torch.Tensor:
        sp = self.space
        if not hasattr(self, "_elem_tid"):
            tid = torch.zeros(sp.shard_size, dtype=torch.long)
            seg_t, seg_s, seg_l = sp._seg_cpu
            valid = torch.zeros(sp.shard_size, dtype=torch.bool)
            for t, s, l in zip(seg_t, seg_s, seg_l):
                tid[s:s + l] = t
                valid[s:s + l] = True
            self._elem_tid = tid.to(sp.device)
            self._elem_valid = valid.to(sp.device)
        return per_tensor[self._elem_tid]

    def _valid_mask(self):
        self._per_elem(self._wd)
        return self._elem_valid


class FusedAdam(_FlatOptimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 adamw=True, space=None, no_decay=None, names=None):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay),
                         space, no_decay, names)
        sp = self.space
        self.exp_avg = torch.zeros(sp.shard_size, dtype=torch.float32, device=sp.device)
        self.exp_avg_sq = torch.zeros(sp.shard_size, dtype=torch.float32, device=sp.device)
        self.betas, self.eps, self.adamw = betas, eps, adamw

    def _flat_state(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}

    @torch.no_grad()
    def step(self, closure=None):
        _sync_grads()
        loss = closure() if closure is not None else None
        self.space.flush_grads()
        self.step_count += 1
        sp = self.space
        b1, b2 = self.betas
        self._push_dyn(b1, b2)
        g = sp.shard_grad
        if _is_native(g):
            from cloudtik_amd import ops
            wm = sp.shard_model if sp.master is not None else None
            ops.require_native().adam_step(g, self.exp_avg, self.exp_avg_sq, sp.shard_params, wm,
                                           sp.seg_tensor, sp.seg_start, sp.seg_len, self._wd, self.dyn,
                                           b1, b2, self.eps, self.adamw)
        else:
            t = self.step_count
            lr, gs = self._lr(), self.grad_scale
            w = sp.shard_params
            wd = LAMBHelper.per_elem(self, self._wd)
            gf = g.float() * gs
            if not self.adamw:
                gf = gf + wd * w
            self.exp_avg.mul_(b1).add_(gf, alpha=1 - b1)
            self.exp_avg_sq.mul_(b2).addcmul_(gf, gf, value=1 - b2)
            upd = (self.exp_avg / (1 - b1 ** t)) / ((self.exp_avg_sq / (1 - b2 ** t)).sqrt() + self.eps)
            if self.adamw:
                upd = upd + wd * w
            w.sub_(lr * upd)
            if sp.master is not None:
                sp.shard_model.copy_(w)
        sp.after_step()
        return loss


class FusedSGD(_FlatOptimizer):
    def __init__(self, params, lr=0.1, momentum=0.9, dampening=0.0, weight_decay=0.0,
                 nesterov=False, space=None, no_decay=None, names=None):
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay),
                         space, no_decay, names)
        sp = self.space
        self.momentum, self.dampening, self.nesterov = momentum, dampening, nesterov
        self.momentum_buffer = torch.zeros(sp.shard_size, dtype=torch.float32, device=sp.device) \
            if momentum else None

    def _flat_state(self):
        return {"momentum_buffer": self.momentum_buffer} if self.momentum_buffer is not None else {}

    @torch.no_grad()
    def step(self, closure=None):
        _sync_grads()
        loss = closure() if closure is not None else None
        self.space.flush_grads()
        self.step_count += 1
        sp = self.space
        self._push_dyn()
        g = sp.shard_grad
        first = self.step_count == 1
        if _is_native(g):
            from cloudtik_amd import ops
            wm = sp.shard_model if sp.master is not None else None
            ops.require_native().sgd_step(g, self.momentum_buffer, sp.shard_params, wm, sp.seg_tensor,
                                          sp.seg_start, sp.seg_len, self._wd, self.dyn,
                                          self.momentum, self.dampening, self.nesterov, first)
        else:
            w = sp.shard_params
            wd = LAMBHelper.per_elem(self, self._wd)
            gf = g.float() * self.grad_scale + wd * w
            if self.momentum:
                b = self.momentum_buffer
                if first:
                    b.copy_(gf)
                else:
                    b.mul_(self.momentum).add_(gf, alpha=1 - self.dampening)
                gf = gf + self.momentum * b if self.nesterov else b
            w.sub_(self._lr() * gf)
            if sp.master is not None:
                sp.shard_model.copy_(w)
        sp.after_step()
        return loss


class LAMBHelper:
    per_elem = FusedLAMB._per_elem
    valid = FusedLAMB._valid_mask


def param_groups_for(model: torch.nn.Module, weight_decay: float,
                     no_decay: Callable[[str], bool]) -> Tuple[list, list]:
    """Reference grouping (run_pretrain_mlperf.py:491-497): decay vs. no-decay groups."""
    named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
    decay = [p for n, p in named if not no_decay(n)]
    nodecay = [p for n, p in named if no_decay(n)]
    return ([{"params": decay, "weight_decay": weight_decay},
             {"params": nodecay, "weight_decay": 0.0}], [n for n, _ in named])


def build_optimizer(name: str, model: torch.nn.Module, lr: float, weight_decay: float = 0.0,
                    no_decay: Optional[Callable[[str], bool]] = None, shard: Tuple[int, int] = (0, 1),
                    **kw):
    named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named], shard=shard)
    nd = no_decay or (lambda n: False)
    cls = {"lamb": FusedLAMB, "adam": FusedAdam, "adamw": FusedAdam, "sgd": FusedSGD}[name.lower()]
    if name.lower() == "adam":
        kw.setdefault("adamw", False)
    return cls(space, lr=lr, weight_decay=weight_decay, space=space, no_decay=nd, **kw)
