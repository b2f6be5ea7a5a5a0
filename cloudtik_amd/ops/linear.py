"""Linear layer with the weight-gradient GEMM accumulating straight into the flat gradient
buffer ("gradient-accumulation fusion").

With PyTorch's stock ``F.linear`` backward, dW is produced into a fresh tensor and then
``AccumulateGrad`` adds it into ``param.grad`` -- one extra read-read-write pass over every
weight per step (the flat buffer of train.optim.FlatParamSpace is pre-set as ``.grad``).
Here the backward issues ``grad.addmm_(dY^T, X)`` instead: hipBLASLt's beta=1 epilogue does
the accumulation inside the GEMM, and no extra elementwise kernel runs.  Because autograd
then never sees a weight gradient, the data-parallel bucketer is notified explicitly
(``param._ct_grad_ready``, installed by parallel.ddp.GradBucketer).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

# bias gradients out of the MFMA weight-gradient GEMM (extra all-ones MFMA; ops/csrc/gemm_nt.hip)
_WGRAD_BIAS_FUSE = os.environ.get("CLOUDTIK_AMD_WGRAD_BIAS_FUSE", "1") == "1"
# split-K for weight-gradient GEMMs: 0 disables, otherwise the maximum split factor
_SPLITK_MAX = int(os.environ.get("CLOUDTIK_AMD_WGRAD_SPLITK", "8"))

# Weight-gradient GEMMs on a side HIP stream: they depend only on (dY, X) and write disjoint
# slices of the flat gradient buffer, so they can run concurrently with the dgrad chain of the
# backward pass (filling the CUs the dgrad GEMM's last wave leaves idle).  Consumers of the
# gradients -- the bucketed all-reduce and the optimizer -- order themselves after this
# stream via ``sync_grad_stream()``.
#
# The choice is a property of each weight (``param._ct_wgrad_side``, set per model by
# ``use_wgrad_side_stream``), read by the backward that produces its gradient: two models in
# one process keep their own routing, and nothing a model builder does changes another
# model's backward.  CLOUDTIK_AMD_WGRAD_STREAM (0 / 1) pins it for every model.
_WGRAD_STREAM_ENV = os.environ.get("CLOUDTIK_AMD_WGRAD_STREAM")
_DEFAULT_SIDE = (_WGRAD_STREAM_ENV or "1") == "1"
# weight-gradient GEMMs through the MFMA kernel's TN layout (csrc/gemm_nt.hip, ct_gemm_tn2)
# instead of hipBLASLt's batched split-K GEMM: 13-17 % faster per BERT-large layer
# (bench/gemm_tn2_probe.py); "blas" restores hipBLASLt
_HIP_WGRAD = os.environ.get("CLOUDTIK_AMD_WGRAD_KERNEL", "hip") == "hip"
# split-K partial GEMMs through the binding's strided-batched hipBLASLt call whose algorithm is
# chosen by timing every solution once per shape (torch.bmm's heuristic pick is not tuned:
# TunableOp skips bf16 -> fp32 batched GEMMs)
_LT_WGRAD = os.environ.get("CLOUDTIK_AMD_WGRAD_LT", "0") == "1"
_streams = {}


def grad_stream():
    """The side stream used for weight-gradient GEMMs on the current device (or None
    without a GPU).  Created on first use; cached per device."""
    if not torch.cuda.is_available():
        return None
    dev = torch.cuda.current_device()
    s = _streams.get(dev)
    if s is None:
        s = _streams[dev] = torch.cuda.Stream(device=dev)
    return s


def use_wgrad_side_stream(params, enabled: Optional[bool]) -> bool:
    """A model's weight-gradient routing: ``params`` (an ``nn.Module`` or an iterable of
    parameters) get their gradients on the side stream when ``enabled`` (None: the process
    default), unless CLOUDTIK_AMD_WGRAD_STREAM pins it.  Worth it where the backward's
    critical path is memory-bound (ResNet-50: BatchNorm passes; the side stream saves 2.0 ms
    of 24.0 per step), not where it is two compute-bound GEMM streams competing for the
    matrix cores (BERT-large: 71.3 ms with it, 70.6 without; profiles/r4/bert_rejected_r4.md).
    Returns the setting in force."""
    val = _DEFAULT_SIDE if (_WGRAD_STREAM_ENV is not None or enabled is None) else bool(enabled)
    it = params.parameters() if hasattr(params, "parameters") else params
    for p in it:
        p._ct_wgrad_side = val
    return val


def wgrad_side(p) -> bool:
    """Whether parameter ``p``'s weight gradient goes to the side stream."""
    v = getattr(p, "_ct_wgrad_side", None)
    return _DEFAULT_SIDE if v is None else bool(v)


def sync_grad_stream() -> None:
    """Make the current stream wait for every weight gradient issued so far."""
    s = _streams.get(torch.cuda.current_device()) if torch.cuda.is_available() else None
    if s is not None:
        torch.cuda.current_stream().wait_stream(s)


_end_of_backward_sync_queued = False


def _join_grad_stream():
    """Autograd final callback: the streams that read gradients after ``backward()`` returns
    wait (on the GPU, no host sync) for every weight gradient issued on the side stream, so a
    plain ``param.grad`` read -- clipping, logging, a test -- never races the side stream."""
    global _end_of_backward_sync_queued
    _end_of_backward_sync_queued = False
    s = _streams.get(torch.cuda.current_device())
    if s is None:
        return
    cur = torch.cuda.current_stream()
    cur.wait_stream(s)
    default = torch.cuda.default_stream()
    if default != cur and not torch.cuda.is_current_stream_capturing():
        default.wait_stream(s)


def side_grad_stream():
    """``grad_stream()`` for work issued from inside a backward pass: the first call of a
    backward also queues the end-of-backward join (``_join_grad_stream``)."""
    global _end_of_backward_sync_queued
    s = grad_stream()
    if s is not None and not _end_of_backward_sync_queued and torch._C._current_graph_task_id() != -1:
        torch.autograd.Variable._execution_engine.queue_callback(_join_grad_stream)
        _end_of_backward_sync_queued = True
    return s


def wgrad_on_side_stream(g: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor,
                         dbias: Optional[torch.Tensor] = None, enabled: bool = True) -> bool:
    """Issue ``g += dy2^T x2`` (and ``dbias += column sums of dy2``) on the gradient side
    stream; False (nothing issued) when ``enabled`` is False or there is no GPU."""
    s = side_grad_stream() if (g.is_cuda and enabled) else None
    if s is None:
        return False
    cur = torch.cuda.current_stream()
    s.wait_stream(cur)                       # dY / X produced (and grad zeroed) on the main stream
    with torch.cuda.stream(s):
        wgrad_accumulate(g, dy2, x2, dbias)
    dy2.record_stream(s)
    x2.record_stream(s)
    return True


def splitk_factor(T: int, N: int, K: int) -> int:
    """Split factor for dW[N,K] = dY[T,N]^T X[T,K].  hipBLASLt's 256x256 macro-tiles give only
    ceil(N/256)*ceil(K/256) workgroups (16..192 for BERT-large), far fewer than the 256 CUs;
    splitting the T reduction S ways multiplies the workgroup count (measured on MI355X,
    bench/gemm_bench.py: 1024x1024 wgrad 0.51 -> 0.81 PF/s at S=8, 3072x1024 0.67 -> 0.89)."""
    tiles = -(-N // 256) * -(-K // 256)
    S = 1
    while tiles * S < 256 and S < _SPLITK_MAX:
        S *= 2
    while S > 1 and (T % S or T // S < 2048):
        S //= 2
    return S


def tn2_splits(T: int, N: int, K: int, cus: int = 256) -> int:
    """Split factor for the MFMA wgrad kernel (any S: the kernel deals the T / 64 K-tiles out
    over the slices).  Modelled time = K loop + fp32 slab round trip:
      loop(S) = t_full * waves(S) * cus / (tiles * S), waves = ceil(tiles * S / cus), with
      t_full the loop time at a perfect spread (2 N K T at ~1.3 PF/s, measured K-loop rate);
      slab(S) = S * tiles * 256 KiB * 2 (written, read back by the reduce) at ~5 TB/s (0 at S=1).
    BERT-large: qkv 48 tiles -> 5 (240 workgroups, one wave; 16 power-of-two slices cost 3x the
    slab bytes), proj 16 tiles -> 16, FFN 64 tiles -> 4.  >= 512 tokens per slice."""
    tiles = (N // 256) * (K // 256)
    if tiles <= 0 or T % 64:
        return 1
    t_full = 2.0 * N * K * T / 1.3e15
    best, best_cost = 1, None
    for S in range(1, 33):
        if S > 1 and (T // S < 512 or T // 64 < S):
            continue
        waves = -(-tiles * S // cus)
        cost = t_full * waves * cus / (tiles * S) + (S * tiles * 262144 * 2 / 5e12 if S > 1 else 0.0)
        if best_cost is None or cost < best_cost * (1 - 1e-9):
            best, best_cost = S, cost
    return best


def _bias_colsum(dbias: torch.Tensor, dy2: torch.Tensor) -> None:
    """dbias += column sums of dy2 (fp32 accumulation)."""
    if dbias.is_cuda and dbias.dtype == torch.bfloat16 and dbias.is_contiguous() and dy2.shape[1] % 8 == 0:
        from cloudtik_amd import ops
        ops.require_native().bias_act_bwd_into(dy2.contiguous(), dy2.contiguous(), None, 0, dbias, False)
    else:
        dbias.add_(dy2.float().sum(0).to(dbias.dtype))


def wgrad_accumulate(g: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor,
                     dbias: Optional[torch.Tensor] = None) -> None:
    """g += dy2^T x2 (bf16 g, fp32 accumulation); with ``dbias``, also dbias += column sums of
    dy2 (the bias gradient).  The MFMA kernel's TN layout with split-K fp32 slabs + one fused
    reduce-accumulate kernel (or, unsplit, accumulating straight into g), the bias sums coming
    out of the same kernel (one extra MFMA per A fragment against an all-ones operand);
    otherwise hipBLASLt's batched split-K GEMM, or its beta=1 epilogue when one split fills
    the GPU, plus a column-sum kernel for the bias."""
    T, N = dy2.shape
    K = x2.shape[1]
    if (_HIP_WGRAD and g.is_cuda and g.dtype == torch.bfloat16 and dy2.dtype == torch.bfloat16
            and N % 256 == 0 and K % 256 == 0 and T % 64 == 0):
        from cloudtik_amd import ops
        C = ops.require_native()
        S = tn2_splits(T, N, K)
        dy2c, x2c = dy2.contiguous(), x2.contiguous()
        fuse_bias = (_WGRAD_BIAS_FUSE and dbias is not None and dbias.dtype == torch.bfloat16
                     and dbias.is_contiguous())
        bP = torch.empty(S, N, device=g.device, dtype=torch.float32) if fuse_bias else None
        out = g if S == 1 else torch.empty(S, N, K, device=g.device, dtype=torch.float32)
        ok = (C.gemm_tn2_bias(dy2c, x2c, out, S, S == 1, bP) if fuse_bias
              else C.gemm_tn2(dy2c, x2c, out, S, S == 1))
        if ok:
            if S > 1 and fuse_bias:
                C.splitk_reduce2(out, g, bP, dbias, True)     # slabs + bias partials, one launch
            elif S > 1:
                C.splitk_reduce(out, g, True)
            elif fuse_bias:
                C.splitk_reduce(bP, dbias, True)
            if dbias is not None and not fuse_bias:
                _bias_colsum(dbias, dy2)
            return
    if dbias is not None:
        _bias_colsum(dbias, dy2)
    S = splitk_factor(T, N, K) if (g.is_cuda and g.dtype == torch.bfloat16 and g.is_contiguous()) else 1
    if S == 1:
        g.addmm_(dy2.t(), x2)
        return
    from cloudtik_amd import ops
    dy2 = dy2.contiguous()
    x2 = x2.contiguous()
    if _LT_WGRAD:
        C = ops.require_native()
        Ts = T // S
        P = torch.empty(S, N, K, device=g.device, dtype=torch.float32)
        # P[s] = dy2[s*Ts:(s+1)*Ts]^T @ x2[s*Ts:(s+1)*Ts]
        if C.lt_bmm_tuned(dy2[:Ts], x2[:Ts], P[0], True, False, S, Ts * N, Ts * K, N * K, 0) >= 0:
            C.splitk_reduce(P, g, True)
            return
    P = torch.bmm(dy2.view(S, T // S, N).transpose(1, 2), x2.view(S, T // S, K), out_dtype=torch.float32)
    ops.require_native().splitk_reduce(P, g, True)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.weight_param = weight
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        Wp = ctx.weight_param
        out_f, in_f = W.shape
        dy2 = dy.reshape(-1, out_f)
        x2 = x.reshape(-1, in_f)
        dx = torch.matmul(dy, W) if ctx.needs_input_grad[0] else None
        dW = None
        if ctx.needs_input_grad[1]:
            g = Wp.grad
            if g is not None and getattr(Wp, "_ct_flat_grad", False) and g.dtype == dy.dtype:
                if not wgrad_on_side_stream(g, dy2, x2, enabled=wgrad_side(Wp)):
                    wgrad_accumulate(g, dy2, x2)
                cb = getattr(Wp, "_ct_grad_ready", None)
                if cb is not None:
                    cb(Wp)
            else:
                dW = torch.matmul(dy2.t(), x2)
        db = dy2.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dW, db


def linear(x, weight, bias=None):
    """y = x @ weight^T + bias with flat-buffer weight-gradient accumulation on GPU.

    Assumes ``weight`` is used by exactly one ``linear`` call per backward pass (its
    readiness is reported to the gradient bucketer when this GEMM has been issued); use
    ``F.linear`` for shared/tied weights."""
    if x.is_cuda and weight.requires_grad and torch.is_grad_enabled():
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)
