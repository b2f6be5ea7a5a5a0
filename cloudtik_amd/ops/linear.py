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

import torch
import torch.nn.functional as F


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
                g.addmm_(dy2.t(), x2)
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
