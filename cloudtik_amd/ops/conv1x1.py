"""Stride-1 1x1 convolutions over NHWC activations as plain GEMMs, with the residual-gradient
sum folded into the data-gradient GEMM.

In channels_last a 1x1 stride-1 convolution is a GEMM over the ``[N*H*W, C]`` rows of the
activation: ``Y = X W^T``, ``dX = dY W``, ``dW = dY^T X``.  Measured on MI355X over every
1x1 shape of ResNet-50 at batch 256 (``bench/conv1x1_gemm_probe.py``,
``profiles/r2/conv1x1_gemm.md``):

* dgrad: hipBLASLt beats MIOpen's implicit-GEMM kernels once the output has >= 128 channels
  (28x28 512->128: 0.085 vs 0.162 ms); MIOpen stays ahead for 64-channel outputs;
* fwd: hipBLASLt is ahead for >= 1024 input channels, MIOpen's CK kernels below;
* wgrad: the reduction runs over N*H*W (up to 802816) rows into a small output; MIOpen is
  ahead at every shape (hipBLASLt's split-K path included), so it stays on MIOpen.

``keep_input=True`` also returns an alias of ``x`` for the block's other consumer (the
residual / downsample branch).  Autograd then sees ``x`` used once, and the backward adds the
alias gradient into the data-gradient GEMM's output (hipBLASLt beta=1 on the freshly produced
residual gradient) instead of autograd summing the two branch gradients with a separate
elementwise kernel (16 such adds per ResNet-50 step).

Stride-1 3x3 convolutions (``conv3x3``) keep MIOpen for fwd and wgrad but issue the data
gradient as a forward convolution of dY with the flipped, transposed filter
(``dX = conv2d(dY, flip(W)^T, pad 1)``): MIOpen's forward kernels beat its backward-data
kernels at every ResNet-50 3x3 shape (``bench/conv3x3_dgrad_probe.py``: 1.90 -> 1.45 ms per
step).

Parity: the reference trains torchvision's ``resnet50`` (nn.Conv2d everywhere;
applications/ai/quickstart/models/image_recognition/pytorch/common/main.py:276-296); the
module structure and state dict here are unchanged -- only the kernels differ.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

_ENABLED = os.environ.get("CLOUDTIK_AMD_CONV1X1_GEMM", "1") == "1"
_DGRAD_AS_FWD = os.environ.get("CLOUDTIK_AMD_CONV3X3_DGRAD_FWD", "1") == "1"
# conv weight gradients on the gradient side stream (ops.linear.grad_stream), accumulated
# straight into the flat gradient buffer: MIOpen's wgrad kernels (and their zero-fill / cast
# helpers) overlap the bandwidth-bound BatchNorm backward and dgrad chain on the main stream
_SIDE_WGRAD = os.environ.get("CLOUDTIK_AMD_CONV_WGRAD_STREAM", "1") == "1"
DGRAD_GEMM_MIN_CIN = 128
FWD_GEMM_MIN_CIN = 1024


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last -> the [N*H*W, C] row view (a copy only if not NHWC-dense)."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _nchw(rows: torch.Tensor, N: int, H: int, W: int) -> torch.Tensor:
    return rows.view(N, H, W, rows.shape[1]).permute(0, 3, 1, 2)


def _conv_bwd(dy, x, w, mask, pad=0):
    return torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [pad, pad], [1, 1], False, [0, 0], 1, mask)


def _flat_target(wp):
    """The flat-buffer gradient slice of parameter ``wp`` (train.optim.FlatParamSpace), if any."""
    v = getattr(wp, "_ct_flat_view", None)        # deferred conv grads: .grad stays unset
    if v is not None:
        return v
    if getattr(wp, "_ct_flat_grad", False) and wp.grad is not None:
        return wp.grad
    return None


def _weight_grad(wp, dy, x, w, pad):
    """MIOpen dW.  When the weight lives in a flat gradient buffer and the gradient side
    stream is on, it is computed there and added into the buffer (returns None: autograd
    never sees it, so the data-parallel bucketer is told via ``_ct_grad_ready``); otherwise
    it is returned for AccumulateGrad."""
    from cloudtik_amd.ops.linear import side_grad_stream, wgrad_side
    target = _flat_target(wp) if (_SIDE_WGRAD and wgrad_side(wp)) else None
    side = side_grad_stream() if target is not None else None
    if side is None:
        return _conv_bwd(dy, x, w, [False, True, False], pad)[1]
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        target.add_(_conv_bwd(dy, x, w, [False, True, False], pad)[1])
    dy.record_stream(side)
    x.record_stream(side)
    cb = getattr(wp, "_ct_grad_ready", None)
    if cb is not None:
        cb(wp)
    return None


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, keep_input):
        ctx.save_for_backward(x, w)
        ctx.wp = w
        N, C, H, W = x.shape
        co = w.shape[0]
        if C >= FWD_GEMM_MIN_CIN:
            y = _nchw(torch.mm(_rows(x), w.reshape(co, C).t()), N, H, W)
        else:
            y = F.conv2d(x, w)
        if keep_input:
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dx_other=None):
        x, w = ctx.saved_tensors
        N, C, H, W = x.shape
        co = w.shape[0]
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dy2 = _rows(dy)
            w2 = w.reshape(co, C)
            if dx_other is not None and not torch.is_grad_enabled() and dx_other.dtype == dy.dtype \
                    and dx_other.is_contiguous(memory_format=torch.channels_last):
                # the other branch's gradient is a fresh tensor owned by this backward:
                # accumulate the dgrad GEMM into it (beta = 1) -- no separate add kernel
                dx = dx_other
                _rows(dx).addmm_(dy2, w2)
            else:
                if C >= DGRAD_GEMM_MIN_CIN:
                    dx = _nchw(torch.mm(dy2, w2), N, H, W)
                else:
                    dx = _conv_bwd(dy, x, w, [True, False, False])[0]
                if dx_other is not None:
                    dx = dx + dx_other
        if ctx.needs_input_grad[1]:
            dw = _weight_grad(ctx.wp, dy, x, w, 0)
        return dx, dw, None


def conv1x1_eligible(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    return (_ENABLED and x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16
            and conv.weight.dtype == x.dtype and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and x.is_contiguous(memory_format=torch.channels_last))


def conv1x1(x: torch.Tensor, conv: torch.nn.Conv2d, keep_input: bool = False):
    """``conv(x)`` for a stride-1 1x1 bias-free conv over channels_last bf16 on GPU (GEMM
    paths above); with ``keep_input`` returns ``(conv(x), x_alias)`` where ``x_alias`` must be
    used in place of ``x`` by every other consumer.  Anything else falls back to ``conv(x)``."""
    if not conv1x1_eligible(x, conv):
        return (conv(x), x) if keep_input else conv(x)
    return _Conv1x1Fn.apply(x, conv.weight, keep_input)


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        ctx.wp = w
        return F.conv2d(x, w, padding=1)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
            dx = F.conv2d(dy, wt, padding=1)
        if ctx.needs_input_grad[1]:
            dw = _weight_grad(ctx.wp, dy, x, w, 1)
        return dx, dw


def conv3x3_eligible(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    return (_ENABLED and _DGRAD_AS_FWD and x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16
            and conv.weight.dtype == x.dtype and conv.kernel_size == (3, 3) and conv.stride == (1, 1)
            and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and x.is_contiguous(memory_format=torch.channels_last))


def conv3x3(x: torch.Tensor, conv: torch.nn.Conv2d):
    """``conv(x)`` for a stride-1 pad-1 3x3 bias-free conv over channels_last bf16 on GPU with
    the data gradient as a forward convolution; anything else falls back to ``conv(x)``."""
    if not conv3x3_eligible(x, conv):
        return conv(x)
    return _Conv3x3Fn.apply(x, conv.weight)
