"""Autograd front-ends for the HIP op library (GPU) with reference fallbacks (CPU)."""
from __future__ import annotations

import os

import torch

from . import reference as ref

ACT_NONE, ACT_GELU, ACT_RELU = ref.ACT_NONE, ref.ACT_GELU, ref.ACT_RELU


def _pkg():
    from cloudtik_amd import ops
    return ops


def _native(*ts):
    return _pkg()._use_native(*ts)


def _C():
    return _pkg().require_native()


def _opt(t):
    return t if (t is not None and isinstance(t, torch.Tensor)) else None


# ----------------------------------------------------------------------------- LayerNorm
class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, bias, residual, eps, p, seed, offset, rms):
        y, s, mean, rstd = _C().layernorm_fwd(x, bias, residual, gamma, beta, eps, rms, p, seed, offset)
        s_saved = s if s is not None and s.numel() > 0 else x
        ctx.save_for_backward(s_saved, gamma, mean, rstd)
        ctx.cfg = (p, seed, offset, rms, beta is not None, bias is not None, residual is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        s, gamma, mean, rstd = ctx.saved_tensors
        p, seed, offset, rms, has_beta, has_bias, has_res = ctx.cfg
        need_dx = p > 0.0
        ds, dx, dgamma, dbeta, dbias = _C().layernorm_bwd(
            dy.contiguous(), s, gamma, mean, rstd, None, rms, has_beta, has_bias, need_dx, p, seed, offset)
        dx_out = dx if need_dx else ds
        return (dx_out, dgamma, dbeta if has_beta else None, dbias if has_bias else None,
                ds if has_res else None, None, None, None, None, None)


def layer_norm(x, gamma, beta=None, eps=1e-12, bias=None, residual=None, p=0.0,
               training=True, rms=False):
    """y = LayerNorm(residual + dropout(x + bias)) * gamma + beta  (all parts optional)."""
    p = float(p) if training else 0.0
    ops = _pkg()
    if _native(x):
        seed, offset = ops._rng.next(x.numel()) if p > 0 else (0, 0)
        N = x.shape[-1]
        if N % 8 == 0 and N <= 2048 and x.dtype == torch.bfloat16:
            return _LayerNormFn.apply(x.contiguous(), gamma, beta, bias,
                                      residual.contiguous() if residual is not None else None,
                                      float(eps), p, seed, offset, bool(rms))
    else:
        seed, offset = ops._rng.next(x.numel()) if p > 0 else (0, 0)
    y, _ = ref.layer_norm(x, gamma, beta, eps, bias, residual, p, seed, offset, rms)
    return y


# ----------------------------------------------------------------------------- bias + act
class _BiasActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, bias, act):
        ctx.save_for_backward(z, bias)
        ctx.act = act
        ctx.has_bias = bias is not None
        return _C().bias_act_fwd(z, bias, act)

    @staticmethod
    def backward(ctx, dy):
        z, bias = ctx.saved_tensors
        dz, dbias = _C().bias_act_bwd(dy.contiguous(), z, bias, ctx.act, ctx.has_bias)
        return dz, (dbias if ctx.has_bias else None), None


def bias_act(z, bias=None, act=ACT_GELU):
    if _native(z) and z.dtype == torch.bfloat16 and z.shape[-1] % 8 == 0:
        return _BiasActFn.apply(z.contiguous(), bias, int(act))
    return ref.bias_act(z, bias, act)


def bias_gelu(z, bias=None):
    return bias_act(z, bias, ACT_GELU)


# ----------------------------------------------------------------------------- dropout
class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, offset):
        ctx.cfg = (p, seed, offset)
        return _C().dropout_fwd(x, p, seed, offset)

    @staticmethod
    def backward(ctx, dy):
        p, seed, offset = ctx.cfg
        return _C().dropout_fwd(dy.contiguous(), p, seed, offset), None, None, None


def dropout(x, p=0.1, training=True):
    if not training or p <= 0.0:
        return x
    seed, offset = _pkg()._rng.next(x.numel())
    if _native(x) and x.dtype == torch.bfloat16 and x.numel() % 8 == 0:
        return _DropoutFn.apply(x.contiguous(), float(p), seed, offset)
    if x.numel() % 8 == 0:
        return ref.dropout(x, p, seed, offset)
    return torch.nn.functional.dropout(x, p, True)


# ----------------------------------------------------------------------------- embeddings
class _Embed3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tt, W, P, T):
        ctx.save_for_backward(ids, tt)
        ctx.shapes = (W.shape, None if P is None else P.shape, None if T is None else T.shape)
        ctx.dtypes = (W.dtype,)
        ctx.has = (P is not None, T is not None)
        return _C().embed3_fwd(ids, tt, W, P, T)

    @staticmethod
    def backward(ctx, g):
        ids, tt = ctx.saved_tensors
        ws, ps, ts = ctx.shapes
        f32 = dict(dtype=torch.float32, device=g.device)
        dW = torch.zeros(ws, **f32)
        dP = torch.zeros(ps, **f32) if ctx.has[0] else None
        dT = torch.zeros(ts, **f32) if ctx.has[1] else None
        _C().embed3_bwd(ids, tt, g.contiguous(), dW, dP, dT)
        dt = ctx.dtypes[0]
        return (None, None, dW.to(dt), dP.to(dt) if dP is not None else None,
                dT.to(dt) if dT is not None else None)


def embedding3(ids, token_type_ids, W, P=None, T=None):
    """word[ids] + position[arange(S)] + token_type[tt] (sum of up to three tables)."""
    if _native(W) and W.dtype == torch.bfloat16 and W.shape[1] % 8 == 0:
        tt = token_type_ids.contiguous() if (token_type_ids is not None and T is not None) else None
        return _Embed3Fn.apply(ids.contiguous(), tt, W, P, T)
    return ref.embedding3(ids, token_type_ids, W, P, T)


# ----------------------------------------------------------------------------- linear + CE
class _LinearXentFn(torch.autograd.Function):
    """loss = CE(x @ W[:ld].T + b, labels) over valid labels; gradient built in forward."""

    @staticmethod
    def forward(ctx, x, W, b, labels, V, ignore_index, label_smoothing):
        logits = torch.nn.functional.linear(x, W, b)
        valid = (labels != ignore_index).sum().clamp_min(1).to(torch.float32)
        inv = (1.0 / valid).reshape(1)
        loss_rows, _ = _C().xent_fwd(logits, logits, V, labels, inv, ignore_index, label_smoothing)
        ctx.save_for_backward(x, W, logits)   # `logits` now holds d(loss)/d(logits)
        ctx.has_b = b is not None
        return loss_rows.sum() * inv[0]

    @staticmethod
    def backward(ctx, g):
        x, W, dlogits = ctx.saved_tensors
        dx = torch.matmul(dlogits, W) * g.to(dlogits.dtype)
        dW = None
        import importlib
        _lin = importlib.import_module("cloudtik_amd.ops.linear")   # (ops.linear is also a function)
        db = None
        if (_lin._HIP_WGRAD and dlogits.dtype == torch.bfloat16 and W.shape[0] % 256 == 0
                and x.shape[1] % 256 == 0 and x.shape[0] % 64 == 0):
            # decoder weight gradient on the MFMA kernel's TN layout (the vocabulary is padded to
            # a multiple of 256 for it): one split fills ~2 waves of the GPU, bf16 out directly.
            # The decoder bias gradient (column sums of dlogits) comes out of the same kernel
            # (the all-ones MFMA of gemm_tn2_bias) instead of a separate reduction over the
            # whole [rows, vocabulary] gradient (1.2 GB at BERT-large's 19456 x 30720)
            dW = torch.empty_like(W)
            bP = torch.empty(1, W.shape[0], device=W.device, dtype=torch.float32) if ctx.has_b else None
            ok = (_C().gemm_tn2_bias(dlogits, x.contiguous(), dW, 1, False, bP) if ctx.has_b
                  else _C().gemm_tn2(dlogits, x.contiguous(), dW, 1, False))
            if ok:
                if ctx.has_b:
                    db = bP[0].mul_(g).to(dlogits.dtype)
            else:
                dW = None
        if dW is None:
            dW = torch.matmul(dlogits.t(), x)
        dW = dW * g.to(dlogits.dtype)
        if ctx.has_b and db is None:
            db = dlogits.sum(0, dtype=torch.float32).mul_(g).to(dlogits.dtype)
        return dx, dW, db, None, None, None, None


def cross_entropy_fused(x, W, b, labels, V=None, ignore_index=-100, label_smoothing=0.0):
    """Mean cross entropy of ``x @ W.T + b`` against ``labels``.

    ``W`` may have rows padded beyond the true class count ``V`` (rows >= V are masked out
    of the softmax); on the GPU the softmax/NLL/gradient run in one HIP kernel whose
    gradient overwrites the logits buffer in place."""
    V = int(V or W.shape[0])
    if _native(x) and x.dtype == torch.bfloat16 and W.shape[0] % 8 == 0:
        return _LinearXentFn.apply(x.contiguous(), W, b, labels.contiguous(), V, int(ignore_index),
                                   float(label_smoothing))
    logits = torch.nn.functional.linear(x, W, b)
    return ref.cross_entropy(logits, labels, V, ignore_index, label_smoothing)




# ----------------------------------------------------------------------------- batchnorm
# BN + residual + ReLU keeps a ReLU bitmask for its backward instead of re-reading y
_BN_RELU_BITMASK = os.environ.get("CLOUDTIK_AMD_BN_RELU_BITMASK", "1") == "1"


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, run_mean, run_var, relu, momentum, eps):
        has_res = residual is not None
        # ReLU mask for the backward: without a residual it is recomputed from x and the
        # forward's affine coefficients (stat), so y is neither saved nor re-read; with one the
        # forward also writes a bitmask (1 byte per 8 channels, 1/16 of y) that the backward
        # reads instead of y (mode 3; mode 1 = read y itself)
        mode = 0 if not relu else ((3 if _BN_RELU_BITMASK and x.numel() % 8 == 0 else 1) if has_res else 2)
        mask = torch.empty(x.numel() // 8, device=x.device, dtype=torch.uint8) if mode == 3 else None
        given = getattr(x, "_ct_bn_part", None)
        if given is not None:
            # statistics already reduced per tile by the conv that produced x (ops/conv.py)
            y, stat = _C().bn_fwd_train_given(x, residual, gamma, beta, run_mean, run_var, given[0], given[1],
                                              eps, momentum, relu, mask)
        else:
            y, stat = _C().bn_fwd_train(x, residual, gamma, beta, run_mean, run_var, eps, momentum, relu, mask)
        ctx.save_for_backward(x, y if mode == 1 else mask, gamma, stat)
        ctx.params = (gamma, beta)
        ctx.cfg = (mode, has_res)
        ctx.bn_link = None
        if mode != 0 and x.dim() == 4:
            # a conv consuming y may run our backward reduction in its dgrad epilogue (ops/conv.py)
            from cloudtik_amd.ops.conv import BnBwdLink
            ctx.bn_link = BnBwdLink(x, stat, mode, mask)
            y._ct_bn_bwd = ctx.bn_link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, stat = ctx.saved_tensors
        mode, has_res = ctx.cfg
        wp, bp = ctx.params
        flat = all(p is not None and p.grad is not None and getattr(p, "_ct_flat_grad", False)
                   and p.grad.is_contiguous() and p.grad.dtype == gamma.dtype for p in (wp, bp))
        given = ctx.bn_link.take(dy) if ctx.bn_link is not None else None
        if given is not None and dy.is_contiguous(memory_format=torch.channels_last):
            # dy arrives ReLU-masked with its reduction done by the conv's dgrad epilogue
            part, tiles, rows = given
            from cloudtik_amd.ops.conv import flush_deferred_wgrads
            if flat:
                dx, _, _ = _C().bn_bwd_given(dy, x, gamma, stat, part, tiles, rows, wp.grad, bp.grad)
                flush_deferred_wgrads()         # the producing conv's weight gradient (ops/conv.py)
                for p in (wp, bp):
                    cb = getattr(p, "_ct_grad_ready", None)
                    if cb is not None:
                        cb(p)
                # with a residual add the masked dy IS the residual branch's gradient
                return dx, None, None, (dy if has_res else None), None, None, None, None, None
            dx, dg, db = _C().bn_bwd_given(dy, x, gamma, stat, part, tiles, rows, None, None)
            flush_deferred_wgrads()
            return dx, dg, db, (dy if has_res else None), None, None, None, None, None
        if flat:
            # accumulate straight into the flat gradient buffer (no AccumulateGrad kernels)
            dx, dres, _, _ = _C().bn_bwd(dy, y, x, gamma, stat, mode, has_res, wp.grad, bp.grad)
            for p in (wp, bp):
                cb = getattr(p, "_ct_grad_ready", None)
                if cb is not None:
                    cb(p)
            return dx, None, None, (dres if has_res else None), None, None, None, None, None
        dx, dres, dg, db = _C().bn_bwd(dy, y, x, gamma, stat, mode, has_res, None, None)
        return dx, dg, db, (dres if has_res else None), None, None, None, None, None


# BN(x) + BN2(x2) + ReLU in one apply pass when both statistics come from conv epilogues
_BN_ADD_BN_FUSE = os.environ.get("CLOUDTIK_AMD_BN_ADD_BN_FUSE", "1") == "1"
# ... and its two BatchNorm backwards with one apply pass over the masked gradient
_BN_PAIR_BWD = os.environ.get("CLOUDTIK_AMD_BN_PAIR_BWD", "1") == "1"


class _BNAddBNActFn(torch.autograd.Function):
    """``relu(bn(x) + bn2(x2))`` -- a ResNet downsample block's ``bn3(conv3) + down_bn(down)``
    -- with the downsample BatchNorm's output never materialised (batchnorm.hip
    ``bn_apply2_kernel``): forward and gradients are those of ``_BNActFn(x2, relu=False)`` feeding
    ``_BNActFn(x, residual=..., relu=True)`` (bitmask mode), which it replaces."""

    @staticmethod
    def forward(ctx, x, gamma, beta, run_mean, run_var, x2, gamma2, beta2, run_mean2, run_var2, momentum, eps):
        g1, g2 = x._ct_bn_part, x2._ct_bn_part
        y, mask, stat, stat2 = _C().bn_fwd_train_given2(x, gamma, beta, run_mean, run_var, g1[0], g1[1],
                                                         x2, gamma2, beta2, run_mean2, run_var2, g2[0], g2[1],
                                                         eps, momentum)
        ctx.save_for_backward(x, mask, gamma, stat, x2, gamma2, stat2)
        ctx.params = (gamma, beta, gamma2, beta2)
        from cloudtik_amd.ops.conv import BnBwdLink
        ctx.bn_link = BnBwdLink(x, stat, 3, mask)
        y._ct_bn_bwd = ctx.bn_link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, gamma, stat, x2, gamma2, stat2 = ctx.saved_tensors
        wp, bp, wp2, bp2 = ctx.params

        def flat_ok(w, b, g):
            return all(p is not None and p.grad is not None and getattr(p, "_ct_flat_grad", False)
                       and p.grad.is_contiguous() and p.grad.dtype == g.dtype for p in (w, b))

        def ready(*ps):
            for p in ps:
                cb = getattr(p, "_ct_grad_ready", None)
                if cb is not None:
                    cb(p)

        f1, f2 = flat_ok(wp, bp, gamma), flat_ok(wp2, bp2, gamma2)
        given = ctx.bn_link.take(dy)
        dg = db = dg2 = db2 = None
        if (_BN_PAIR_BWD and given is not None and dy.is_contiguous(memory_format=torch.channels_last)
                and f1 == f2 and gamma.dtype == gamma2.dtype):
            # both BatchNorm backwards with ONE apply pass over the masked gradient
            part, tiles, rows = given
            acc = [wp.grad, bp.grad, wp2.grad, bp2.grad] if f1 else [None] * 4
            dx, dx2, dg, db, dg2, db2 = _C().bn_bwd_given_pair(dy, x, gamma, stat, part, tiles, rows, x2, gamma2,
                                                               stat2, *acc)
            from cloudtik_amd.ops.conv import flush_deferred_wgrads
            flush_deferred_wgrads()
            if f1:
                ready(wp, bp, wp2, bp2)
                return dx, None, None, None, None, dx2, None, None, None, None, None, None
            return dx, dg, db, None, None, dx2, dg2, db2, None, None, None, None
        if given is not None and dy.is_contiguous(memory_format=torch.channels_last):
            part, tiles, rows = given
            dym = dy                                   # already ReLU-masked by the conv epilogue
            dx, dg, db = _C().bn_bwd_given(dym, x, gamma, stat, part, tiles, rows,
                                           wp.grad if f1 else None, bp.grad if f1 else None)
            from cloudtik_amd.ops.conv import flush_deferred_wgrads
            flush_deferred_wgrads()
        else:
            dx, dym, dg, db = _C().bn_bwd(dy, mask, x, gamma, stat, 3, True,
                                          wp.grad if f1 else None, bp.grad if f1 else None)
        if f1:
            dg = db = None
            ready(wp, bp)
        # the downsample BatchNorm (no ReLU) sees the masked gradient, as the residual input did
        dx2, _, dg2, db2 = _C().bn_bwd(dym, None, x2, gamma2, stat2, 0, False,
                                       wp2.grad if f2 else None, bp2.grad if f2 else None)
        if f2:
            dg2 = db2 = None
            ready(wp2, bp2)
        return dx, dg, db, None, None, dx2, dg2, db2, None, None, None, None


def batch_norm_add_bn_act(x, weight, bias, running_mean, running_var, x2, weight2, bias2, running_mean2,
                          running_var2, momentum=0.1, eps=1e-5):
    """``relu(bn(x) + bn2(x2))`` in training mode; one apply pass when both inputs carry conv
    epilogue statistics (``_ct_bn_part``), else the two-step form."""
    if (_BN_ADD_BN_FUSE and _native(x) and x.dim() == 4 and x2.shape == x.shape
            and getattr(x, "_ct_bn_part", None) is not None and getattr(x2, "_ct_bn_part", None) is not None
            and x.stride() == x2.stride() and x.numel() % 8 == 0):
        return _BNAddBNActFn.apply(x, weight, bias, running_mean, running_var, x2, weight2, bias2, running_mean2,
                                   running_var2, float(momentum), float(eps))
    idt = batch_norm_act(x2, weight2, bias2, running_mean2, running_var2, relu=False, training=True,
                         momentum=momentum, eps=eps)
    return batch_norm_act(x, weight, bias, running_mean, running_var, residual=idt, relu=True, training=True,
                          momentum=momentum, eps=eps)


def _bn_param_grads(wp, bp, gamma, x, stat, dy, y, mode, has_res):
    """BN backward shared by the BN(+ReLU)(+pool) autograd functions: accumulates the affine
    gradients straight into the flat gradient buffer when the parameters live there."""
    flat = all(p is not None and p.grad is not None and getattr(p, "_ct_flat_grad", False)
               and p.grad.is_contiguous() and p.grad.dtype == gamma.dtype for p in (wp, bp))
    if flat:
        dx, dres, _, _ = _C().bn_bwd(dy, y, x, gamma, stat, mode, has_res, wp.grad, bp.grad)
        for p in (wp, bp):
            cb = getattr(p, "_ct_grad_ready", None)
            if cb is not None:
                cb(p)
        return dx, dres, None, None
    return tuple(_C().bn_bwd(dy, y, x, gamma, stat, mode, has_res, None, None))


# the stem backward's pool gather and BatchNorm reduction in one kernel (batchnorm.hip
# maxpool3s2_bwd_bn_kernel): on by default since its window loads are issued together (the
# separate 308 us reduce pass leaves the backward's tail: 20.56 / 20.60 / 20.57 -> 20.45 / 20.46
# / 20.42 ms same box; before that change it measured neutral)
_STEM_POOL_BN_FUSE = os.environ.get("CLOUDTIK_AMD_STEM_POOL_BN_FUSE", "1") == "1"


class _BNReLUPoolFn(torch.autograd.Function):
    """ResNet stem ``maxpool3x3/s2/p1(relu(bn(x)))`` (batchnorm.hip ``bn_apply_pool_kernel``):
    the full-resolution BN output is never materialised; the backward gathers the pooled
    gradient through the byte argmax and runs the BN backward with the ReLU mask recomputed
    from x."""

    @staticmethod
    def forward(ctx, x, gamma, beta, run_mean, run_var, momentum, eps):
        given = getattr(x, "_ct_bn_part", None)           # the stem conv's epilogue statistics
        if given is not None:
            y, arg, stat = _C().bn_fwd_train_pool_given(x, gamma, beta, run_mean, run_var, given[0], given[1],
                                                        eps, momentum)
        else:
            y, arg, stat = _C().bn_fwd_train_pool(x, gamma, beta, run_mean, run_var, eps, momentum)
        ctx.save_for_backward(x, gamma, stat, arg)
        ctx.params = (gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dyp):
        x, gamma, stat, arg = ctx.saved_tensors
        wp, bp = ctx.params
        if _STEM_POOL_BN_FUSE and x.shape[1] in (8, 16, 32, 64, 128, 256):
            # pool gradient, ReLU mask and the BN-backward sums in one pass (partials per block
            # of input rows), then the finalize + apply of bn_bwd_given: x is not re-read for a
            # reduction
            rows = _C().maxpool3s2_bwd_bn_rows(x.shape[0], x.shape[2])
            part = torch.empty(2 * rows * x.shape[1], device=x.device, dtype=torch.float32)
            dym = _C().maxpool3s2_bwd_bn(dyp, arg, x, stat, part)
            flat = all(p is not None and p.grad is not None and getattr(p, "_ct_flat_grad", False)
                       and p.grad.is_contiguous() and p.grad.dtype == gamma.dtype for p in (wp, bp))
            if flat:
                dx, _, _ = _C().bn_bwd_given(dym, x, gamma, stat, part, rows, rows, wp.grad, bp.grad)
                for p in (wp, bp):
                    cb = getattr(p, "_ct_grad_ready", None)
                    if cb is not None:
                        cb(p)
                return dx, None, None, None, None, None, None
            dx, dg, db = _C().bn_bwd_given(dym, x, gamma, stat, part, rows, rows, None, None)
            return dx, dg, db, None, None, None, None
        dy = _C().maxpool3s2_bwd(dyp, arg, x.shape[2], x.shape[3])
        dx, _, dg, db = _bn_param_grads(wp, bp, gamma, x, stat, dy, None, 2, False)
        return dx, dg, db, None, None, None, None


# the ResNet stem's BatchNorm backward folded into the stem conv's weight gradient (_StemBlockFn).
# Opt-in: the backward's tail loses its apply pass, but G2 (as much MFMA work as the weight
# gradient itself) then runs during the forward, where nothing else is on the side stream:
# 20.44 / 20.46 / 20.46 -> 20.53 / 20.57 / 20.56 ms (profiles/r5/stem_pairs.md)
_STEM_FOLD = os.environ.get("CLOUDTIK_AMD_STEM_FOLD", "0") == "1"


def _stem_tap_colsum(x4, c, R, S, stride, padding):
    """G0[ch, r, s] = sum over the batch and the output pixels of the input at tap (r, s): the
    column sums of the stem conv's implicit im2col matrix (zero padding included), fp32."""
    xs = x4.sum(0, dtype=torch.float32)[:c]                   # [c, H, W]
    xp = torch.nn.functional.pad(xs, (padding[1], padding[1], padding[0], padding[0]))
    cols = torch.nn.functional.unfold(xp.unsqueeze(0), (R, S), stride=stride)   # [1, c R S, L]
    return cols.sum(-1).view(c, R, S)


class _StemBlockFn(torch.autograd.Function):
    """ResNet stem ``maxpool3x3/s2(relu(bn(conv7x7/s2(x))))`` with the BatchNorm backward folded
    into the conv's weight gradient.  The stem conv's input needs no gradient, so the BatchNorm
    input gradient dx = ca dym + c1 y + c0 (per-channel coefficients of the backward, dym the
    masked pooled gradient, y the conv output) only feeds dW = sum_p dx (x) X, which splits into

        dW = ca G1 + c1 G2 + c0 G0,   G1 = sum dym (x) X,  G2 = sum y (x) X,  G0 = sum X

    G2 and G0 depend on the forward only: they run on the gradient side stream during the step.
    The backward's tail is then the fused pool-gradient + BatchNorm-sums pass, the coefficient
    finalize and G1 -- no BatchNorm apply pass over the 411 MB activation (with the old chain:
    pool gradient, BatchNorm reduce, apply, weight gradient)."""

    @staticmethod
    def forward(ctx, x4, w, gamma, beta, run_mean, run_var, momentum, eps, stride, padding):
        from cloudtik_amd.ops import conv as CV
        from cloudtik_amd.ops.linear import grad_stream
        y = CV.stem_fwd(x4, w, stride, padding, partials=True)
        part, rows = y._ct_bn_part
        yp, arg, stat = _C().bn_fwd_train_pool_given(y, gamma, beta, run_mean, run_var, part, rows, eps, momentum)
        ctx.save_for_backward(x4, y, arg, stat, gamma)
        ctx.cfg = (tuple(w.shape), stride, padding)
        ctx.wp, ctx.params = w, (gamma, beta)
        ctx.g = None
        if ctx.needs_input_grad[1]:
            side = grad_stream()
            side.wait_stream(torch.cuda.current_stream())
            co, c, R, S = w.shape
            with torch.cuda.stream(side):
                g2 = CV.stem_wgrad(y, x4, tuple(w.shape), stride, padding, fp32=True, blocks=256)
                g0 = _stem_tap_colsum(x4, c, R, S, stride, padding)
                ev = torch.cuda.Event()
                ev.record(side)
            y.record_stream(side)
            x4.record_stream(side)
            ctx.g = (g2, g0, ev)
        return yp

    @staticmethod
    def backward(ctx, dyp):
        from cloudtik_amd.ops import conv as CV
        x4, y, arg, stat, gamma = ctx.saved_tensors
        wp, bp = ctx.params
        w_shape, stride, padding = ctx.cfg
        C = _C()
        rows = C.maxpool3s2_bwd_bn_rows(y.shape[0], y.shape[2])
        part = torch.empty(2 * rows * y.shape[1], device=y.device, dtype=torch.float32)
        dym = C.maxpool3s2_bwd_bn(dyp.contiguous(memory_format=torch.channels_last), arg, y, stat, part)
        M = y.numel() // y.shape[1]
        flat = all(p is not None and p.grad is not None and getattr(p, "_ct_flat_grad", False)
                   and p.grad.is_contiguous() and p.grad.dtype == gamma.dtype for p in (wp, bp))
        dg, db, coef = C.bn_bwd_coefs_given(M, gamma, stat, part, rows, rows, wp.grad if flat else None,
                                            bp.grad if flat else None)
        if flat:
            for p in (wp, bp):
                cb = getattr(p, "_ct_grad_ready", None)
                if cb is not None:
                    cb(p)
            dg = db = None
        dw = None
        if ctx.g is not None:
            g2, g0, ev = ctx.g
            g1 = CV.stem_wgrad(dym, x4, w_shape, stride, padding, fp32=True)
            cur = torch.cuda.current_stream()
            cur.wait_event(ev)
            g2.record_stream(cur)
            g0.record_stream(cur)
            ca, c1, c0 = (t.view(-1, 1, 1, 1) for t in coef.view(3, -1))
            dwf = ca * g1 + c1 * g2 + c0 * g0.unsqueeze(0)
            dw = dwf.to(ctx.wp.dtype).contiguous(memory_format=torch.channels_last)
            ctx.g = None
            from cloudtik_amd.ops.conv1x1 import _flat_target
            target = _flat_target(ctx.wp)
            if target is not None:                    # straight into the flat gradient buffer
                target.add_(dw)
                cb = getattr(ctx.wp, "_ct_grad_ready", None)
                if cb is not None:
                    cb(ctx.wp)
                dw = None
        return None, dw, dg, db, None, None, None, None, None, None


def stem_block(x, conv, bn):
    """``max_pool2d(relu(bn(conv(x))), 3, 2, 1)`` for the ResNet stem in training, with the
    BatchNorm backward folded into the conv weight gradient (_StemBlockFn) when the pieces are
    on their native paths; None when not eligible (the caller composes the ops itself)."""
    from cloudtik_amd.ops import conv as CV
    w = conv.weight
    if not (_STEM_FOLD and bn.training and _native(w) and CV.stem_eligible(x, conv)
            and CV.stem_pairs(x.shape, w.shape, tuple(conv.stride), tuple(conv.padding))
            and w.shape[0] in (8, 16, 32, 64, 128, 256) and bn.weight is not None and bn.bias is not None
            and bn.running_mean is not None and bn.weight.dtype == torch.bfloat16):
        return None
    CV.ROUTES["igemm"] += 1
    x4 = CV.to_nhwc8(x, 4)
    return _StemBlockFn.apply(x4, w, bn.weight, bn.bias, bn.running_mean, bn.running_var, float(bn.momentum),
                              float(bn.eps), tuple(conv.stride), tuple(conv.padding))


def batch_norm_relu_maxpool(x, weight, bias, running_mean, running_var, training=True, momentum=0.1, eps=1e-5):
    """``max_pool2d(relu(BatchNorm(x)), 3, 2, 1)`` -- fused on GPU in training (NHWC bf16)."""
    if _native(x) and _bn_native_ok(x) and x.dim() == 4 and training:
        return _BNReLUPoolFn.apply(x, weight, bias, running_mean, running_var, float(momentum), float(eps))
    y = batch_norm_act(x, weight, bias, running_mean, running_var, relu=True, training=training,
                       momentum=momentum, eps=eps)
    return torch.nn.functional.max_pool2d(y, 3, 2, 1)


class _BNAffineFn(torch.autograd.Function):
    """Frozen BatchNorm (running statistics) + residual + ReLU with autograd: the forward is
    the fused ``bn_apply`` HIP kernel; the backward is ``dy * relu_mask * scale`` (the affine
    parameters are frozen, so no parameter gradients)."""

    @staticmethod
    def forward(ctx, x, a, b, residual, relu):
        res = residual.contiguous(memory_format=torch.channels_last) if (residual is not None and x.dim() == 4) \
            else residual
        y = _C().bn_apply(x, res, a, b, bool(relu))
        ctx.save_for_backward(y if relu else torch.empty(0), a)
        ctx.cfg = (relu, residual is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, a = ctx.saved_tensors
        relu, has_res = ctx.cfg
        g = dy * (y > 0) if relu else dy
        shape = (1, -1, 1, 1) if dy.dim() == 4 else (1, -1)
        dx = g * a.view(shape).to(g.dtype)
        return dx, None, None, (g if has_res else None), None


def _bn_native_ok(x):
    if x.dtype != torch.bfloat16 or x.dim() not in (2, 4):
        return False
    C = x.shape[1]
    if C % 8 or C > 2048:
        return False
    return x.is_contiguous(memory_format=torch.channels_last) if x.dim() == 4 else x.is_contiguous()


def batch_norm_act(x, weight, bias, running_mean, running_var, residual=None, relu=True,
                   training=True, momentum=0.1, eps=1e-5):
    """relu(BatchNorm(x) + residual) over NHWC/channels_last bf16 (training: batch stats)."""
    if _native(x) and _bn_native_ok(x) and training and (
            residual is None or residual.is_contiguous(memory_format=torch.channels_last)
            or (x.dim() == 2 and residual.is_contiguous())):
        return _BNActFn.apply(x, weight, bias, residual, running_mean, running_var, bool(relu),
                              float(momentum), float(eps))
    if _native(x) and _bn_native_ok(x) and not training and not torch.is_grad_enabled():
        a = weight.float() * torch.rsqrt(running_var + eps)
        b = bias.float() - running_mean * a
        res = residual.contiguous(memory_format=torch.channels_last) if (residual is not None and x.dim() == 4) else residual
        return _C().bn_apply(x, res, a.contiguous(), b.contiguous(), bool(relu))
    if _native(x) and _bn_native_ok(x) and not training and not (weight.requires_grad or bias.requires_grad):
        # frozen BN inside a trained network (detection backbones)
        with torch.no_grad():
            a = (weight.float() * torch.rsqrt(running_var + eps)).contiguous()
            b = (bias.float() - running_mean * a).contiguous()
        return _BNAffineFn.apply(x, a, b, residual, bool(relu))
    if x.dtype != running_mean.dtype:
        y = torch.nn.functional.batch_norm(x.float(), running_mean, running_var, weight.float(), bias.float(),
                                           training, momentum, eps).to(x.dtype)
        if residual is not None:
            y = y + residual
        return torch.relu(y) if relu else y
    y = torch.nn.functional.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if relu else y
