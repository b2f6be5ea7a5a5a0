"""Hand-scheduled post-LN transformer encoder blocks (forward + backward).

Each block is ONE autograd node with a hand-written backward, so that

* the residual branch's gradient is added inside a GEMM epilogue
  (``dx = addmm(d_residual, d_qkv, W_qkv)``: hipBLASLt beta=1) instead of by the autograd
  engine's separate elementwise add (2 x [tokens, hidden] per layer);
* weight gradients are accumulated by the wgrad GEMMs straight into the flat gradient
  buffer (``grad.addmm_``) and every LayerNorm / bias gradient is accumulated by the
  LayerNorm / bias-GELU backward kernels into the same buffer -- no AccumulateGrad kernels;
* the data-parallel bucketer is told the moment a parameter's gradient has been issued
  (``param._ct_grad_ready``), so RCCL all-reduces overlap the rest of backward.

Block structure (BERT / HF BertLayer, reference run_pretrain_mlperf.py:449-471):

  attention block:  x -> qkv = x Wqkv^T + b -> MFMA flash attention -> a = ctx Wo^T
                      -> x1 = LN(x + dropout(a + bo))
  FFN block:        x1 -> z = x1 W1^T -> h = gelu(z + b1) -> f = h W2^T
                      -> x2 = LN(x1 + dropout(f + b2))
"""
from __future__ import annotations

import math
import os

import torch

from cloudtik_amd.ops.linear import wgrad_accumulate, wgrad_on_side_stream, wgrad_side


def _C():
    from cloudtik_amd import ops
    return ops.require_native()


# FFN dgrad through the hand-written MFMA GEMM with the dGELU + bias-gradient epilogue
# (csrc/gemm_nt.hip, B read in place as [K, N]): dz = (df @ W2) * gelu'(z + b1) and db1 in one
# kernel instead of a hipBLASLt GEMM + a bias_act_bwd pass over the [tokens, 4H] activation;
# BERT-large step 75.75 -> 74.2 ms (scripts/gpu_ab_wgrad.sh, two rounds each)
_FUSED_FFN_DGRAD = os.environ.get("CLOUDTIK_AMD_FUSED_FFN_DGRAD", "1") == "1"


# FFN1 forward through the same GEMM with the bias + GELU epilogue: h = gelu(x W1^T + b1) and the
# biased pre-activation kept for backward, instead of hipBLASLt + a bias_act_fwd pass (~20 us
# faster per layer in isolation; BERT-large step A/B 73.07 / 72.89 -> 73.01 / 72.75 ms, on by
# default; the epilogue's erf-GELU VALU work is what keeps it from gaining more)
_FUSED_FFN_FWD = os.environ.get("CLOUDTIK_AMD_FUSED_FFN_FWD", "1") == "1"


# The FFN1 forward keeps gelu'(z) (bf16) for backward instead of z itself (gemm_nt.hip EPI 6):
# the forward epilogue computes the erf / exp terms anyway and is store-bound, and the FFN
# data-gradient epilogue becomes a multiply (EPI 7) instead of ~2,150 VALU instructions per wave
# of dGELU (profiles/r3/gemm_epilogue_cost.md).  0 = keep z (EPI 1 / EPI 2).
_STORE_DGELU = os.environ.get("CLOUDTIK_AMD_FFN_STORE_DGELU", "1") == "1"


def _fused_ffn1(C, x2, W1, b1f):
    """(aux, h, kind): h = gelu(x2 W1^T + b1f); aux = gelu'(x2 W1^T + b1f) (kind "dgelu") or
    the biased pre-activation itself (kind "z").  None when unsupported."""
    T, H = x2.shape
    F = W1.shape[0]
    if T % 256 or F % 256 or H % 64 or b1f.dtype != torch.bfloat16:
        return None
    aux = torch.empty(T, F, device=x2.device, dtype=x2.dtype)
    h = torch.empty_like(aux)
    epi = 6 if _STORE_DGELU else 1
    if not C.gemm_nt(x2, W1, h, epi, False, b1f, aux, None):
        return None
    return aux, h, ("dgelu" if epi == 6 else "z")


# fp32 bias-gradient accumulators of the fused FFN dgrad, one per (device, width), kept
# zeroed between uses: the reduce that moves the sums into the bf16 gradient clears them
# (splitk_reduce_clear), so no fill kernel runs per layer.  Uses are stream-ordered on the
# main stream.
_DB_ACC = {}


# rows of the fp32 bias-gradient accumulator: the fused dgrad epilogue can spread its column-sum
# atomics over them (csrc/gemm_nt.hip), the reduce sums them.  Default 1: back to back in the
# epilogue probe 16 rows took the FFN data gradient from 363 to 334 us (the same-address atomics
# of consecutive launches queue up), but in the BERT-large step 16 rows ran 72.43 / 72.50 ms/step
# against 72.28 / 72.33 with one (the atomics drain behind the next kernels; the 16-row reduce
# adds a few us) -- profiles/r5/SUMMARY.md
_DB_ROWS = int(os.environ.get("CLOUDTIK_AMD_DBIAS_ROWS", "1"))


def _zeroed_acc(device, F, rows=1):
    key = (device, F, rows)
    t = _DB_ACC.get(key)
    if t is None:
        t = _DB_ACC[key] = torch.zeros(rows, F, device=device, dtype=torch.float32)
    return t


# FFN1's bias gradient from the FFN1 weight-gradient GEMM (all-ones MFMA on its dz operand,
# as the QKV one) instead of column-sum atomics in the FFN data-gradient epilogue.  On by
# default: BERT-large 71.39 / 71.42 / 71.51 -> 71.34 / 71.33 / 71.43 ms/step (3 interleaved
# rounds, profiles/r6/SUMMARY.md), and the bias gradient no longer depends on atomic order
_FFN_BGRAD_IN_WGRAD = os.environ.get("CLOUDTIK_AMD_FFN_BGRAD_IN_WGRAD", "1") == "1"
# LayerNorm backward from the block's OUTPUT y (xhat = (y - beta) / gamma; csrc/layernorm.hip
# FROMY) instead of a saved copy of its input sum s: y is kept anyway as the next block's
# input, so the forward writes one [tokens, hidden] tensor less (268 -> 201 MB per call on
# BERT-large).  On by default since the backward's loads became unconditional (clamped
# addresses, so the compiler's wait counts no longer drain every prefetched row): BERT-large
# (bench/ln_from_y_probe.py) forward 42 -> 35 us, backward 60 us either way, step 70.85 ->
# 70.50 ms (3 interleaved rounds, profiles/r6/SUMMARY.md).  A channel whose gamma is exactly 0
# gets xhat 0 there (its y carries no information about x), so its dgamma is 0: set
# CLOUDTIK_AMD_LN_FROM_Y=0 for models that zero-initialise LayerNorm gammas.
_LN_FROM_Y = os.environ.get("CLOUDTIK_AMD_LN_FROM_Y", "1") == "1"


def _fused_ffn_dgrad(C, df, W2, z, b1f, db1f, dgelu=False):
    """dz = (df @ W2) * gelu'(z [+ b1f]) -- or, ``dgelu``, (df @ W2) * z with z already holding
    gelu'(.) (EPI 7); db1f += column sums of dz (b1f None: z already holds the bias).  W2 [H, F]
    is read in place as the [K, N] operand (gemm_nn: no transposed copy); the fp32 column sums
    land in db1f through the split-K reduce kernel (one slab).  None when unsupported."""
    T, F = z.shape
    if T % 256 or F % 256 or df.shape[1] % 64:
        return None
    dz = torch.empty_like(z)
    if db1f is None:                                   # no bias-gradient sums in the epilogue
        return dz if C.gemm_nn(df, W2, dz, 7 if dgelu else 2, False, None if dgelu else b1f, z, None) else None
    direct = db1f.dtype == torch.bfloat16 and db1f.is_contiguous()
    rows = _DB_ROWS if direct else 1
    db = _zeroed_acc(z.device, F, rows) if direct else torch.zeros(1, F, device=z.device, dtype=torch.float32)
    if not C.gemm_nn(df, W2, dz, 7 if dgelu else 2, False, None if dgelu else b1f, z, db):
        return None
    if direct:
        C.splitk_reduce_clear(db, db1f, True)          # sums the rows and zeroes them for next time
    else:
        db1f.add_(db[0])
    return dz


# Plain forward / data-gradient GEMMs through the streamed persistent MFMA kernel
# (csrc/gemm_nt.hip gemm_nt_stream_kernel: one workgroup per CU, one continuous K-tile DMA
# stream across its tiles, epilogue stores overlapped with the next tile's loads) instead of
# hipBLASLt.  Comma list of sites (qkv, wo, ffn2, do, dx_attn, dx_ffn), "all" or "" (none);
# bench/gemm_stream_probe.py measures each shape against hipBLASLt.
_STREAM_SITES = os.environ.get("CLOUDTIK_AMD_STREAM_GEMM", "")
_STREAM_SITES = ({"qkv", "wo", "ffn2", "do", "dx_attn", "dx_ffn"} if _STREAM_SITES == "all"
                 else {t for t in _STREAM_SITES.split(",") if t})


# The same sites through the one-tile MFMA kernel (gemm_nt / gemm_nn: one 256 x 256 tile per
# workgroup); CLOUDTIK_AMD_ONETILE_GEMM takes the same site list.
_ONETILE_ENV = os.environ.get("CLOUDTIK_AMD_ONETILE_GEMM")
_ONETILE_SITES = ({"qkv", "wo", "ffn2", "do", "dx_attn", "dx_ffn"} if _ONETILE_ENV == "all"
                  else {t for t in (_ONETILE_ENV or "").split(",") if t})
# Unless CLOUDTIK_AMD_ONETILE_GEMM says otherwise, the data-gradient sites take the one-tile
# kernel while the weight gradients run in line (no side stream): BERT-large 73.40 -> 73.16
# ms/step on one box (3 interleaved rounds; profiles/r4/bert_rejected_r4.md).  Beside the side
# stream's weight-gradient GEMMs it was 1.6 ms slower, so there hipBLASLt keeps them.
_ONETILE_INLINE_SITES = {"do", "dx_attn", "dx_ffn"} if _ONETILE_ENV is None else set()


def _onetile(site, side: bool) -> bool:
    """``side``: whether this layer's weight gradients run on the side stream (the weight's
    own routing, ops.linear.wgrad_side)."""
    if site in _ONETILE_SITES:
        return True
    return site in _ONETILE_INLINE_SITES and not side


def _stream_mm(site, A, B, b_kn, bias=None, out=None, side=True):
    """A [M,K] . B^T (b_kn False: B [N,K]) or A . B (b_kn True: B [K,N]) [+ bias], or
    ``out += A . B`` when ``out`` is given, on the in-tree MFMA kernel the site is routed to
    (streamed or one-tile).  None when the site is not routed or the shape is outside the
    kernels' tiling (M, N multiples of 256, K of 64)."""
    stream = site in _STREAM_SITES
    if not stream and not _onetile(site, side):
        return None
    M, K = A.shape
    N = B.shape[1] if b_kn else B.shape[0]
    if M % 256 or N % 256 or K % 64 or not A.is_contiguous() or not B.is_contiguous():
        return None
    if bias is not None and (bias.dtype != torch.bfloat16 or not bias.is_contiguous()):
        return None
    acc = out is not None
    D = out if acc else torch.empty(M, N, device=A.device, dtype=A.dtype)
    C = _C()
    if stream:
        ok = C.gemm_nt_stream(A, B, D, bias, b_kn, 0, acc)
    elif b_kn:
        ok = bias is None and C.gemm_nn(A, B, D, 0, acc, None, None, None)
    else:
        ok = C.gemm_nt(A, B, D, 5 if bias is not None else 0, acc, bias, None, None)
    return D if ok else None


def _flat(p) -> bool:
    return p.grad is not None and getattr(p, "_ct_flat_grad", False)


def _ready(*params):
    for p in params:
        cb = getattr(p, "_ct_grad_ready", None)
        if cb is not None:
            cb(p)


def _wgrad(p, dy2, x2, bias=None):
    """dW = dy2^T x2, accumulated into the flat buffer when possible.  With ``bias`` (a flat
    parameter), its gradient -- the column sums of dy2 -- comes out of the same GEMM."""
    if _flat(p):
        db = bias.grad if bias is not None else None
        if not wgrad_on_side_stream(p.grad, dy2, x2, db, enabled=wgrad_side(p)):
            wgrad_accumulate(p.grad, dy2, x2, db)
        _ready(p)
        if bias is not None:
            _ready(bias)
        return None
    return dy2.t() @ x2


def _vec_grad_out(p):
    """(target tensor for an accumulating kernel, whether it is the flat grad)."""
    if _flat(p):
        return p.grad, True
    return torch.zeros_like(p), False


class _AttnBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, Wqkv, bqkv, Wo, bo, g1, b1, key_bias, nh, p_attn, p_hid, eps,
                seed_a, off_a, seed_h, off_h):
        C = _C()
        B, S, H = x.shape
        D = H // nh
        x2 = x.reshape(B * S, H)
        qkv = _stream_mm("qkv", x2, Wqkv, False, bias=bqkv)
        if qkv is None:
            qkv = torch.addmm(bqkv, x2, Wqkv.t())
        v5 = qkv.view(B, S, 3, nh, D)
        o = torch.empty(B, S, nh, D, dtype=x.dtype, device=x.device)
        scale = 1.0 / math.sqrt(D)
        lse = C.attn_fwd(v5[:, :, 0], v5[:, :, 1], v5[:, :, 2], o, key_bias, scale, p_attn,
                         seed_a, off_a, False)
        a = _stream_mm("wo", o.view(B * S, H), Wo, False)
        if a is None:
            a = torch.mm(o.view(B * S, H), Wo.t())
        from_y = _LN_FROM_Y and b1 is not None
        y, s, mean, rstd = C.layernorm_fwd(a, bo, x2, g1, b1, eps, False, p_hid, seed_h, off_h,
                                           keep_sum=not from_y)
        yv = y.view(B, S, H)
        ctx.save_for_backward(x2, qkv, o, lse, yv if from_y else s, mean, rstd,
                              key_bias if key_bias is not None else torch.empty(0))
        ctx.params = (Wqkv, bqkv, Wo, bo, g1, b1)
        ctx.cfg = (B, S, H, nh, D, scale, p_attn, p_hid, seed_a, off_a, seed_h, off_h,
                   key_bias is not None, from_y)
        return yv

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        x2, qkv, o, lse, s, mean, rstd, kb = ctx.saved_tensors
        Wqkv, bqkv, Wo, bo, g1, b1 = ctx.params
        B, S, H, nh, D, scale, p_attn, p_hid, seed_a, off_a, seed_h, off_h, has_kb, from_y = ctx.cfg
        dy2 = dy.reshape(B * S, H).contiguous()
        s = s.view(B * S, H)
        dg1, fg1 = _vec_grad_out(g1)
        db1, fb1 = _vec_grad_out(b1)
        dbo, fbo = _vec_grad_out(bo)
        need_dx = p_hid > 0.0
        # the output-projection bias gradient (column sums of da) is accumulated by the LayerNorm
        # backward: moving it into the projection's weight-gradient GEMM (all-ones MFMA) made the
        # LayerNorm pass 11 % faster but the GEMMs 1.5 ms per step slower
        ds, da = C.layernorm_bwd_into(dy2, s, g1, mean, rstd, False, dg1, db1, dbo, need_dx,
                                      p_hid, seed_h, off_h, beta_y=b1 if from_y else None)
        if not need_dx:
            da = ds
        _ready(*[p for p, f in ((g1, fg1), (b1, fb1), (bo, fbo)) if f])
        o2 = o.view(B * S, H)
        dWo = _wgrad(Wo, da, o2)
        do = _stream_mm("do", da, Wo, True, side=wgrad_side(Wo))
        if do is None:
            do = torch.mm(da, Wo)
        do = do.view(B, S, nh, D)
        dqkv = torch.empty_like(qkv)
        v5 = qkv.view(B, S, 3, nh, D)
        d5 = dqkv.view(B, S, 3, nh, D)
        C.attn_bwd(v5[:, :, 0], v5[:, :, 1], v5[:, :, 2], o, do, d5[:, :, 0], d5[:, :, 1], d5[:, :, 2],
                   kb if has_kb else None, lse, scale, p_attn, seed_a, off_a, False)
        dbq, fbq = _vec_grad_out(bqkv)
        if fbq and _flat(Wqkv):
            dWqkv = _wgrad(Wqkv, dqkv, x2, bias=bqkv)          # bias grad fused into the wgrad GEMM
        else:
            C.bias_act_bwd_into(dqkv, dqkv, None, 0, dbq, False)   # column sum of dqkv
            if fbq:
                _ready(bqkv)
            dWqkv = _wgrad(Wqkv, dqkv, x2)
        dx = _stream_mm("dx_attn", dqkv, Wqkv, True, out=ds, side=wgrad_side(Wqkv))
        if dx is None:
            dx = ds.addmm_(dqkv, Wqkv)    # residual grad fused: in-place beta=1 epilogue, no C copy
        return (dx.view(B, S, H), dWqkv, None if fbq else dbq, dWo, None if fbo else dbo,
                None if fg1 else dg1, None if fb1 else db1, None, None, None, None, None,
                None, None, None, None)


class _FFNBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x1, W1, b1f, W2, b2f, g2, b2, p_hid, eps, seed_h, off_h):
        C = _C()
        B, S, H = x1.shape
        x2 = x1.reshape(B * S, H)
        fused = _fused_ffn1(C, x2, W1, b1f) if _FUSED_FFN_FWD else None
        kind = None
        if fused is not None:
            z, h, kind = fused                  # z includes the bias, or is gelu'(z + b1)
        else:
            z = torch.mm(x2, W1.t())
            h = C.bias_act_fwd(z, b1f, 1)
        f = _stream_mm("ffn2", h, W2, False)
        if f is None:
            f = torch.mm(h, W2.t())
        from_y = _LN_FROM_Y and b2 is not None
        y, s, mean, rstd = C.layernorm_fwd(f, b2f, x2, g2, b2, eps, False, p_hid, seed_h, off_h,
                                           keep_sum=not from_y)
        yv = y.view(B, S, H)
        ctx.save_for_backward(x2, z, h, yv if from_y else s, mean, rstd)
        ctx.params = (W1, b1f, W2, b2f, g2, b2)
        ctx.cfg = (B, S, H, p_hid, seed_h, off_h, kind, from_y)
        return yv

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        x2, z, h, s, mean, rstd = ctx.saved_tensors
        W1, b1f, W2, b2f, g2, b2 = ctx.params
        B, S, H, p_hid, seed_h, off_h, kind, from_y = ctx.cfg
        s = s.view(B * S, H)
        dgelu = kind == "dgelu"                 # z holds gelu'(pre-activation) itself
        zbias = None if kind is not None else b1f   # the bias gelu' still has to add to z
        dy2 = dy.reshape(B * S, H).contiguous()
        dg2, fg2 = _vec_grad_out(g2)
        db2, fb2 = _vec_grad_out(b2)
        db2f, fb2f = _vec_grad_out(b2f)
        need_dx = p_hid > 0.0
        ds, df = C.layernorm_bwd_into(dy2, s, g2, mean, rstd, False, dg2, db2, db2f, need_dx,
                                      p_hid, seed_h, off_h, beta_y=b2 if from_y else None)
        if not need_dx:
            df = ds
        _ready(*[p for p, f in ((g2, fg2), (b2, fb2), (b2f, fb2f)) if f])
        dW2 = _wgrad(W2, df, h)
        db1f, fb1f = _vec_grad_out(b1f)
        bias_in_wgrad = _FFN_BGRAD_IN_WGRAD and dgelu and fb1f and _flat(W1)
        dz = (_fused_ffn_dgrad(C, df.contiguous(), W2, z, zbias, None if bias_in_wgrad else db1f, dgelu)
              if _FUSED_FFN_DGRAD else None)
        if dz is not None and bias_in_wgrad:
            dW1 = _wgrad(W1, dz, x2, bias=b1f)         # bias gradient fused into the wgrad GEMM
            dx = _stream_mm("dx_ffn", dz, W1, True, out=ds, side=wgrad_side(W1))
            if dx is None:
                dx = ds.addmm_(dz, W1)
            return (dx.view(B, S, H), dW1, None, dW2, None if fb2f else db2f,
                    None if fg2 else dg2, None if fb2 else db2, None, None, None, None)
        bias_in_wgrad = False
        if dz is None and dgelu:
            dz = torch.mm(df, W2).mul_(z)
            db1f.add_(dz.float().sum(0).to(db1f.dtype))
        elif dz is None:
            dh = torch.mm(df, W2)
            dz = C.bias_act_bwd_into(dh, z, zbias, 1, db1f, True)
        if fb1f:
            _ready(b1f)
        dW1 = _wgrad(W1, dz, x2)
        dx = _stream_mm("dx_ffn", dz, W1, True, out=ds, side=wgrad_side(W1))
        if dx is None:
            dx = ds.addmm_(dz, W1)
        return (dx.view(B, S, H), dW1, None if fb1f else db1f, dW2, None if fb2f else db2f,
                None if fg2 else dg2, None if fb2 else db2, None, None, None, None)


def attention_block(x, Wqkv, bqkv, Wo, bo, g1, b1, key_bias, num_heads, p_attn, p_hidden, eps,
                    training=True):
    from cloudtik_amd import ops
    B, S, H = x.shape
    p_attn = float(p_attn) if training else 0.0
    p_hidden = float(p_hidden) if training else 0.0
    sa, oa = ops._rng.next(B * num_heads * S * S) if p_attn > 0 else (0, 0)
    sh, oh = ops._rng.next(x.numel()) if p_hidden > 0 else (0, 0)
    if key_bias is not None:
        key_bias = key_bias.float().contiguous()
    return _AttnBlockFn.apply(x.contiguous(), Wqkv, bqkv, Wo, bo, g1, b1, key_bias, num_heads,
                              p_attn, p_hidden, float(eps), sa, oa, sh, oh)


def ffn_block(x1, W1, b1f, W2, b2f, g2, b2, p_hidden, eps, training=True):
    from cloudtik_amd import ops
    p_hidden = float(p_hidden) if training else 0.0
    sh, oh = ops._rng.next(x1.numel()) if p_hidden > 0 else (0, 0)
    return _FFNBlockFn.apply(x1.contiguous(), W1, b1f, W2, b2f, g2, b2, p_hidden, float(eps), sh, oh)


def blocks_supported(x, H, nh) -> bool:
    from cloudtik_amd import ops
    return (x.is_cuda and ops.native_available() and x.dtype == torch.bfloat16 and H // nh == 64
            and H % 8 == 0 and H <= 2048 and torch.is_grad_enabled() is not None)
