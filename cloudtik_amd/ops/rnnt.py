"""RNN-Transducer loss (HIP kernels in csrc/rnnt.hip; SURVEY.md §2.12 RNN-T workload).

``rnnt_loss(logits, labels, logit_lengths, label_lengths, blank=0, reduction="mean")``

* ``logits``  [B, T, U+1, V] joint-network outputs (bf16 or fp32, unnormalised)
* ``labels``  [B, U] int targets (padded), ``label_lengths`` [B], ``logit_lengths`` [B]

Returns the negative log-likelihood per utterance (``reduction="none"``), its sum or its
mean.  The GPU path computes log-softmax statistics, the alpha / beta lattices and the
logits gradient in three kernels; ``rnnt_loss_reference`` is the fp32 PyTorch definition
used on CPU and as the numerics reference.
"""
from __future__ import annotations

import torch


def _C():
    from cloudtik_amd import ops
    return ops.require_native()


def rnnt_loss_reference(logits, labels, logit_lengths, label_lengths, blank: int = 0):
    """Per-utterance NLL, differentiable (autograd through log_softmax and the DP)."""
    lp = torch.log_softmax(logits.float(), -1)
    B, T, U1, V = lp.shape
    out = []
    for b in range(B):
        Tb, Ub = int(logit_lengths[b]), int(label_lengths[b])
        lpb = lp[b, :Tb, :Ub + 1]
        blank_lp = lpb[..., blank]                                  # [Tb, Ub+1]
        if Ub:
            y = labels[b, :Ub].long().to(lp.device)
            label_lp = lpb[:, :Ub].gather(-1, y.view(1, Ub, 1).expand(Tb, Ub, 1)).squeeze(-1)   # [Tb, Ub]
        alpha = [[None] * (Ub + 1) for _ in range(Tb)]
        for t in range(Tb):
            for u in range(Ub + 1):
                if t == 0 and u == 0:
                    alpha[t][u] = lp.new_zeros(())
                    continue
                terms = []
                if t > 0:
                    terms.append(alpha[t - 1][u] + blank_lp[t - 1, u])
                if u > 0:
                    terms.append(alpha[t][u - 1] + label_lp[t, u - 1])
                alpha[t][u] = torch.logsumexp(torch.stack(terms), 0)
        out.append(-(alpha[Tb - 1][Ub] + blank_lp[Tb - 1, Ub]))
    return torch.stack(out)


class _RNNTLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, tlen, ulen, blank):
        logits = logits.contiguous()
        loglik, lse, lp, alpha, beta = _C().rnnt_fwd(logits, labels, tlen, ulen, blank)
        ctx.save_for_backward(logits, labels, tlen, ulen, lse, lp, alpha, beta, loglik)
        ctx.blank = blank
        return -loglik

    @staticmethod
    def backward(ctx, g):
        logits, labels, tlen, ulen, lse, lp, alpha, beta, loglik = ctx.saved_tensors
        grad = _C().rnnt_bwd(logits, labels, tlen, ulen, lse, lp, alpha, beta, loglik, g.float().contiguous(),
                             ctx.blank)
        return grad, None, None, None, None


def rnnt_loss(logits, labels, logit_lengths, label_lengths, blank: int = 0, reduction: str = "mean"):
    from cloudtik_amd import ops
    if logits.is_cuda and ops._use_native(logits):
        dev = logits.device
        U = logits.shape[2] - 1
        lab = labels.to(dev, torch.int32)
        if lab.shape[1] != U:                         # pad / trim to the lattice width
            lab = torch.nn.functional.pad(lab, (0, max(0, U - lab.shape[1])))[:, :U]
        nll = _RNNTLossFn.apply(logits, lab.contiguous(), logit_lengths.to(dev, torch.int32).contiguous(),
                                label_lengths.to(dev, torch.int32).contiguous(), int(blank))
    else:
        nll = rnnt_loss_reference(logits, labels, logit_lengths, label_lengths, blank)
    if reduction == "none":
        return nll
    if reduction == "sum":
        return nll.sum()
    return nll.mean()
