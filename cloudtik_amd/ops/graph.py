"""Graph-ML and boosted-tree ops (csrc/graph_ml.hip) with torch references.

* ``gbdt_histogram``  -- per-node (grad, hess) histograms over binned features, the inner
  loop of histogram gradient boosting (XGBoost ``tree_method=hist``; reference
  modeling/classical_ml/classification_and_regression/xgboost/modeling/model/trainer.py).
* ``gbdt_predict``    -- ensemble inference over complete binary trees on binned features.
* ``spmm`` / ``SpMM`` -- CSR sparse x dense aggregation with autograd (GraphSAGE mean /
  sum neighbour aggregation; reference graph_sage/model/homogeneous/*.py uses DGL's
  SAGEConv 'mean').  The backward is the same kernel on the transposed CSR.

GPU tensors always take the HIP kernels (the extension is required there); CPU tensors use
the torch references, which the GPU tests compare against.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch


def _native():
    from cloudtik_amd import ops
    return ops.require_native()


def _use_native(*ts) -> bool:
    from cloudtik_amd import ops
    return ops._use_native(*ts)


# ---------------------------------------------------------------------- GBDT histograms
MAX_SLOTS_PER_PASS = 32          # 32 slots x 256 bins x 8 B = 64 KB of LDS per feature


def gbdt_histogram_reference(bins: torch.Tensor, n_rows: int, node: torch.Tensor, gh: torch.Tensor,
                             n_slots: int, n_bins: int) -> torch.Tensor:
    F = bins.shape[0]
    node = node[:n_rows].long()
    rows = torch.nonzero((node >= 0) & (node < n_slots)).squeeze(1)
    nd = node[rows]
    g = gh[:n_rows][rows].float()
    b = bins[:, :n_rows][:, rows].long()                                    # [F, R]
    idx = ((nd[None, :] * F + torch.arange(F, device=bins.device)[:, None]) * n_bins + b).reshape(-1)
    hist = torch.zeros(n_slots * F * n_bins, 2, dtype=torch.float32, device=bins.device)
    hist.index_add_(0, idx, g.repeat(F, 1))
    return hist.view(n_slots, F, n_bins, 2)


def gbdt_histogram(bins: torch.Tensor, n_rows: int, node: torch.Tensor, gh: torch.Tensor, n_slots: int,
                   n_bins: int, out: Optional[torch.Tensor] = None,
                   slot_map: Optional[torch.Tensor] = None) -> torch.Tensor:
    """hist[s, f, b] = sum over rows r with node[r] == s and bins[f, r] == b of gh[r].

    bins: uint8 [F, ldb] feature-major (ldb % 4 == 0); node: int32 [N] (-1 = inactive);
    gh: fp32 [N, 2].  Returns fp32 [n_slots, F, n_bins, 2]."""
    if not _use_native(bins):
        if slot_map is not None:
            node = torch.where((node >= 0) & (node < slot_map.numel()), slot_map[node.clamp(0, slot_map.numel() - 1).long()],
                               torch.full_like(node, -1))
        return gbdt_histogram_reference(bins, n_rows, node, gh, n_slots, n_bins)
    F = bins.shape[0]
    hist = out if out is not None else torch.empty(n_slots, F, n_bins, 2, dtype=torch.float32, device=bins.device)
    hist.zero_()
    per_pass = max(1, min(MAX_SLOTS_PER_PASS, (64 * 1024) // (n_bins * 8)))
    C = _native()
    for lo in range(0, n_slots, per_pass):
        C.gbdt_hist(bins, int(n_rows), node, gh, hist, lo, min(per_pass, n_slots - lo), slot_map)
    return hist


# ---------------------------------------------------------------------- ensemble predict
def gbdt_predict_reference(bins, n_rows, feat, thr, dleft, leaf, n_outputs) -> torch.Tensor:
    T, M = feat.shape
    out = torch.zeros(n_rows, n_outputs, dtype=torch.float32, device=bins.device)
    rows = torch.arange(n_rows, device=bins.device)
    for t in range(T):
        n = torch.zeros(n_rows, dtype=torch.long, device=bins.device)
        while True:
            f = feat[t][n].long()
            active = f >= 0
            if not bool(active.any()):
                break
            b = bins[f.clamp(min=0), rows].long()
            left = torch.where(b == 0, dleft[t][n].bool(), b <= thr[t][n].long())
            n = torch.where(active, 2 * n + torch.where(left, 1, 2), n)
        out[:, t % n_outputs] += leaf[t][n]
    return out


def gbdt_predict(bins, n_rows: int, feat, thr, dleft, leaf, n_outputs: int = 1) -> torch.Tensor:
    """Sum of leaf values of every tree (tree t adds to output column t % n_outputs)."""
    if not _use_native(bins):
        return gbdt_predict_reference(bins, n_rows, feat, thr, dleft, leaf, n_outputs)
    out = torch.zeros(n_rows, n_outputs, dtype=torch.float32, device=bins.device)
    _native().gbdt_predict(bins, int(n_rows), feat.int().contiguous(), thr.int().contiguous(),
                           dleft.to(torch.uint8).contiguous(), leaf.float().contiguous(), out)
    return out


# ---------------------------------------------------------------------- CSR SpMM
@dataclass
class CSR:
    """rows x cols sparse matrix in CSR form (int64 indices, optional fp32 edge weights)."""
    rowptr: torch.Tensor
    col: torch.Tensor
    n_cols: int
    weight: Optional[torch.Tensor] = None

    @property
    def n_rows(self) -> int:
        return self.rowptr.numel() - 1

    def degrees(self) -> torch.Tensor:
        return self.rowptr[1:] - self.rowptr[:-1]

    def to(self, device) -> "CSR":
        return CSR(self.rowptr.to(device), self.col.to(device), self.n_cols,
                   None if self.weight is None else self.weight.to(device))

    @staticmethod
    def from_edges(dst: torch.Tensor, src: torch.Tensor, n_dst: int, n_src: int,
                   weight: Optional[torch.Tensor] = None) -> "CSR":
        """Rows are destinations (who aggregates), columns sources (whose features)."""
        order = torch.argsort(dst * n_src + src)
        d = dst[order]
        counts = torch.bincount(d, minlength=n_dst)
        rowptr = torch.zeros(n_dst + 1, dtype=torch.long, device=dst.device)
        rowptr[1:] = torch.cumsum(counts, 0)
        w = None if weight is None else weight[order].float().contiguous()
        return CSR(rowptr, src[order].long().contiguous(), n_src, w)

    def transpose(self, row_scale: Optional[torch.Tensor] = None) -> "CSR":
        """A^T, with edge weights w_e * row_scale[dst_e] folded in (for mean backward)."""
        dst = torch.repeat_interleave(torch.arange(self.n_rows, device=self.col.device), self.degrees())
        w = self.weight
        if row_scale is not None:
            rs = row_scale[dst].float()
            w = rs if w is None else w * rs
        return CSR.from_edges(self.col, dst, self.n_cols, self.n_rows, w)


def spmm_reference(csr: CSR, x: torch.Tensor, mean: bool = False) -> torch.Tensor:
    dst = torch.repeat_interleave(torch.arange(csr.n_rows, device=x.device), csr.degrees())
    msg = x[csr.col].float()
    if csr.weight is not None:
        msg = msg * csr.weight[:, None]
    out = torch.zeros(csr.n_rows, x.shape[1], dtype=torch.float32, device=x.device)
    out.index_add_(0, dst, msg)
    if mean:
        out = out / csr.degrees().clamp(min=1)[:, None].float()
    return out.to(x.dtype)


def _spmm_raw(csr: CSR, x: torch.Tensor, mean: bool) -> torch.Tensor:
    if not _use_native(x):
        return spmm_reference(csr, x, mean)
    D = x.shape[1]
    vec = 4 if x.dtype == torch.float32 else 8            # 16-byte rows for the kernel
    if D % vec:
        x = torch.nn.functional.pad(x, (0, vec - D % vec))
    x = x.contiguous()
    out = torch.empty(csr.n_rows, x.shape[1], dtype=x.dtype, device=x.device)
    _native().csr_spmm(csr.rowptr, csr.col, csr.weight, None, bool(mean), x, out, False)
    return out[:, :D] if out.shape[1] != D else out


def _mean_scale(csr: CSR) -> torch.Tensor:
    return 1.0 / csr.degrees().clamp(min=1).float()


class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, csr, csr_t, mean):
        ctx.csr_t = csr_t
        return _spmm_raw(csr, x, mean)

    @staticmethod
    def backward(ctx, gy):
        # d/dx of (D^-1) A x is A^T D^-1 gy; csr_t already carries the D^-1 weights
        return _spmm_raw(ctx.csr_t, gy.contiguous(), False), None, None, None


class SpMM:
    """Reusable aggregation operator for one graph block: forward A x (optionally row
    normalised) and the cached transpose for the backward."""

    def __init__(self, csr: CSR, mean: bool = True):
        self.csr = csr
        self.mean = mean
        self.csr_t = csr.transpose(_mean_scale(csr) if mean else None)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return _SpMM.apply(x, self.csr, self.csr_t, self.mean)


def spmm(csr: CSR, x: torch.Tensor, mean: bool = False) -> torch.Tensor:
    return SpMM(csr, mean)(x)
