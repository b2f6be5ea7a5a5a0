"""Histogram gradient-boosted decision trees on MI355X (the library behind
``ai.modeling.xgboost``; reference runtime/ai/modeling/classical_ml/classification_and_regression/
xgboost/modeling/model/trainer.py:1-201, which drives xgboost / xgboost-ray / xgboost-spark).

XGBoost itself is not part of this stack, so the algorithm of its ``tree_method=hist`` is
implemented directly, GPU-resident end to end:

* features are quantised once into <=255 quantile bins per feature (bin 0 = missing) and
  kept on the GPU as a feature-major uint8 matrix;
* trees grow level by level to ``max_depth``.  For every level the (grad, hess) histograms
  of the nodes being split come from one HIP kernel (``ops.gbdt_histogram``, LDS
  histograms + global atomics); only the smaller child of each split is built, its sibling
  is parent - child (the subtraction trick halves histogram work);
* split search over every (node, feature, bin, missing-direction) is a handful of batched
  tensor ops on the histogram; regularisation follows XGBoost (lambda, alpha,
  min_child_weight, gamma, max_delta_step, eta, subsample, colsample_bytree);
* data-parallel training: each rank holds a row shard, histograms and node statistics are
  summed with one all-reduce per level (RCCL on GPUs, gloo on CPUs) -- the role Rabit plays
  for XGBoost -- so every rank grows the identical tree;
* trees are stored as complete binary arrays and the whole ensemble is evaluated by one
  HIP kernel (``ops.gbdt_predict``).
"""
from __future__ import annotations

import json
import math
from dataclasses import asdict, dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.distributed as dist

from cloudtik_amd import ops

MISSING_BIN = 0


# ---------------------------------------------------------------------- distributed helpers
def _dist_on() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _allreduce_(t: torch.Tensor) -> torch.Tensor:
    if _dist_on():
        dist.all_reduce(t)
    return t


# ---------------------------------------------------------------------- quantisation
class BinMapper:
    """Quantile cuts per feature: value v of feature f goes to bin 1 + #(cuts[f] < v);
    NaN goes to bin 0.  ``cuts`` is [F, max_bin - 2] padded with +inf."""

    def __init__(self, max_bin: int = 256):
        if not 3 <= max_bin <= 256:
            raise ValueError("max_bin must be in [3, 256]")
        self.max_bin = max_bin
        self.cuts: Optional[torch.Tensor] = None

    def fit(self, X: torch.Tensor, sample_rows: int = 200_000, seed: int = 0) -> "BinMapper":
        Xs = X
        if X.shape[0] > sample_rows:
            g = torch.Generator(device="cpu").manual_seed(seed)
            idx = torch.randperm(X.shape[0], generator=g)[:sample_rows].to(X.device)
            Xs = X[idx]
        if _dist_on():
            # every rank contributes a sample; all ranks derive identical cuts
            n = torch.tensor([Xs.shape[0]], device=Xs.device)
            sizes = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
            dist.all_gather(sizes, n)
            m = int(max(s.item() for s in sizes))
            pad = torch.full((m, Xs.shape[1]), float("nan"), device=Xs.device, dtype=torch.float32)
            pad[:Xs.shape[0]] = Xs.float()
            parts = [torch.empty_like(pad) for _ in sizes]
            dist.all_gather(parts, pad)
            Xs = torch.cat(parts)
        # quantiles on the sample's device (the GPU when training there): one sort of the
        # [S, F] sample, then per feature either its distinct values (few of them) or the
        # values at the quantile ranks
        Xs = Xs.float()
        nb = self.max_bin - 2          # cuts; gives up to max_bin - 1 value bins
        srt, _ = torch.sort(Xs, dim=0)                      # NaN sorts last
        valid = (~torch.isnan(srt)).sum(0).cpu()
        cuts = torch.full((Xs.shape[1], nb), float("inf"), device=Xs.device)
        qs = torch.linspace(0, 1, nb + 2, device=Xs.device)[1:-1]
        for f in range(Xs.shape[1]):
            n = int(valid[f])
            if n == 0:
                continue
            col = srt[:n, f]
            u = torch.unique_consecutive(col)
            if u.numel() <= nb + 1:
                c = u[:-1]
            else:
                c = torch.unique_consecutive(col[(qs * (n - 1)).round().long()])
                c = c[c < u[-1]]
            cuts[f, :c.numel()] = c[:nb]
        cuts = cuts.cpu()
        self.cuts = cuts
        return self

    @property
    def n_features(self) -> int:
        return int(self.cuts.shape[0])

    def transform(self, X: torch.Tensor, device=None) -> Tuple[torch.Tensor, int]:
        """-> (uint8 [F, ldb] feature-major bins, n_rows); ldb is rounded up to 4."""
        device = device or X.device
        Xf = X.to(device=device, dtype=torch.float32)
        N, F = Xf.shape
        if F != self.n_features:
            raise ValueError(f"expected {self.n_features} features, got {F}")
        ldb = (N + 3) // 4 * 4
        out = torch.zeros(F, ldb, dtype=torch.uint8, device=device)
        cuts = self.cuts.to(device)
        for f in range(F):
            col = Xf[:, f].contiguous()
            b = torch.searchsorted(cuts[f].contiguous(), col, right=False) + 1
            b = torch.where(torch.isnan(col), torch.zeros_like(b), b)
            out[f, :N] = b.to(torch.uint8)
        return out, N

    def threshold_value(self, f: int, bin_thr: int) -> float:
        """Raw split value of 'bin <= bin_thr' (x <= value)."""
        return float(self.cuts[f, bin_thr - 1])

    def state_dict(self):
        return {"max_bin": self.max_bin, "cuts": self.cuts.tolist()}

    @classmethod
    def from_state(cls, s):
        m = cls(s["max_bin"])
        m.cuts = torch.tensor(s["cuts"], dtype=torch.float32)
        return m


# ---------------------------------------------------------------------- objectives / metrics
def _sigmoid(x):
    return torch.sigmoid(x)


class Objective:
    name = ""
    n_outputs = 1

    def grad_hess(self, margin, y, w):
        raise NotImplementedError

    def transform(self, margin):
        return margin

    def base_margin(self, y, w) -> List[float]:
        return [0.0] * self.n_outputs


class SquaredError(Objective):
    name = "reg:squarederror"

    def grad_hess(self, margin, y, w):
        g = margin[:, 0] - y
        h = torch.ones_like(g)
        return [(g * w, h * w)]

    def base_margin(self, y, w):
        s = _allreduce_(torch.stack([(y * w).sum(), w.sum()]).double())
        return [float(s[0] / s[1].clamp(min=1e-12))]


class Logistic(Objective):
    name = "binary:logistic"

    def grad_hess(self, margin, y, w):
        p = _sigmoid(margin[:, 0])
        return [((p - y) * w, (p * (1 - p)).clamp(min=1e-16) * w)]

    def transform(self, margin):
        return _sigmoid(margin)

    def base_margin(self, y, w):
        s = _allreduce_(torch.stack([(y * w).sum(), w.sum()]).double())
        p = float(s[0] / s[1].clamp(min=1e-12))
        p = min(max(p, 1e-6), 1 - 1e-6)
        return [math.log(p / (1 - p))]


class LogitRaw(Logistic):
    name = "binary:logitraw"

    def transform(self, margin):
        return margin


class Softmax(Objective):
    name = "multi:softprob"

    def __init__(self, num_class: int):
        if num_class < 2:
            raise ValueError("multi-class objectives need num_class >= 2")
        self.n_outputs = num_class

    def grad_hess(self, margin, y, w):
        p = torch.softmax(margin, dim=1)
        out = []
        yl = y.long()
        for k in range(self.n_outputs):
            pk = p[:, k]
            g = pk - (yl == k).float()
            h = (2 * pk * (1 - pk)).clamp(min=1e-16)
            out.append((g * w, h * w))
        return out

    def transform(self, margin):
        return torch.softmax(margin, dim=1)


class SoftmaxClass(Softmax):
    name = "multi:softmax"


def make_objective(name: str, num_class: int = 0) -> Objective:
    if name in ("reg:squarederror", "reg:linear"):
        return SquaredError()
    if name in ("binary:logistic", "reg:logistic"):
        return Logistic()
    if name == "binary:logitraw":
        return LogitRaw()
    if name == "multi:softprob":
        return Softmax(num_class)
    if name == "multi:softmax":
        return SoftmaxClass(num_class)
    raise ValueError(f"unsupported objective {name!r}")


def _rank_auc(score, y, w):
    order = torch.argsort(score)
    s, yy, ww = score[order], y[order], w[order]
    # average ranks over ties, weighted
    uniq, inv = torch.unique_consecutive(s, return_inverse=True)
    grp_end = torch.zeros(uniq.numel(), dtype=ww.dtype, device=ww.device)
    pos_w = (ww * yy).sum()
    neg_w = (ww * (1 - yy)).sum()
    if pos_w <= 0 or neg_w <= 0:
        return float("nan")
    # weighted Mann-Whitney U: sum over positives of the negative weight ranked below
    neg_cum = torch.cumsum(ww * (1 - yy), 0)
    grp_neg_end = torch.zeros_like(grp_end).scatter_reduce(0, inv, neg_cum, "amax")
    grp_neg = torch.zeros_like(grp_end).index_add_(0, inv, ww * (1 - yy))
    below = (grp_neg_end - grp_neg)[inv] + 0.5 * grp_neg[inv]
    return float(((ww * yy) * below).sum() / (pos_w * neg_w))


def _average_precision(score, y, w):
    order = torch.argsort(score, descending=True)
    s, yy, ww = score[order], y[order], w[order]
    tp = torch.cumsum(ww * yy, 0)
    fp = torch.cumsum(ww * (1 - yy), 0)
    # evaluate only at the last element of each tie group
    last = torch.ones_like(s, dtype=torch.bool)
    last[:-1] = s[1:] != s[:-1]
    tp, fp = tp[last], fp[last]
    total_pos = tp[-1]
    if total_pos <= 0:
        return float("nan")
    precision = tp / (tp + fp).clamp(min=1e-12)
    recall = tp / total_pos
    dr = torch.diff(recall, prepend=torch.zeros(1, dtype=recall.dtype, device=recall.device))
    return float((dr * precision).sum())


def evaluate_metric(name: str, pred: torch.Tensor, y: torch.Tensor, w: torch.Tensor) -> float:
    """pred: transformed predictions [N, K] (probabilities for classification)."""
    p = pred[:, 0] if pred.shape[1] == 1 else pred
    W = w.sum().clamp(min=1e-12)
    if name == "rmse":
        return float(torch.sqrt(((p - y) ** 2 * w).sum() / W))
    if name == "mae":
        return float(((p - y).abs() * w).sum() / W)
    if name == "logloss":
        q = p.clamp(1e-15, 1 - 1e-15)
        return float((-(y * q.log() + (1 - y) * (1 - q).log()) * w).sum() / W)
    if name == "error":
        return float((((p > 0.5).float() != y).float() * w).sum() / W)
    if name == "auc":
        return _rank_auc(p.double(), y.double(), w.double())
    if name == "aucpr":
        return _average_precision(p.double(), y.double(), w.double())
    if name == "mlogloss":
        q = p.gather(1, y.long()[:, None]).squeeze(1).clamp(min=1e-15)
        return float((-q.log() * w).sum() / W)
    if name == "merror":
        return float(((p.argmax(1) != y.long()).float() * w).sum() / W)
    raise ValueError(f"unsupported eval_metric {name!r}")


MAXIMIZE = {"auc", "aucpr"}


# ---------------------------------------------------------------------- parameters / trees
@dataclass
class BoostParams:
    objective: str = "reg:squarederror"
    num_class: int = 0
    eta: float = 0.3
    max_depth: int = 6
    min_child_weight: float = 1.0
    reg_lambda: float = 1.0
    reg_alpha: float = 0.0
    gamma: float = 0.0
    max_delta_step: float = 0.0
    subsample: float = 1.0
    colsample_bytree: float = 1.0
    max_bin: int = 256
    base_score: Optional[float] = None
    seed: int = 0
    eval_metric: List[str] = field(default_factory=list)

    ALIASES = {"learning_rate": "eta", "lambda": "reg_lambda", "alpha": "reg_alpha",
               "min_split_loss": "gamma", "random_state": "seed"}
    IGNORED = {"tree_method", "nthread", "n_jobs", "verbosity", "device", "gpu_id", "predictor"}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "BoostParams":
        p = cls()
        for k, v in (d or {}).items():
            k = cls.ALIASES.get(k, k)
            if k in cls.IGNORED:
                continue
            if k == "eval_metric":
                v = [v] if isinstance(v, str) else list(v)
            if not hasattr(p, k):
                raise ValueError(f"unknown booster parameter {k!r}")
            setattr(p, k, v)
        return p


@dataclass
class TreeArrays:
    """All trees of the ensemble as complete binary trees of M = 2^(max_depth+1)-1 nodes."""
    feat: torch.Tensor      # int32 [T, M], -1 = leaf
    thr: torch.Tensor       # int32 [T, M], go left if bin <= thr
    dleft: torch.Tensor     # uint8 [T, M], missing goes left
    leaf: torch.Tensor      # fp32  [T, M]
    gain: torch.Tensor      # fp32  [T, M] split gain (feature importance)
    cover: torch.Tensor     # fp32  [T, M] hessian sum


# ---------------------------------------------------------------------- DMatrix
class DMatrix:
    """Features (float, NaN = missing), label, weight; binned lazily against a BinMapper."""

    def __init__(self, data, label=None, weight=None, feature_names: Optional[List[str]] = None):
        if hasattr(data, "to_numpy") and hasattr(data, "columns"):      # pandas DataFrame
            feature_names = feature_names or [str(c) for c in data.columns]
            data = data.to_numpy(dtype=np.float32, na_value=np.nan)
        if hasattr(label, "to_numpy"):
            label = label.to_numpy()
        self.X = torch.as_tensor(np.asarray(data, dtype=np.float32) if not torch.is_tensor(data) else data).float()
        self.y = None if label is None else torch.as_tensor(np.asarray(label, dtype=np.float32)).float()
        self.w = None if weight is None else torch.as_tensor(np.asarray(weight, dtype=np.float32)).float()
        self.feature_names = feature_names or [f"f{i}" for i in range(self.X.shape[1])]
        self._binned: Dict[int, Tuple[torch.Tensor, int]] = {}

    @property
    def num_row(self) -> int:
        return int(self.X.shape[0])

    def binned(self, mapper: BinMapper, device) -> Tuple[torch.Tensor, int]:
        key = id(mapper)
        if key not in self._binned:
            self._binned[key] = mapper.transform(self.X.to(device), device)
        return self._binned[key]


# ---------------------------------------------------------------------- booster
class Booster:
    def __init__(self, params: Union[BoostParams, Dict[str, Any], None] = None, device=None):
        self.params = params if isinstance(params, BoostParams) else BoostParams.from_dict(params or {})
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.mapper: Optional[BinMapper] = None
        self.objective = make_objective(self.params.objective, self.params.num_class)
        self.base_margin: List[float] = []
        self.trees: Optional[TreeArrays] = None
        self.feature_names: List[str] = []
        self.best_iteration: Optional[int] = None
        self.best_score: Optional[float] = None

    # ------------------------------------------------------------ tree construction
    @property
    def M(self) -> int:
        return 2 ** (self.params.max_depth + 1) - 1

    def _score(self, G, H):
        p = self.params
        if p.reg_alpha > 0:
            G = torch.sign(G) * (G.abs() - p.reg_alpha).clamp(min=0)
        return G * G / (H + p.reg_lambda)

    def _leaf_value(self, G, H):
        p = self.params
        if p.reg_alpha > 0:
            G = torch.sign(G) * (G.abs() - p.reg_alpha).clamp(min=0)
        w = -G / (H + p.reg_lambda)
        if p.max_delta_step > 0:
            w = w.clamp(-p.max_delta_step, p.max_delta_step)
        return w * p.eta

    def _best_splits(self, hist: torch.Tensor, feat_mask: torch.Tensor):
        """hist [S, F, B, 2] -> per slot (gain, feat, thr_bin, default_left, G, H)."""
        p = self.params
        S, F, B, _ = hist.shape
        miss = hist[:, :, 0, :]                                          # [S, F, 2]
        cum = torch.cumsum(hist[:, :, 1:, :], dim=2)                     # bins 1..B-1
        tot = hist[:, 0].sum(dim=1)                                      # [S, 2]: every row in one bin of f=0
        G, H = tot[:, 0], tot[:, 1]
        parent = self._score(G, H)                                       # [S]
        cand = cum[:, :, :-1, :]                                         # thresholds 1..B-2
        best_gain = torch.full((S,), -float("inf"), device=hist.device)
        best = None
        for dl in (1, 0):                                                # missing left / right
            L = cand + (miss[:, :, None, :] if dl else 0)
            GL, HL = L[..., 0], L[..., 1]
            GR, HR = G[:, None, None] - GL, H[:, None, None] - HL
            gain = self._score(GL, HL) + self._score(GR, HR) - parent[:, None, None]
            ok = (HL >= p.min_child_weight) & (HR >= p.min_child_weight) & feat_mask[None, :, None]
            gain = torch.where(ok, gain, torch.full_like(gain, -float("inf")))
            g, idx = gain.reshape(S, -1).max(dim=1)
            take = g > best_gain
            best_gain = torch.where(take, g, best_gain)
            f = idx // (B - 2)
            t = idx % (B - 2) + 1
            d = torch.full_like(f, dl)
            best = (f, t, d) if best is None else tuple(torch.where(take, a, b) for a, b in zip((f, t, d), best))
        split = torch.isfinite(best_gain) & (best_gain > max(p.gamma, 1e-12))
        return best_gain, best[0], best[1], best[2], G, H, split

    def _grow_tree(self, bins, n_rows, g, h, sampled, feat_mask):
        """Level-wise growth of one tree; returns its arrays and every row's final node."""
        p = self.params
        dev = bins.device
        M = self.M
        feat = torch.full((M,), -1, dtype=torch.int32, device=dev)
        thr = torch.zeros(M, dtype=torch.int32, device=dev)
        dleft = torch.zeros(M, dtype=torch.uint8, device=dev)
        leaf = torch.zeros(M, dtype=torch.float32, device=dev)
        gain_a = torch.zeros(M, dtype=torch.float32, device=dev)
        cover = torch.zeros(M, dtype=torch.float32, device=dev)
        gh = torch.stack([g, h], dim=1).float().contiguous()
        B = self.mapper.max_bin
        rows = torch.arange(n_rows, device=dev)
        node = torch.zeros(n_rows, dtype=torch.int32, device=dev)       # level-local slot, -1 = finished
        final = torch.zeros(n_rows, dtype=torch.long, device=dev)       # global node id
        hist_prev = None
        for level in range(p.max_depth + 1):
            n_level = 1 << level
            first = n_level - 1
            build_node = torch.where(sampled, node, torch.full_like(node, -1))
            if level == 0:
                hist = ops.gbdt_histogram(bins, n_rows, build_node.contiguous(), gh, 1, B)
                _allreduce_(hist)
            else:
                # build the smaller sibling of each pair, derive the other from the parent
                cnt = torch.bincount(build_node[build_node >= 0].long(), minlength=n_level).float()
                _allreduce_(cnt)
                pairs = cnt.view(-1, 2)
                small_is_right = (pairs[:, 1] < pairs[:, 0]).long()               # [n_level/2]
                small = torch.arange(0, n_level, 2, device=dev) + small_is_right
                slot_of = torch.full((n_level,), -1, dtype=torch.int32, device=dev)
                slot_of[small] = torch.arange(n_level // 2, dtype=torch.int32, device=dev)
                bnode = torch.where(build_node >= 0, slot_of[build_node.clamp(min=0).long()],
                                    torch.full_like(build_node, -1)).contiguous()
                part = ops.gbdt_histogram(bins, n_rows, bnode, gh, n_level // 2, B)
                _allreduce_(part)
                hist = torch.empty(n_level, *part.shape[1:], device=dev)
                other = small ^ 1
                hist[small] = part
                hist[other] = hist_prev - part
            gain, f, t, d, G, H, split = self._best_splits(hist, feat_mask)
            gidx = torch.arange(first, first + n_level, device=dev)
            cover[gidx] = H
            if level == p.max_depth:
                split = torch.zeros_like(split)
            # nodes that receive no rows at all stay leaves with value 0
            leaf[gidx] = torch.where(split, torch.zeros_like(G), self._leaf_value(G, H))
            feat[gidx] = torch.where(split, f.int(), torch.full_like(f, -1).int())
            thr[gidx] = t.int()
            dleft[gidx] = d.to(torch.uint8)
            gain_a[gidx] = torch.where(split, gain, torch.zeros_like(gain))
            active = node >= 0
            nd = node.clamp(min=0).long()
            is_split = split[nd] & active
            # rows whose node became a leaf are done
            done = active & ~is_split
            final = torch.where(done, first + nd, final)
            if not bool(split.any()):
                break
            rf = f[nd]
            b = bins[rf, rows].long()
            go_left = torch.where(b == MISSING_BIN, d[nd].bool(), b <= t[nd])
            child = 2 * nd + torch.where(go_left, 0, 1)
            node = torch.where(is_split, child.int(), torch.full_like(node, -1))
            # parents of the next level's pairs; a node that became a leaf has empty children
            hist_prev = hist * split.view(-1, 1, 1, 1)
        return (feat, thr, dleft, leaf, gain_a, cover), final


    def _grow_tree_gpu(self, bins, n_rows, g, h, sampled, feat_mask, margin, k_out):
        """Single process: the whole tree (about 4 launches per level) is captured once into a
        HIP graph and replayed every round, so growth is not bound by host launch latency.
        With several ranks the per-level all-reduces run eagerly instead."""
        import os
        if _dist_on() or os.environ.get("CLOUDTIK_AMD_GBDT_GRAPH", "1") == "0":
            return self._grow_tree_native(bins, n_rows, g, h, sampled, feat_mask, margin, k_out)
        key = (k_out, bins.data_ptr(), n_rows, margin.data_ptr())
        graphs = self.__dict__.setdefault("_graphs", {})
        st = graphs.get(key)
        if st is None:
            bufs = (torch.empty_like(g), torch.empty_like(h), torch.empty_like(sampled), torch.empty_like(feat_mask))
            for b, v in zip(bufs, (g, h, sampled, feat_mask)):
                b.copy_(v)
            side = torch.cuda.Stream(device=bins.device)
            side.wait_stream(torch.cuda.current_stream(bins.device))
            with torch.cuda.stream(side):                    # warm-up: workspace + allocator
                self._grow_tree_native(bins, n_rows, *bufs, margin.clone(), k_out)
            torch.cuda.current_stream(bins.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = self._grow_tree_native(bins, n_rows, *bufs, margin, k_out)
            st = graphs[key] = (graph, bufs, out)
        graph, bufs, out = st
        for b, v in zip(bufs, (g, h, sampled, feat_mask)):
            b.copy_(v)
        graph.replay()
        return tuple(t.clone() for t in out)

    def _grow_tree_native(self, bins, n_rows, g, h, sampled, feat_mask, margin, k_out):
        """GPU tree growth: per level one histogram kernel (smaller children only), one
        split-search kernel (subtraction trick + scan + argmax per node/feature), one
        finalize kernel (tree arrays + next slot map) and one row-partition kernel that also
        adds leaf values to the margin.  No host synchronisation inside the tree."""
        from cloudtik_amd import ops as _ops
        C = _ops.require_native()
        p = self.params
        dev = bins.device
        M, D = self.M, p.max_depth
        F, B = bins.shape[0], self.mapper.max_bin
        feat = torch.full((M,), -1, dtype=torch.int32, device=dev)
        thr = torch.zeros(M, dtype=torch.int32, device=dev)
        dleft = torch.zeros(M, dtype=torch.uint8, device=dev)
        leaf = torch.zeros(M, dtype=torch.float32, device=dev)
        gain = torch.zeros(M, dtype=torch.float32, device=dev)
        cover = torch.zeros(M, dtype=torch.float32, device=dev)
        sf = sampled.float()
        gh = torch.stack([g * sf, h * sf], dim=1).float().contiguous()
        node = torch.zeros(n_rows, dtype=torch.int32, device=dev)
        ws = getattr(self, "_ws", None)
        if ws is None or ws[0].numel() < (1 << D) * F:
            L = (1 << D) * F
            ws = (torch.empty(L, device=dev), torch.empty(L, dtype=torch.int32, device=dev),
                  torch.empty(L, dtype=torch.int32, device=dev), torch.empty(L, device=dev),
                  torch.empty(2 << D, device=dev), torch.empty(0, dtype=torch.int32, device=dev))
            self._ws = ws
        fmask = feat_mask.to(torch.uint8).contiguous()
        hist_prev, smap = None, None
        for level in range(D + 1):
            n_level = 1 << level
            last = level == D
            part = ops.gbdt_histogram(bins, n_rows, node, gh, max(1, n_level // 2), B, slot_map=smap)
            _allreduce_(part)
            hist_cur = torch.empty(n_level, F, B, 2, device=dev)
            slot_next = torch.empty(2 * n_level, dtype=torch.int32, device=dev) if not last else ws[5]
            C.gbdt_level(part, hist_prev, smap, hist_cur, fmask, level, last, p.reg_lambda, p.reg_alpha,
                         p.min_child_weight, p.gamma, p.eta, p.max_delta_step, feat, thr, dleft, leaf, gain, cover,
                         slot_next, ws[0], ws[1], ws[2], ws[3], ws[4])
            C.gbdt_partition(bins, n_rows, node, feat, thr, dleft, leaf, level, margin, k_out)
            hist_prev, smap = hist_cur, slot_next
        return feat, thr, dleft, leaf, gain, cover

    # ------------------------------------------------------------ training
    def _margin_init(self, n: int) -> torch.Tensor:
        K = self.objective.n_outputs
        m = torch.empty(n, K, device=self.device)
        m[:] = torch.tensor(self.base_margin, device=self.device)
        return m

    def train(self, dtrain: DMatrix, num_boost_round: int = 10, evals: Sequence[Tuple[DMatrix, str]] = (),
              early_stopping_rounds: Optional[int] = None, verbose_eval: Union[bool, int] = False,
              callback: Optional[Callable[[int, Dict[str, float]], None]] = None,
              evals_result: Optional[Dict[str, Dict[str, List[float]]]] = None) -> "Booster":
        p = self.params
        dev = self.device
        self.feature_names = dtrain.feature_names
        if self.mapper is None:
            self.mapper = BinMapper(p.max_bin).fit(dtrain.X.to(dev), seed=p.seed)
        bins, n = dtrain.binned(self.mapper, dev)
        y = dtrain.y.to(dev)
        w = dtrain.w.to(dev) if dtrain.w is not None else torch.ones_like(y)
        if not self.base_margin:
            if p.base_score is not None:
                bs = float(p.base_score)
                if isinstance(self.objective, Logistic) and not isinstance(self.objective, LogitRaw):
                    bs = math.log(bs / (1 - bs))
                self.base_margin = [bs] * self.objective.n_outputs
            else:
                self.base_margin = self.objective.base_margin(y, w)
        margin = self._margin_init(n)
        if self.trees is not None:
            margin += self._predict_margin_binned(bins, n)
        eval_sets = []
        for dm, name in evals:
            eb, en = dm.binned(self.mapper, dev)
            em = self._margin_init(en)
            if self.trees is not None:
                em += self._predict_margin_binned(eb, en)
            eval_sets.append((name, eb, en, em, dm.y.to(dev),
                              dm.w.to(dev) if dm.w is not None else torch.ones(en, device=dev)))
        metrics = p.eval_metric or [self._default_metric()]
        # row sampling on the device (no per-round host->device copy); the feature mask is
        # drawn on the host from a seed shared by every rank so all ranks agree on it.  Both
        # are re-seeded from the GLOBAL round index (trees already in the model count), so
        # training in several calls -- the checkpoint segments of elastic training -- draws
        # exactly what one call would
        rank = dist.get_rank() if _dist_on() else 0
        gen = torch.Generator(device=dev)
        fgen = torch.Generator(device="cpu")
        K = self.objective.n_outputs
        F = bins.shape[0]
        start_round = self.num_trees // K
        new_trees: List[Tuple[torch.Tensor, ...]] = []
        best_score, best_it, history = None, None, {}
        for it in range(num_boost_round):
            rnd = start_round + it
            gen.manual_seed((p.seed * 1_000_003 + rank * 7_919 + rnd) & 0x7FFFFFFFFFFFFFFF)
            fgen.manual_seed((p.seed * 1_000_003 + rnd) & 0x7FFFFFFFFFFFFFFF)
            if p.subsample < 1:
                sampled = torch.rand(n, device=dev, generator=gen) < p.subsample
            else:
                sampled = torch.ones(n, dtype=torch.bool, device=dev)
            if p.colsample_bytree < 1:
                k = max(1, int(round(p.colsample_bytree * F)))
                fm = torch.zeros(F, dtype=torch.bool)
                fm[torch.randperm(F, generator=fgen)[:k]] = True
                feat_mask = fm.to(dev)
            else:
                feat_mask = torch.ones(F, dtype=torch.bool, device=dev)
            for k_out, (g, h) in enumerate(self.objective.grad_hess(margin, y, w)):
                if bins.is_cuda:
                    arrays = self._grow_tree_gpu(bins, n, g, h, sampled, feat_mask, margin, k_out)
                else:
                    arrays, final = self._grow_tree(bins, n, g, h, sampled, feat_mask)
                    margin[:, k_out] += arrays[3][final]
                new_trees.append(arrays)
                for (_, eb, en, em, _, _) in eval_sets:
                    em[:, k_out] += self._predict_one(eb, en, arrays)
            scores = {}
            for (name, _, _, em, ey, ew) in eval_sets:
                pred = self.objective.transform(em)
                for mname in metrics:
                    scores[f"{name}-{mname}"] = evaluate_metric(mname, pred, ey, ew)
                    if evals_result is not None:
                        evals_result.setdefault(name, {}).setdefault(mname, []).append(scores[f"{name}-{mname}"])
            if verbose_eval and scores and (verbose_eval is True or it % int(verbose_eval) == 0):
                msg = "\t".join(f"{k}:{v:.5f}" for k, v in scores.items())
                if not _dist_on() or dist.get_rank() == 0:
                    print(f"[{it}]\t{msg}", flush=True)
            if callback:
                callback(rnd, scores)
            if early_stopping_rounds and eval_sets:
                key = f"{eval_sets[-1][0]}-{metrics[-1]}"
                s = scores[key]
                better = best_score is None or (s > best_score if metrics[-1] in MAXIMIZE else s < best_score)
                if better:
                    best_score, best_it = s, it
                elif it - best_it >= early_stopping_rounds:
                    break
            history = scores
        self._append_trees(new_trees)
        self.__dict__.pop("_graphs", None)
        self.best_iteration = best_it if best_it is not None else (self.num_trees // K) - 1
        self.best_score = best_score
        self.last_scores = history
        return self

    def _default_metric(self) -> str:
        return {"reg:squarederror": "rmse", "binary:logistic": "logloss", "binary:logitraw": "logloss",
                "multi:softprob": "mlogloss", "multi:softmax": "mlogloss"}.get(self.objective.name, "rmse")

    def _append_trees(self, new):
        if not new:
            return
        cols = [torch.stack([t[i] for t in new]) for i in range(6)]
        if self.trees is not None:
            cols = [torch.cat([a.to(self.device), b]) for a, b in zip(
                (self.trees.feat, self.trees.thr, self.trees.dleft, self.trees.leaf, self.trees.gain,
                 self.trees.cover), cols)]
        self.trees = TreeArrays(*cols)

    # ------------------------------------------------------------ prediction
    @property
    def num_trees(self) -> int:
        return 0 if self.trees is None else int(self.trees.feat.shape[0])

    def _predict_one(self, bins, n, arrays) -> torch.Tensor:
        feat, thr, dleft, leaf = (a[None] for a in arrays[:4])
        return ops.gbdt_predict(bins, n, feat, thr, dleft, leaf, 1)[:, 0]

    def _predict_margin_binned(self, bins, n, ntree_limit: Optional[int] = None) -> torch.Tensor:
        K = self.objective.n_outputs
        t = self.trees
        T = t.feat.shape[0] if ntree_limit is None else min(t.feat.shape[0], ntree_limit * K)
        dev = bins.device
        return ops.gbdt_predict(bins, n, t.feat[:T].to(dev), t.thr[:T].to(dev), t.dleft[:T].to(dev),
                                t.leaf[:T].to(dev), K)

    def predict(self, data: Union[DMatrix, np.ndarray, torch.Tensor], output_margin: bool = False,
                iteration_range: Optional[Tuple[int, int]] = None) -> np.ndarray:
        dm = data if isinstance(data, DMatrix) else DMatrix(data)
        bins, n = dm.binned(self.mapper, self.device)
        margin = self._margin_init(n)
        if self.trees is not None:
            limit = iteration_range[1] if iteration_range else None
            margin += self._predict_margin_binned(bins, n, limit)
        out = margin if output_margin else self.objective.transform(margin)
        if isinstance(self.objective, SoftmaxClass) and not output_margin:
            out = out.argmax(1, keepdim=True).float()
        out = out.cpu().numpy()
        return out[:, 0] if out.shape[1] == 1 else out

    def get_score(self, importance_type: str = "gain") -> Dict[str, float]:
        """Feature importance: total / average gain, or split count ('weight')."""
        t = self.trees
        f = t.feat.flatten().long().cpu()
        g = t.gain.flatten().cpu()
        m = f >= 0
        F = len(self.feature_names)
        cnt = torch.bincount(f[m], minlength=F).float()
        tot = torch.zeros(F).index_add_(0, f[m], g[m])
        val = {"weight": cnt, "total_gain": tot, "gain": tot / cnt.clamp(min=1)}[importance_type]
        return {self.feature_names[i]: float(val[i]) for i in range(F) if cnt[i] > 0}

    # ------------------------------------------------------------ persistence
    def save_model(self, path: str):
        t = self.trees
        doc = {"format": "cloudtik_amd.gbdt/1", "params": {k: v for k, v in asdict(self.params).items()},
               "base_margin": self.base_margin, "feature_names": self.feature_names,
               "mapper": self.mapper.state_dict(), "best_iteration": self.best_iteration,
               "trees": None if t is None else {k: getattr(t, k).cpu().tolist()
                                                for k in ("feat", "thr", "dleft", "leaf", "gain", "cover")}}
        with open(path, "w") as f:
            json.dump(doc, f)

    @classmethod
    def load_model(cls, path: str, device=None) -> "Booster":
        with open(path) as f:
            doc = json.load(f)
        if doc.get("format") != "cloudtik_amd.gbdt/1":
            raise ValueError(f"{path} is not a cloudtik_amd GBDT model")
        params = BoostParams(**doc["params"])
        b = cls(params, device=device)
        b.base_margin = doc["base_margin"]
        b.feature_names = doc["feature_names"]
        b.mapper = BinMapper.from_state(doc["mapper"])
        b.best_iteration = doc.get("best_iteration")
        tr = doc["trees"]
        if tr:
            dt = {"feat": torch.int32, "thr": torch.int32, "dleft": torch.uint8, "leaf": torch.float32,
                  "gain": torch.float32, "cover": torch.float32}
            b.trees = TreeArrays(**{k: torch.tensor(v, dtype=dt[k], device=b.device) for k, v in tr.items()})
        return b

    def dump_model(self) -> List[Dict[str, Any]]:
        """Trees as nested dicts with raw-value thresholds (x < value goes... see 'split_condition')."""
        out = []
        t = self.trees
        for ti in range(self.num_trees):
            feat, thr, dl, leaf = (t.feat[ti].tolist(), t.thr[ti].tolist(), t.dleft[ti].tolist(), t.leaf[ti].tolist())

            def node(n):
                if feat[n] < 0:
                    return {"nodeid": n, "leaf": leaf[n]}
                return {"nodeid": n, "split": self.feature_names[feat[n]],
                        "split_condition": self.mapper.threshold_value(feat[n], thr[n]),
                        "missing_left": bool(dl[n]), "children": [node(2 * n + 1), node(2 * n + 2)]}
            out.append(node(0))
        return out


def train(params: Dict[str, Any], dtrain: DMatrix, num_boost_round: int = 10, evals=(),
          early_stopping_rounds: Optional[int] = None, verbose_eval: Union[bool, int] = False,
          evals_result: Optional[Dict] = None, device=None) -> Booster:
    """xgboost.train-style entry point."""
    return Booster(params, device=device).train(dtrain, num_boost_round, evals, early_stopping_rounds,
                                                verbose_eval, evals_result=evals_result)
