"""cloudtik_amd op library: hand-written CDNA4 (gfx950) HIP kernels + autograd wrappers.

Dispatch rule (no silent fallback on the GPU path):

* tensors on a ROCm device  -> the HIP kernel in ``_C`` is REQUIRED; if the extension
  is missing the call raises (build it with ``python -m cloudtik_amd.ops.build``).
* CPU tensors               -> a plain PyTorch reference implementation
  (``cloudtik_amd.ops.reference``), used by the CPU test-suite and by gloo-only
  configs (north-star config #1: MNIST MLP on CPU).

The reference implementations double as the fp32 oracle the GPU numerics tests compare
against.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch

from . import reference as ref


from . import miopen_solvers as _miopen_db  # noqa: E402

# MIOpen solver records for this framework's conv shapes (see ops/miopen_solvers.py): installed
# before anything creates a MIOpen handle; never silently skipped (bench.py prints status())
_miopen_db.install()

_C_ERR = None
try:  # the extension is built in-tree (see ops/build.py)
    _C = importlib.import_module(__name__ + "._C")
except Exception as e:  # pragma: no cover - depends on build state
    _C = None
    _C_ERR = e


def _check_build_current():
    """The library must have been linked from the sources in this tree: a stale ``.so`` (sources
    edited, or reverted, without a rebuild) would run other kernels than the ones the tree
    shows.  Warns; ``CLOUDTIK_AMD_STRICT_BUILD=1`` raises instead."""
    if _C is None:
        return
    try:
        from .build import stale_sources
        stale = stale_sources()
    except Exception:  # noqa: BLE001 - a missing csrc dir (installed package) is not an error
        return
    if stale:
        msg = ("cloudtik_amd: the in-tree HIP library was built from other sources than "
               f"{', '.join(stale[:6])}{' ...' if len(stale) > 6 else ''}; run `python -m cloudtik_amd.ops.build`")
        if os.environ.get("CLOUDTIK_AMD_STRICT_BUILD", "0") == "1":
            raise RuntimeError(msg)
        import warnings
        warnings.warn(msg, RuntimeWarning, stacklevel=2)


_check_build_current()


def native_available() -> bool:
    return _C is not None


def require_native():
    if _C is None:
        raise RuntimeError(
            "cloudtik_amd HIP op library (_C) is not built or failed to load: %r. "
            "Run `python -m cloudtik_amd.ops.build`." % (_C_ERR,))
    return _C


def _use_native(*tensors) -> bool:
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            require_native()
            return True
    return False


# --------------------------------------------------------------------------- RNG streams
class _DropoutRNG(threading.local):
    """(seed, offset) pairs for the counter-based (hash) dropout kernels.

    Each dropout site draws a fresh 64-bit offset; the kernels regenerate the mask in
    backward from the same pair, so no mask is ever stored."""

    def __init__(self):
        self.seed = int(os.environ.get("CLOUDTIK_AMD_SEED", "24301"))
        self.offset = 0

    def next(self, n_elements: int = 1):
        off = self.offset
        self.offset += max(1, (n_elements + 7) // 8)
        return self.seed, off


_rng = _DropoutRNG()


def manual_seed(seed: int):
    _rng.seed = int(seed) & ((1 << 63) - 1)
    _rng.offset = 0


def rng_state():
    return {"seed": _rng.seed, "offset": _rng.offset}


def set_rng_state(state):
    _rng.seed = int(state["seed"])
    _rng.offset = int(state["offset"])


from .functional import (  # noqa: E402,F401
    layer_norm, bias_act, bias_gelu, dropout, embedding3, cross_entropy_fused, batch_norm_act,
    batch_norm_relu_maxpool, batch_norm_add_bn_act, stem_block,
    ACT_NONE, ACT_GELU, ACT_RELU,
)
from .attention import attention, attention_packed, attention_relbias  # noqa: E402,F401
from .linear import linear  # noqa: E402,F401
from .rope import apply_rotary, rotary_cache  # noqa: E402,F401
from .embedding import EmbeddingBagCollection, dot_interaction, embedding_bag, pack_bags  # noqa: E402,F401
from .vision import batched_nms, images_to_tensor, nms, nms_segments, roi_align, roi_align_multilevel, roi_pool, sigmoid_focal_loss  # noqa: E402,F401
from . import multi_tensor  # noqa: E402,F401
from .graph import CSR, SpMM, gbdt_histogram, gbdt_predict, spmm  # noqa: E402,F401
from .deform import (DeformConv, DeformRoIPooling, DeformRoIPoolingPack, ModulatedDeformConv,  # noqa: E402,F401
                     ModulatedDeformConvPack, deform_conv2d, deform_roi_pooling)
from .rnnt import rnnt_loss, rnnt_loss_reference  # noqa: E402,F401
