"""Convolutions on the in-tree implicit-GEMM MFMA kernels (csrc/conv.hip) instead of MIOpen.

Why: MIOpen's immediate mode picks its solver per problem from a user find-db.  On a fresh
node without the right records it either searches (~60 s of warm-up for ResNet-50) or falls
back to naive kernels (25-200 ms per call); the driver measured ResNet-50 at 1,111 img/s on
such a node against 10,149 on a warm one.  These kernels have no solver state: the same code
runs on every box.

Every convolution is planned as ``Y[m, n] = sum_t sum_c X[pixel(m) + tap_t, c] W'[n, t*Ci + c]``
over NHWC (channels_last) bf16 tensors:

* forward: row grid = output pixels, taps = (r - pad, s - pad) at input stride ``stride``;
* data gradient, stride 1: X = dY, taps = (pad - r, pad - s), W' = W transposed to
  [Ci][R][S][Co] (no flip needed: the tap carries the sign);
* data gradient, stride > 1: one launch per output-pixel phase (h mod s, w mod s), with the
  filter taps that reach that phase (a phase no tap reaches is zero-filled);
* weight gradient: a TN implicit GEMM over the pixels (both NHWC operands are pixel-major),
  split-K with fp32 slabs summed by ``splitk_reduce``.

The forward epilogue can also emit per-tile BatchNorm statistics (``stats=True``): the
BatchNorm that follows the conv then skips its statistics pass over the output.

Parity: torchvision ``nn.Conv2d`` semantics (bias-free, groups=1, dilation=1) as the
reference trains them (applications/ai/quickstart/models/image_recognition/pytorch/common/
main.py:276-296); tests compare against ``F.conv2d`` in fp32.
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F

ENABLED = os.environ.get("CLOUDTIK_AMD_CONV_IGEMM", "1") == "1"
_CFG = int(os.environ.get("CLOUDTIK_AMD_CONV_CFG", "-1"))


def _C():
    from cloudtik_amd import ops
    return ops.require_native()


def eligible(x: torch.Tensor, w: torch.Tensor, stride, padding, dilation=(1, 1), groups=1) -> bool:
    """Shapes the kernels take: NHWC bf16 on GPU, Ci and Co multiples of 64, taps within
    [-8, 7], at most 16 taps per launch."""
    if not (ENABLED and x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    co, ci, R, S = w.shape
    if groups != 1 or tuple(dilation) != (1, 1) or ci % 64 or co % 64 or R * S > 16 or x.shape[1] != ci:
        return False
    ph, pw = padding
    if max(R - 1 - ph, S - 1 - pw, ph, pw) > 7:
        return False
    return x.is_contiguous(memory_format=torch.channels_last)


def out_size(h, k, s, p):
    return (h + 2 * p - k) // s + 1


# ------------------------------------------------------------------ plans
def fwd_plan(x_shape, w_shape, stride, padding):
    N, ci, H, W = x_shape
    co, _, R, S = w_shape
    sh, sw = stride
    ph, pw = padding
    Ho, Wo = out_size(H, R, sh, ph), out_size(W, S, sw, pw)
    taps = []
    for r in range(R):
        for s in range(S):
            taps += [r - ph, s - pw]
    geo = [Ho, Wo, sh, sw, Ho, Wo, 1, 1, 0, 0, co, N * Ho * Wo]
    return geo, taps, (N, co, Ho, Wo)


def weight_rows(w: torch.Tensor) -> torch.Tensor:
    """[Co, R*S*Ci] rows of a conv weight (a view when the weight is channels_last)."""
    co = w.shape[0]
    return w.permute(0, 2, 3, 1).reshape(co, -1)


def dgrad_phases(x_shape, w_shape, stride, padding):
    """Per output-pixel phase (a, b) of dX: (row-grid size, taps (dy, dx) into dY, filter taps (r, s))."""
    N, ci, H, W = x_shape
    co, _, R, S = w_shape
    sh, sw = stride
    ph, pw = padding
    out = []
    for a in range(sh):
        for b in range(sw):
            Hr, Wr = (H - a + sh - 1) // sh, (W - b + sw - 1) // sw
            if Hr <= 0 or Wr <= 0:
                continue
            taps, rs = [], []
            for r in range(R):
                if (a + ph - r) % sh:
                    continue
                for s in range(S):
                    if (b + pw - s) % sw:
                        continue
                    taps += [(a + ph - r) // sh, (b + pw - s) // sw]
                    rs.append((r, s))
            out.append(((a, b), (Hr, Wr), taps, rs))
    return out


# ------------------------------------------------------------------ launches
def conv_fwd(x: torch.Tensor, w: torch.Tensor, stride=(1, 1), padding=(0, 0), out: Optional[torch.Tensor] = None,
             accumulate: bool = False, stats: bool = False, partials: bool = False):
    """Y = conv2d(x, w) (NHWC bf16).  With ``stats`` also returns (mean, biased var) per output
    channel of the bf16 Y, from the epilogue's tile partials; with ``partials`` the raw
    partials instead: (Y, part, rows_per_tile), part = means [tiles][Co] then M2 [tiles][Co]
    (what ops.batch_norm_act consumes when Y carries them as ``Y._ct_bn_part``)."""
    geo, taps, shape = fwd_plan(x.shape, w.shape, tuple(stride), tuple(padding))
    N, co, Ho, Wo = shape
    if out is None:
        out = torch.empty(shape, device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    C = _C()
    part = None
    if stats or partials:
        # one (mean, M2) partial per wave row block of the tile (conv.hip cv_wave_stats)
        bm = C.conv_igemm_part_rows(_CFG, co, geo[11], len(taps) // 2 * max(1, x.shape[1] // 64))
        tiles = (geo[11] + bm - 1) // bm
        # + room for the first-level merge of the BatchNorm finalize (batchnorm.hip)
        part = torch.empty((tiles + (tiles + 63) // 64) * 2 * co, device=x.device, dtype=torch.float32)
    ok = C.conv_igemm(x, weight_rows(w).contiguous(), out, geo, taps, accumulate, part, _CFG)
    if not ok:
        raise RuntimeError(f"conv_igemm rejected x{tuple(x.shape)} w{tuple(w.shape)} s{stride} p{padding}")
    if partials:
        return out, part, bm
    if not stats:
        return out
    mean = torch.empty(co, device=x.device, dtype=torch.float32)
    var = torch.empty_like(mean)
    C.bn_partials_finalize(part, bm, geo[11], mean, var)
    return out, mean, var


class _DgradWeights:
    """The data-gradient weight matrices ([Ci, taps * Co], taps flipped per phase) of every
    conv weight that lives in one parameter storage (train.optim.FlatParamSpace), rebuilt by
    ONE gather kernel per backward pass instead of one transposing copy per conv and phase
    (56 small launches on the critical path of a ResNet-50 backward).

    Weights change only between backward passes (optimizer steps), so the matrices are
    refreshed at the first data gradient of each backward (a new autograd graph task); a key
    first seen mid-backward is gathered on its own and joins the batched gather from the next
    pass.  Outside a backward pass (direct calls) nothing is cached."""

    def __init__(self):
        self.groups = {}          # storage ptr -> dict(keys, idx, buf, flat, task, slices)

    @staticmethod
    def _index(w, rs):
        co, ci, R, S = w.shape
        wi = torch.arange(w.storage_offset(), w.storage_offset() + w.numel(), device=w.device).view(co, R, S, ci)
        wti = wi.permute(3, 1, 2, 0)                            # [Ci, R, S, Co] of storage indices
        if len(rs) == R * S:
            return wti.reshape(ci, -1).contiguous()
        return torch.stack([wti[:, r, q, :] for r, q in rs], 1).reshape(ci, -1).contiguous()

    @staticmethod
    def _tiles(keys, slices, device):
        """The 64 x 64 transpose tiles of every key for conv.hip dgrad_wgather_kernel (int32
        [tiles, 10]), or None when a key's channel counts are not multiples of 64."""
        rows = []
        for key in keys:
            soff, (co, ci, R, S), rs = key
            # T | a << 16 | b << 24 must stay a non-negative int32 (b < 128), and the kernel
            # moves 16-B pieces: both offsets must be multiples of 8 elements
            if co % 64 or ci % 64 or co // 64 > 255 or ci // 64 > 127:
                return None
            doff = slices[key][0]
            if soff % 8 or doff % 8:
                return None
            taps = [(r, q) for r in range(R) for q in range(S)] if len(rs) == R * S else list(rs)
            T = len(taps)
            for t, (r, q) in enumerate(taps):
                for a in range(co // 64):
                    for b in range(ci // 64):
                        rows.append([soff >> 16, soff & 0xFFFF, doff >> 16, doff & 0xFFFF, co, ci, R * S * ci,
                                     (r * S + q) * ci, t, T | (a << 16) | (b << 24)])
        return torch.tensor(rows, dtype=torch.int32).to(device) if rows else None

    def get(self, w: torch.Tensor, rs) -> Optional[torch.Tensor]:
        task = torch._C._current_graph_task_id()
        if task == -1 or not w.is_contiguous(memory_format=torch.channels_last):
            return None
        st = w.untyped_storage()
        g = self.groups.get(st.data_ptr())
        if g is None:
            flat = torch.empty(0, dtype=w.dtype, device=w.device).set_(st)
            g = self.groups[st.data_ptr()] = {"keys": {}, "idx": None, "buf": None, "flat": flat, "task": None}
        key = (w.storage_offset(), tuple(w.shape), tuple(rs))
        if key not in g["keys"]:
            idx = self._index(w, rs)
            g["keys"][key] = idx
            g["idx"] = None                                      # rebuild the batched index next pass
            return torch.index_select(g["flat"], 0, idx.view(-1)).view(idx.shape)
        if g["idx"] is None:
            # batched layout: every key's matrix back to back in one buffer
            parts, off, slices = [], 0, {}
            for k, idx in g["keys"].items():
                slices[k] = (off, idx.shape)
                parts.append(idx.view(-1))
                off += idx.numel()
            g["idx"] = torch.cat(parts)
            g["desc"] = self._tiles(g["keys"], slices, w.device) if (
                _DGRAD_WGATHER and w.is_cuda and w.dtype == torch.bfloat16) else None
            if g["flat"].numel() < 2 ** 31:
                # 4-byte indices: the gather reads one index per element (a ResNet-50 pass: 25M
                # elements, 100 MB of indices instead of 200 MB)
                g["idx"] = g["idx"].to(torch.int32)
            g["buf"] = torch.empty(off, dtype=w.dtype, device=w.device)
            g["slices"] = slices
            g["task"] = None
        if g["task"] != task:
            if g.get("desc") is not None:
                _C().dgrad_wgather(g["flat"], g["buf"], g["desc"])
            else:
                torch.index_select(g["flat"], 0, g["idx"], out=g["buf"])
            g["task"] = task
        off, shape = g["slices"][key]
        n = shape[0] * shape[1]
        return g["buf"][off:off + n].view(shape)


_DGRAD_W = _DgradWeights()
_DGRAD_W_CACHE = os.environ.get("CLOUDTIK_AMD_CONV_DGRAD_WCACHE", "1") == "1"
# the batched refresh as tiled transposes (conv.hip dgrad_wgather_kernel) instead of an element gather
_DGRAD_WGATHER = os.environ.get("CLOUDTIK_AMD_CONV_DGRAD_WGATHER", "1") == "1"


BN_BWD_FUSE = os.environ.get("CLOUDTIK_AMD_CONV_BN_BWD_FUSE", "1") == "1"
_DGRAD_ZFILL = os.environ.get("CLOUDTIK_AMD_CONV_DGRAD_ZFILL", "1") == "1"


class BnBwdLink:
    """Hand-off between a BatchNorm + ReLU (mask recomputed from its input, ops.functional
    ``_BNActFn`` mode 2) and the conv that consumes its output.  The conv's data gradient IS the
    BatchNorm's incoming gradient, so the conv epilogue (conv.hip EPI 2) masks it and reduces the
    BatchNorm-backward sums per tile; ``pending`` carries those partials to the BatchNorm's
    backward, which then skips its own reduction pass over dy and x.  The gradient tensor's
    identity and version are recorded so a gradient that autograd summed with another consumer's
    (or modified) is never paired with stale partials."""

    __slots__ = ("x", "stat", "mode", "mask", "pending")

    def __init__(self, x: torch.Tensor, stat: torch.Tensor, mode: int, mask: Optional[torch.Tensor] = None):
        self.x = x
        self.stat = stat
        # 2: mask recomputed from x; 1: mask read from the BN output; 3: the forward's ReLU
        # bitmask (`mask`, uint8, one byte per 8 channels)
        self.mode = mode
        self.mask = mask
        self.pending = None

    def take(self, dy: torch.Tensor):
        """The partials for ``dy`` (part, tiles, rows), or None."""
        p, self.pending = self.pending, None
        if p is None or dy.data_ptr() != p[3] or dy._version != p[4]:
            return None
        return p[:3]


def conv_dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape, stride=(1, 1), padding=(0, 0),
               out: Optional[torch.Tensor] = None, accumulate: bool = False, bn: Optional[BnBwdLink] = None,
               bn_y: Optional[torch.Tensor] = None):
    """dX of conv2d(x, w) for the NHWC bf16 gradient dy; ``accumulate`` adds into ``out``.

    ``bn``: x is the output of that BatchNorm + ReLU; dX (after the accumulate) is returned
    ReLU-masked and the BatchNorm-backward partial sums are left in ``bn.pending`` (see
    BnBwdLink).  ``bn_y`` = x itself, the mask source of a BatchNorm with a residual add."""
    N, ci, H, W = x_shape
    co, _, R, S = w.shape
    phases = dgrad_phases(x_shape, w.shape, tuple(stride), tuple(padding))
    empty_phase = any(not rs for _, _, _, rs in phases)
    C = _C()
    bn_plan = None
    if bn is not None and (bn.mode in (2, 3) or bn_y is not None) and not (accumulate and empty_phase) \
            and bn.x.shape == tuple(x_shape) and co % 64 == 0:
        tiles = []
        for _, (Hr, Wr), taps, rs in phases:
            if rs:
                m = N * Hr * Wr
                bm = C.conv_igemm_tile_m(_CFG, ci, m, len(taps) // 2 * (co // 64))
                tiles.append((m + bm - 1) // bm)
        rows = sum(tiles)
        bn_plan = (torch.empty(2 * rows * ci, device=dy.device, dtype=torch.float32), rows)
    live = [ph for ph in phases if ph[3]]
    # a 1x1 stride-2 data gradient (the downsample convs) writes only the (even, even) pixels:
    # the kernel stores the three odd-parity zeros beside each of them instead of a zero-fill
    # pass over the whole gradient first (conv.hip accumulate mode 2)
    zfill = (_DGRAD_ZFILL and not accumulate and bn_plan is None and len(live) == 1 and live[0][0] == (0, 0)
             and tuple(stride) == (2, 2) and live[0][1] == (H // 2, W // 2) and H % 2 == 0 and W % 2 == 0
             and ci % 8 == 0)
    if out is None:
        out = torch.empty((N, ci, H, W), device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)
    if empty_phase and not accumulate and not zfill:
        out.zero_()
    wt = w.permute(1, 2, 3, 0)                      # [Ci, R, S, Co]
    sh, sw = stride
    tile0 = 0
    # the output phases of a strided data gradient write disjoint pixels (and disjoint rows of
    # the BatchNorm partials): launched on parallel streams, the short launches overlap instead
    # of each draining the GPU in turn
    cur = torch.cuda.current_stream() if dy.is_cuda else None
    streams = _phase_streams(dy.device, len(live) - 1) if (cur is not None and _PHASE_STREAMS and len(live) > 1
                                                           and not zfill) else []
    # every phase's weight matrix first, on this stream (the batched gather of the dgrad weight
    # cache may launch here), then the side streams join it
    mats = [_dgrad_weights(w, wt, rs, R, S, ci) for _, _, _, rs in live]
    for st in streams:
        st.wait_stream(cur)
    # or: the phases' tiles in ONE grid (conv.hip conv_igemm_phases_kernel)
    batch = _PHASE_BATCH and not streams and len(live) > 1 and dy.is_cuda
    if batch:
        C.conv_batch_begin()
    try:
        for i, ((a, b), (Hr, Wr), taps, rs) in enumerate(live):
            st = streams[i - 1] if i > 0 and streams else None
            with (torch.cuda.stream(st) if st is not None else contextlib.nullcontext()):
                tile0 = _dgrad_phase(C, dy, mats[i], ci, co, N, H, W, Hr, Wr, a, b, sh, sw, taps, out, accumulate,
                                     bn, bn_y, bn_plan, tile0, zfill)
            if tile0 is None:                       # the fused epilogue was declined: plain from here on
                bn_plan = None
                tile0 = 0
    finally:
        if batch:
            C.conv_batch_end()

    if streams:
        for st in streams:
            cur.wait_stream(st)
        for t in (dy, out) + ((bn_plan[0],) if bn_plan is not None else ()):
            for st in streams:
                t.record_stream(st)
    if bn_plan is not None:
        bn.pending = (bn_plan[0], tile0, bn_plan[1], out.data_ptr(), out._version)
    return out


_PHASE_STREAMS = os.environ.get("CLOUDTIK_AMD_CONV_PHASE_STREAMS", "0") == "1"
# the output phases of a strided data gradient as one launch (one grid over all their tiles)
_PHASE_BATCH = os.environ.get("CLOUDTIK_AMD_CONV_PHASE_BATCH", "0") == "1"
_PHASE_STREAM_POOL = {}


def _phase_streams(device, n):
    pool = _PHASE_STREAM_POOL.setdefault(device, [])
    while len(pool) < n:
        pool.append(torch.cuda.Stream(device=device))
    return pool[:n]


def _dgrad_weights(w, wt, rs, R, S, ci):
    """[Ci, taps * Co] weight matrix of one data-gradient phase (taps rs, flipped)."""
    wm = _DGRAD_W.get(w, rs) if _DGRAD_W_CACHE else None
    if wm is None:
        if len(rs) == R * S:
            wm = wt.reshape(ci, -1).contiguous()
        else:
            wm = torch.stack([wt[:, r, s, :] for r, s in rs], 1).reshape(ci, -1).contiguous()
    return wm


def _dgrad_phase(C, dy, wm, ci, co, N, H, W, Hr, Wr, a, b, sh, sw, taps, out, accumulate, bn, bn_y, bn_plan, tile0,
                 zfill):
    """One output phase of conv_dgrad; returns the next BatchNorm-partial row, or None when the
    fused BN-backward epilogue was declined on the first phase."""
    geo = [Hr, Wr, 1, 1, H, W, sh, sw, a, b, ci, N * Hr * Wr]
    if bn_plan is not None:
        part, rows = bn_plan
        msrc = bn.mask if bn.mode == 3 else (bn_y if bn.mode == 1 else None)
        if C.conv_igemm_bn(dy, wm, out, geo, taps, accumulate, _CFG, bn.x, msrc, bn.stat, part, tile0, rows):
            bm = C.conv_igemm_tile_m(_CFG, ci, geo[11], len(taps) // 2 * (co // 64))
            return tile0 + (geo[11] + bm - 1) // bm
        if tile0:
            raise RuntimeError("conv_igemm_bn rejected a later phase of a supported data gradient")
        if not C.conv_igemm(dy, wm, out, geo, taps, int(accumulate), None, _CFG):
            raise RuntimeError(f"conv_igemm (dgrad) rejected dy{tuple(dy.shape)}")
        return None                                 # configuration without the fused epilogue
    if not C.conv_igemm(dy, wm, out, geo, taps, 2 if zfill else int(accumulate), None, _CFG):
        if zfill:                                   # shape the zero-filling mode refuses
            out.zero_()
            if C.conv_igemm(dy, wm, out, geo, taps, 0, None, _CFG):
                return tile0
        raise RuntimeError(f"conv_igemm (dgrad) rejected dy{tuple(dy.shape)}")
    return tile0


_WG_CFG = int(os.environ.get("CLOUDTIK_AMD_CONV_WGRAD_CFG", "-1"))
# 1x1 stride-1 weight gradients with 256-multiple channel counts on the TN GEMM kernel
# (2: every 256-multiple shape; 1: only where it beats the implicit-GEMM kernel's linear 1x1 mode
# alone -- 32K-64K pixels and 1024+ output channels: l3.c3 57 vs 66 us, but l3.c1a at 200K pixels
# 164 vs 88 us, l4.c3 47 vs 43 (bench/wgrad3x3_probe.py).  In the step rule 1 is SLOWER, 21.37 ->
# 21.46 ms (profiles/r5/wgrad3x3.md): the TN GEMM's few large tiles leave the data gradients on the
# main stream more of the chip; 0: never)
_TN_WGRAD_1X1 = int(os.environ.get("CLOUDTIK_AMD_CONV1X1_TN_WGRAD", "2"))
_WG_TILES = {0: (64, 64), 1: (64, 128), 2: (128, 128), 3: (128, 256), 4: (64, 64), 5: (64, 128), 6: (128, 128),
             7: (64, 64), 8: (64, 64), 9: (128, 128), 10: (128, 128), 11: (128, 256), 12: (64, 576), 13: (64, 576),
             14: (128, 64), 15: (64, 256)}
# 3x3 / stride 1 or 2 / pad 1 weight gradients on the nine-tap kernel (conv.hip conv_wgrad3x3_kernel):
# one workgroup owns 64 output x 64 input channels of all nine taps.  -1 = auto (cfg 12, a 3-slot
# ring at one workgroup per CU; cfg 13, 2 slots at two per CU and twice the split-K workgroups,
# where the channel tiles alone make 64+ workgroups), 0 = the per-tap tiles, 12 / 13 = forced.
# Probe (bench/wgrad3x3_probe.py, batch 256): l1.c2 297 -> 95 us, l2.c2 130 -> 92, l3.c2 108 -> 79,
# l4.c2 140 -> 72
_WG3X3 = int(os.environ.get("CLOUDTIK_AMD_WGRAD3X3", "-1"))
_WG3X3_S2 = os.environ.get("CLOUDTIK_AMD_WGRAD3X3_S2", "1") == "1"
_WG3X3_MAXCI = int(os.environ.get("CLOUDTIK_AMD_WGRAD3X3_MAXCI", "4096"))
PARTIAL_BYTES = 64 << 20           # cap of the fp32 split-K slabs per weight gradient
WGRAD_BLOCKS = int(os.environ.get("CLOUDTIK_AMD_WGRAD_BLOCKS", "256"))   # split-K target workgroups
# the same target for the tiles narrower than 128 x 256 (cfg 3 / 11 keep WGRAD_BLOCKS): at 256
# workgroups the 64-wide 4-wave tiles run one wave per SIMD (l1.c2 299 us, 187 at 512)
WGRAD_BLOCKS_SMALL = int(os.environ.get("CLOUDTIK_AMD_WGRAD_BLOCKS_SMALL", "256"))
WGRAD3X3_BLOCKS = int(os.environ.get("CLOUDTIK_AMD_WGRAD3X3_BLOCKS", "128"))
# the stem's weight gradient is the last kernel of the backward, alone on the chip: small tiles,
# many workgroups (bench/stem_wgrad_probe.py, NHWC4: the auto 64 x 128 tile at 256 workgroups
# 418 us -> 64 x 64 at 1,024: 218 us)
STEM_WGRAD_BLOCKS = int(os.environ.get("CLOUDTIK_AMD_STEM_WGRAD_BLOCKS", "1024"))
STEM_WGRAD_CFG = int(os.environ.get("CLOUDTIK_AMD_STEM_WGRAD_CFG", "0"))


def wgrad_plan(M: int, co: int, nn: int, cfg: int, blocks: Optional[int] = None):
    """(splits, rows per split): about ``blocks`` workgroups (default: the per-configuration
    target), each split a multiple of the stage depth and at least 256 deep, the fp32 partials
    capped at PARTIAL_BYTES."""
    bm, bn = _WG_TILES[cfg]
    tiles = (co // bm) * (nn // bn)
    given = blocks
    blocks = WGRAD_BLOCKS if cfg in (3, 11) else WGRAD_BLOCKS_SMALL
    if cfg >= 12:                      # nine-tap kernel: cfg 13 runs two workgroups per CU
        blocks = WGRAD3X3_BLOCKS * (2 if cfg == 13 else 1)
    if given is not None:
        blocks = given
    splits = max(1, min(blocks // max(1, tiles), M // 256, PARTIAL_BYTES // (co * nn * 4)))
    q = 64 if cfg >= 4 and cfg != 9 else 32        # pixels per stage of the configuration
    rows = ((M + splits - 1) // splits + q - 1) // q * q
    return (M + rows - 1) // rows, rows


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, w_shape, stride=(1, 1), padding=(0, 0),
               out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    """dW of conv2d(x, w) (NHWC bf16 dy, x) as a channels_last bf16 [Co, Ci, R, S] tensor;
    ``out`` (same memory layout, e.g. a flat-buffer gradient view) receives it, added when
    ``accumulate``."""
    co, ci, R, S = w_shape
    taps = []
    for r in range(R):
        for s in range(S):
            taps += [r - padding[0], s - padding[1]]
    nn = R * S * ci
    M = dy.shape[0] * dy.shape[2] * dy.shape[3]
    if (_TN_WGRAD_1X1 and R == 1 and S == 1 and tuple(stride) == (1, 1) and tuple(padding) == (0, 0)
            and co % 256 == 0 and ci % 256 == 0 and M % 64 == 0
            and (_TN_WGRAD_1X1 == 2 or (32768 < M <= 65536 and co >= 1024))
            and dy.is_contiguous(memory_format=torch.channels_last)
            and x.is_contiguous(memory_format=torch.channels_last)):
        # a 1x1 stride-1 weight gradient IS the linear one, dW = dY^T X over the pixel rows: the
        # 256 x 256 TN MFMA GEMM with split-K (ops.linear.wgrad_accumulate) instead of the
        # 128-wide implicit-GEMM tiles
        from cloudtik_amd.ops.linear import wgrad_accumulate
        if out is None or not accumulate:
            out = (out if out is not None else torch.empty(
                w_shape, device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)).zero_()
        g2 = out.permute(0, 2, 3, 1).reshape(co, ci)
        if g2.data_ptr() == out.data_ptr() and g2.is_contiguous():
            wgrad_accumulate(g2, dy.permute(0, 2, 3, 1).reshape(M, co), x.permute(0, 2, 3, 1).reshape(M, ci))
            return out
    C = _C()
    cfg = C.conv_wgrad_cfg(_WG_CFG, co, nn)
    if (_WG_CFG < 0 and _WG3X3 != 0 and R == 3 and S == 3
            and (tuple(stride) == (1, 1) or (_WG3X3_S2 and tuple(stride) == (2, 2)))
            and tuple(padding) == (1, 1) and ci % 64 == 0 and co % 64 == 0 and ci <= _WG3X3_MAXCI
            and max(x.numel(), dy.numel()) * 2 < 2 ** 31):      # 32-bit buffer offsets
        cfg = _WG3X3 if _WG3X3 > 0 else (13 if (co // 64) * (ci // 64) >= 64 else 12)
    splits, rows = wgrad_plan(M, co, nn, cfg)
    part = torch.empty(splits * co * nn, device=dy.device, dtype=torch.float32)
    if not C.conv_wgrad(dy, x, part, taps, [stride[0], stride[1], rows], splits, cfg):
        raise RuntimeError(f"conv_wgrad rejected dy{tuple(dy.shape)} x{tuple(x.shape)} w{tuple(w_shape)}")
    if out is None:
        out = torch.empty(w_shape, device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)
        accumulate = False
    flat = out.permute(0, 2, 3, 1).reshape(-1) if out.dim() == 4 else out.reshape(-1)
    if splits <= 16:
        C.splitk_reduce(part.view(splits, -1), flat, accumulate)
    else:                                   # many slabs: parallel over the slabs too
        C.splitk_reduce_wide(part, splits, flat, accumulate)
    return out


def _weight_grad(wp, dy, x, w_shape, stride, padding):
    """dW.  When the weight lives in a flat gradient buffer (train.optim.FlatParamSpace) and the
    gradient side stream is on, the split-K reduce ADDS it straight into its buffer slice on the
    side stream (returns None: autograd never sees it, the data-parallel bucketer is told through
    ``_ct_grad_ready``); otherwise it is returned for AccumulateGrad."""
    from cloudtik_amd.ops.conv1x1 import _SIDE_WGRAD, _flat_target
    from cloudtik_amd.ops.linear import side_grad_stream, wgrad_side
    target = _flat_target(wp) if _SIDE_WGRAD else None
    side = side_grad_stream() if (target is not None and wgrad_side(wp)) else None
    if target is None or not target.is_contiguous(memory_format=torch.channels_last) or target.dtype != dy.dtype:
        return conv_wgrad(dy, x, w_shape, stride, padding)
    if side is None:
        conv_wgrad(dy, x, w_shape, stride, padding, out=target, accumulate=True)
    else:
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            conv_wgrad(dy, x, w_shape, stride, padding, out=target, accumulate=True)
        dy.record_stream(side)
        x.record_stream(side)
    cb = getattr(wp, "_ct_grad_ready", None)
    if cb is not None:
        cb(wp)
    return None


# Weight gradients held back until the BatchNorm backward that consumes the same data gradient
# has launched its kernels (ConvFn.backward -> functional._BNActFn.backward): a side-stream
# weight gradient issued first takes the CUs its big grid can fill, and the short main-stream
# BatchNorm kernels queued behind the data gradient then wait for slots (ResNet-50: ~34 such
# main-stream gaps a step, 0.5 ms; 22.05 -> 21.91 ms/step deferred).  Issued after the NEXT data
# gradient instead measured no better than not deferring.  A callback at the end of the
# backward pass flushes anything left.
_DEFER_WGRAD = os.environ.get("CLOUDTIK_AMD_DEFER_WGRAD", "1") == "1"
_DEFERRED_WGRADS: list = []


def flush_deferred_wgrads() -> None:
    while _DEFERRED_WGRADS:
        _DEFERRED_WGRADS.pop(0)()


def _weight_grad_lands_in_buffer(wp, dy) -> bool:
    """Whether _weight_grad writes the gradient into the flat buffer itself (returns None)."""
    from cloudtik_amd.ops.conv1x1 import _SIDE_WGRAD, _flat_target
    target = _flat_target(wp) if _SIDE_WGRAD else None
    return (target is not None and target.is_contiguous(memory_format=torch.channels_last)
            and target.dtype == dy.dtype)


class ConvFn(torch.autograd.Function):
    """conv2d on the implicit-GEMM kernels.  ``keep_input`` also returns an alias of x for the
    block's other consumer (the residual / downsample branch): autograd then sees x used once
    and the data gradient of this conv is accumulated INTO the other branch's gradient by the
    kernel's epilogue (no separate add pass)."""

    @staticmethod
    def forward(ctx, x, w, stride, padding, keep_input, bn_stats=False):
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.padding = stride, padding
        ctx.wp = w
        # x = the output of a BatchNorm + ReLU: its backward reduction runs in our dgrad epilogue
        ctx.bn_link = getattr(x, "_ct_bn_bwd", None) if BN_BWD_FUSE else None
        if bn_stats:
            # the epilogue reduces the BatchNorm statistics of y per tile; the BatchNorm that
            # consumes y picks them up instead of re-reading y for a statistics pass
            y, part, rows = conv_fwd(x, w, stride, padding, partials=True)
            y._ct_bn_part = (part, rows)
        else:
            y = conv_fwd(x, w, stride, padding)
        return (y, x.view_as(x)) if keep_input else y

    @staticmethod
    def backward(ctx, dy, dx_other=None):
        flush_deferred_wgrads()             # normally the BatchNorm backward has done it
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if (dx_other is not None and not torch.is_grad_enabled() and dx_other.dtype == dy.dtype
                    and dx_other.is_contiguous(memory_format=torch.channels_last)):
                # (a BatchNorm with a residual add: x is its output, the ReLU mask source)
                dx = conv_dgrad(dy, w, x.shape, ctx.stride, ctx.padding, out=dx_other, accumulate=True,
                                bn=ctx.bn_link, bn_y=x)
            else:
                dx = conv_dgrad(dy, w, x.shape, ctx.stride, ctx.padding,
                                bn=ctx.bn_link if dx_other is None else None, bn_y=x)
                if dx_other is not None:
                    dx = dx + dx_other
        if ctx.needs_input_grad[1]:
            args = (ctx.wp, dy, x, tuple(w.shape), ctx.stride, ctx.padding)
            if (_DEFER_WGRAD and ctx.bn_link is not None and ctx.bn_link.pending is not None
                    and _weight_grad_lands_in_buffer(ctx.wp, dy)):
                if not _DEFERRED_WGRADS:
                    torch.autograd.Variable._execution_engine.queue_callback(flush_deferred_wgrads)
                _DEFERRED_WGRADS.append(lambda: _weight_grad(*args))
            else:
                dw = _weight_grad(*args)
        return dx, dw, None, None, None, None


BN_STATS = os.environ.get("CLOUDTIK_AMD_CONV_BN_STATS", "1") == "1"

# forward convolutions by route since import: "igemm" = the in-tree MFMA kernels (stem
# included), "library" = the module's own forward (MIOpen).  bench.py's ResNet audit reads the
# delta over one step -- an exact count, unlike a kernel trace taken in-process.
ROUTES = {"igemm": 0, "library": 0}


def conv2d(x: torch.Tensor, conv: torch.nn.Conv2d, keep_input: bool = False, bn_stats: bool = False):
    """``conv(x)`` on the implicit-GEMM kernels when eligible, else ``conv(x)``; with
    ``keep_input`` returns ``(conv(x), x_alias)`` (see ConvFn); ``bn_stats``: the output feeds a
    training-mode BatchNorm, so the epilogue also reduces its statistics."""
    if conv.bias is not None or not eligible(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups):
        ROUTES["library"] += 1
        return (conv(x), x) if keep_input else conv(x)
    ROUTES["igemm"] += 1
    return ConvFn.apply(x, conv.weight, tuple(conv.stride), tuple(conv.padding), keep_input,
                        bool(bn_stats and BN_STATS))


# ------------------------------------------------------------------ the stem (Ci = 3)
def stem_eligible(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    """ResNet's 7x7/2 stem over an RGB bf16 image batch on GPU (any 3-channel conv with
    R, S <= 8 works: the kernel's pixel-chunk mode)."""
    w = conv.weight
    return (ENABLED and x.is_cuda and x.dim() == 4 and x.shape[1] <= 8 and w.dtype == torch.bfloat16
            and not x.requires_grad
            and x.dtype == torch.bfloat16 and conv.bias is None and conv.groups == 1
            and tuple(conv.dilation) == (1, 1) and w.shape[2] <= 7 and w.shape[3] <= 8 and w.shape[0] % 64 == 0
            and max(conv.padding) <= 7)


_STEM_NHWC8_KERNEL = os.environ.get("CLOUDTIK_AMD_STEM_NHWC8_KERNEL", "1") == "1"
# pair-chunk stem mode (conv.hip pixchunk 2): the image padded to 4 channels, a 64-column K-step =
# 2 filter rows x 8 pixels x 4 channels, so a 7x7 RGB stem takes 4 K-steps (57 % useful
# columns) instead of 7 (33 %).  Needs stride 2 along x, an even image width and an odd x padding
# (the 8-pixel window starts at x * 2 - pad - 1: even, 16-byte aligned)
_STEM_PAIRS = os.environ.get("CLOUDTIK_AMD_STEM_PAIRS", "1") == "1"


def stem_pairs(x_shape, w_shape, stride, padding) -> bool:
    """Whether the stem conv takes the pair-chunk mode."""
    co, c, R, S = w_shape
    return (_STEM_PAIRS and c <= 4 and stride[1] == 2 and x_shape[3] % 2 == 0 and padding[1] % 2 == 1
            and S + 1 <= 8 and padding[1] + 1 <= 8)


def to_nhwc8(x: torch.Tensor, cp: int = 8) -> torch.Tensor:
    """[N, C<=cp, H, W] -> NHWC with the channels zero-padded to cp (8: 16 bytes per pixel; 4: the
    pair-chunk stem mode), returned as the logical [N, cp, H, W] channels_last view the kernels
    take."""
    n, c, h, w = x.shape
    # the kernel is not differentiable: an input that needs a gradient takes the autograd path
    if (x.is_cuda and x.dtype == torch.bfloat16 and _STEM_NHWC8_KERNEL
            and not (x.requires_grad and torch.is_grad_enabled())):
        return _C().to_nhwc8(x, cp)                 # one pass (conv.hip to_nhwc8_kernel)
    return F.pad(x.permute(0, 2, 3, 1), (0, cp - c)).contiguous().permute(0, 3, 1, 2)


def _stem_taps(R, pad, pairs=False):
    taps = []
    if pairs:
        for r in range(0, R, 2):               # kernel rows r, r + 1; pixels x*2 - pad - 1 .. + 7
            taps += [r - pad[0], -pad[1] - 1]
        return taps
    for r in range(R):
        taps += [r - pad[0], -pad[1]]          # the K-step's 8 pixels start at x*s - pad
    return taps


def stem_weight(w: torch.Tensor, pairs=False) -> torch.Tensor:
    """[Co, C, R, S] -> [Co, R * 64]: column r*64 + s*8 + c = w[co, c, r, s] (zero-padded); pair
    mode [Co, ceil(R / 2) * 64]: column = r*32 + (s + 1)*4 + c (the window's first pixel and the
    channels past C are zero)."""
    co, c, R, S = w.shape
    if pairs:
        T = (R + 1) // 2
        wp = torch.zeros(co, 2 * T, 8, 4, device=w.device, dtype=w.dtype)
        wp[:, :R, 1:S + 1, :c] = w.permute(0, 2, 3, 1)
        return wp.reshape(co, T * 64)
    wp = torch.zeros(co, R, 8, 8, device=w.device, dtype=w.dtype)
    wp[:, :, :S, :c] = w.permute(0, 2, 3, 1)
    return wp.reshape(co, R * 64)


# the stem conv's epilogue reduces the BatchNorm statistics of its output per tile (EPI 1), so the
# fused BN + ReLU + max-pool skips its statistics pass over the 112x112x64 activation
_STEM_STATS = os.environ.get("CLOUDTIK_AMD_STEM_STATS", "1") == "1"


def stem_fwd(x8: torch.Tensor, w: torch.Tensor, stride, padding, partials: bool = False) -> torch.Tensor:
    """The stem conv of an NHWC8 (or, pair mode, NHWC4) image batch; with ``partials`` the output
    carries its BatchNorm tile statistics as ``_ct_bn_part`` (ops.batch_norm_relu_maxpool consumes
    them)."""
    n, cp, H, W = x8.shape
    co, c, R, S = w.shape
    pairs = cp == 4
    Ho, Wo = out_size(H, R, stride[0], padding[0]), out_size(W, S, stride[1], padding[1])
    out = torch.empty((n, co, Ho, Wo), device=x8.device, dtype=x8.dtype, memory_format=torch.channels_last)
    geo = [Ho, Wo, stride[0], stride[1], Ho, Wo, 1, 1, 0, 0, co, n * Ho * Wo]
    C = _C()
    part = bm = None
    if partials:
        bm = C.conv_igemm_part_rows(_CFG, co, geo[11], len(_stem_taps(R, padding, pairs)) // 2)
        tiles = (geo[11] + bm - 1) // bm
        part = torch.empty((tiles + (tiles + 63) // 64) * 2 * co, device=x8.device, dtype=torch.float32)
    if not C.conv_igemm(x8, stem_weight(w, pairs), out, geo, _stem_taps(R, padding, pairs), False, part, _CFG):
        raise RuntimeError(f"conv_igemm (stem) rejected x{tuple(x8.shape)} w{tuple(w.shape)}")
    if partials:
        out._ct_bn_part = (part, bm)
    return out


def stem_wgrad(dy: torch.Tensor, x8: torch.Tensor, w_shape, stride, padding, fp32: bool = False,
               blocks: Optional[int] = None) -> torch.Tensor:
    """dW of the stem conv as channels_last [Co, C, R, S]: bf16, or (``fp32``) the fp32 sums
    (ops.functional._StemBlockFn combines three of them)."""
    co, c, R, S = w_shape
    pairs = x8.shape[1] == 4
    T = (R + 1) // 2 if pairs else R
    nn = T * 64
    M = dy.shape[0] * dy.shape[2] * dy.shape[3]
    C = _C()
    cfg = C.conv_wgrad_cfg(_WG_CFG if _WG_CFG >= 0 else STEM_WGRAD_CFG, co, nn)
    # the stem's weight gradient is the last kernel of the backward, on the main stream with the
    # chip to itself: split it over more workgroups than the side-stream gradients
    splits, rows = wgrad_plan(M, co, nn, cfg, STEM_WGRAD_BLOCKS if blocks is None else blocks)
    part = torch.empty(splits * co * nn, device=dy.device, dtype=torch.float32)
    if not C.conv_wgrad(dy, x8, part, _stem_taps(R, padding, pairs), [stride[0], stride[1], rows], splits, cfg):
        raise RuntimeError(f"conv_wgrad (stem) rejected dy{tuple(dy.shape)} x{tuple(x8.shape)}")
    if fp32:
        full = part.view(splits, -1).sum(0)
    else:
        full = torch.empty(co * nn, device=dy.device, dtype=dy.dtype)
        if splits <= 16:
            C.splitk_reduce(part.view(splits, -1), full, False)
        else:
            C.splitk_reduce_wide(part, splits, full, False)
    if pairs:
        full = full.view(co, 2 * T, 8, 4)[:, :R, 1:S + 1, :c]
    else:
        full = full.view(co, R, 8, 8)[:, :, :S, :c]
    return full.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)


class StemFn(torch.autograd.Function):
    """conv2d of a <= 8-channel image batch (no input gradient: it is the network input)."""

    @staticmethod
    def forward(ctx, x8, w, stride, padding):
        ctx.save_for_backward(x8)
        ctx.stride, ctx.padding, ctx.w_shape = stride, padding, tuple(w.shape)
        ctx.wp = w
        return stem_fwd(x8, w, stride, padding, partials=_STEM_STATS)

    @staticmethod
    def backward(ctx, dy):
        (x8,) = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dw = None
        if ctx.needs_input_grad[1]:
            dw = stem_wgrad(dy, x8, ctx.w_shape, ctx.stride, ctx.padding)
            from cloudtik_amd.ops.conv1x1 import _flat_target
            target = _flat_target(ctx.wp)
            if target is not None:                    # straight into the flat gradient buffer
                target.add_(dw)
                cb = getattr(ctx.wp, "_ct_grad_ready", None)
                if cb is not None:
                    cb(ctx.wp)
                dw = None
        return None, dw, None, None


def stem_conv(x: torch.Tensor, conv: torch.nn.Conv2d) -> torch.Tensor:
    """``conv(x)`` for the image-batch stem on the kernels' pixel-chunk mode when eligible."""
    if not stem_eligible(x, conv):
        ROUTES["library"] += 1
        return conv(x)
    ROUTES["igemm"] += 1
    cp = 4 if stem_pairs(x.shape, conv.weight.shape, tuple(conv.stride), tuple(conv.padding)) else 8
    return StemFn.apply(to_nhwc8(x, cp), conv.weight, tuple(conv.stride), tuple(conv.padding))
