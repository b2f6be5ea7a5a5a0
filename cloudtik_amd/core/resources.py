"""Node resource detection: CPU, memory and AMD GPUs (MI355X).

Replaces the reference's NVIDIA-centric detection (``core/_private/resource_spec.py:183-200``:
CUDA_VISIBLE_DEVICES / GPUtil / /proc/driver/nvidia/gpus) with ROCm sources, in order:

1. ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` if set;
2. the KFD topology (``/sys/class/kfd/kfd/topology/nodes/*/properties``: a node with a
   non-zero ``gfx_target_version`` is a GPU) -- no GPU context is created, so this is safe
   to call from any control-plane process;
3. ``amdsmi`` when importable.

The accelerator type (e.g. ``gfx950`` -> ``MI355X``) is reported as a custom resource
``accelerator_type:MI355X`` so scaling policies can target it.
"""
from __future__ import annotations

import glob
import os
from typing import Dict, List, Optional

import psutil

from cloudtik_amd.core import constants

KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"
GFX_NAMES = {"gfx950": "MI355X", "gfx942": "MI300X", "gfx90a": "MI250X", "gfx908": "MI100"}


def _visible_devices_env() -> Optional[List[str]]:
    for k in constants.CLOUDTIK_ROCM_VISIBLE_ENVS:
        v = os.environ.get(k)
        if v is not None:
            v = v.strip()
            if v in ("", "NoDevFiles"):
                return []
            return [x for x in v.split(",") if x != ""]
    return None


def kfd_gpu_nodes(root: str = KFD_TOPOLOGY) -> List[Dict[str, int]]:
    gpus = []
    for props in sorted(glob.glob(os.path.join(root, "*", "properties"))):
        kv = {}
        try:
            with open(props) as f:
                for line in f:
                    parts = line.split()
                    if len(parts) == 2 and parts[1].lstrip("-").isdigit():
                        kv[parts[0]] = int(parts[1])
        except OSError:
            continue
        if kv.get("gfx_target_version", 0) and kv.get("simd_count", 0) > 0:
            gpus.append(kv)
    return gpus


def gfx_name(target_version: int) -> str:
    """gfx_target_version 90500 -> gfx950 (major*10000 + minor*100 + stepping)."""
    major, minor, step = target_version // 10000, (target_version // 100) % 100, target_version % 100
    return f"gfx{major}{minor:x}{step:x}"


def detect_amd_gpu_count(kfd_root: str = KFD_TOPOLOGY) -> int:
    env = _visible_devices_env()
    if env is not None:
        return len(env)
    nodes = kfd_gpu_nodes(kfd_root)
    if nodes:
        return len(nodes)
    try:
        import amdsmi  # type: ignore
        amdsmi.amdsmi_init()
        try:
            return len(amdsmi.amdsmi_get_processor_handles())
        finally:
            amdsmi.amdsmi_shut_down()
    except Exception:  # noqa: BLE001
        return 0


def detect_accelerator_type(kfd_root: str = KFD_TOPOLOGY) -> Optional[str]:
    nodes = kfd_gpu_nodes(kfd_root)
    if not nodes:
        return None
    g = gfx_name(nodes[0]["gfx_target_version"])
    return GFX_NAMES.get(g, g)


def detect_resources(override: Optional[Dict[str, float]] = None, kfd_root: str = KFD_TOPOLOGY) -> Dict[str, float]:
    res = {"CPU": float(psutil.cpu_count(logical=True) or 1),
           "memory": float(psutil.virtual_memory().total)}
    ngpu = detect_amd_gpu_count(kfd_root)
    if ngpu:
        res[constants.CLOUDTIK_GPU_RESOURCE] = float(ngpu)
        acc = detect_accelerator_type(kfd_root)
        if acc:
            res[constants.CLOUDTIK_ACCELERATOR_TYPE_PREFIX + acc] = float(ngpu)
    env = os.environ.get(constants.CLOUDTIK_RESOURCES_ENV)
    if env:
        import json
        res.update({k: float(v) for k, v in json.loads(env).items()})
    if override:
        res.update(override)
    return res


def parse_memory(value) -> int:
    """'16g' / '512Mi' / 1024 -> bytes (reference core_utils memory parsing)."""
    if isinstance(value, (int, float)):
        return int(value)
    s = str(value).strip().lower()
    units = {"k": 1 << 10, "ki": 1 << 10, "kb": 1000, "m": 1 << 20, "mi": 1 << 20, "mb": 10 ** 6,
             "g": 1 << 30, "gi": 1 << 30, "gb": 10 ** 9, "t": 1 << 40, "ti": 1 << 40, "tb": 10 ** 12,
             "b": 1}
    for u in sorted(units, key=len, reverse=True):
        if s.endswith(u):
            return int(float(s[: -len(u)]) * units[u])
    return int(float(s))
