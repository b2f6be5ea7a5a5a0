"""Node resource metrics for heartbeats and ``cloudtik resource-metrics`` (reference
core/_private/node/node_monitor.py + resource_spec.py, which sample psutil and NVIDIA GPUs
through GPUtil).  AMD GPUs are sampled from the amdgpu sysfs files of each card
(``gpu_busy_percent``, ``mem_info_vram_used/total``, hwmon temperature / power), which
cost microseconds and need no SMI library; ``amdsmi`` is used when importable for fields
sysfs lacks.

GPU health (SURVEY.md §5.3 "GPU health to NodeMonitor"): the amdgpu RAS counters under
``device/ras/*_err_count`` ("ue: N" uncorrectable / "ce: M" correctable per IP block:
umc = HBM, xgmi_wafl = xGMI links, gfx, sdma, mmhub, ...) and the edge/junction temperature
against ``CLOUDTIK_GPU_HEALTH_TEMP_C`` give each GPU ``healthy`` + ``health_issues``; the
node row carries ``gpu_healthy`` and the head's scaler recovers a node whose GPUs stay
unhealthy (core/head/scaler.py).
"""
from __future__ import annotations

import glob
import os
import time
from typing import Any, Dict, List, Optional

import psutil

DRM_ROOT = "/sys/class/drm"
AMD_VENDOR = "0x1002"


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _read_int(path: str) -> Optional[int]:
    v = _read(path)
    try:
        return int(v) if v is not None else None
    except ValueError:
        return None


def amd_gpu_cards(root: str = DRM_ROOT) -> List[str]:
    out = []
    for card in sorted(glob.glob(os.path.join(root, "card[0-9]*")), key=lambda p: int(p.rsplit("card", 1)[1])
                       if p.rsplit("card", 1)[1].isdigit() else 1 << 30):
        if not os.path.basename(card)[4:].isdigit():
            continue
        if _read(os.path.join(card, "device", "vendor")) == AMD_VENDOR and \
                os.path.exists(os.path.join(card, "device", "mem_info_vram_total")):
            out.append(card)
    return out


def ras_counts(dev: str) -> Dict[str, Dict[str, int]]:
    """{block: {"ue": n, "ce": m}} from ``<dev>/ras/<block>_err_count``."""
    out: Dict[str, Dict[str, int]] = {}
    for f in sorted(glob.glob(os.path.join(dev, "ras", "*_err_count"))):
        block = os.path.basename(f)[:-len("_err_count")]
        txt = _read(f) or ""
        cnt: Dict[str, int] = {}
        for line in txt.splitlines():
            k, _, v = line.partition(":")
            try:
                cnt[k.strip()] = int(v.strip())
            except ValueError:
                continue
        if cnt:
            out[block] = cnt
    return out


def gpu_health(g: Dict[str, Any], temp_limit_c: Optional[float] = None) -> List[str]:
    """Reasons this GPU is unhealthy (empty list = healthy)."""
    from cloudtik_amd.core import constants as C
    limit = C.CLOUDTIK_GPU_HEALTH_TEMP_C if temp_limit_c is None else temp_limit_c
    issues = []
    for block, cnt in (g.get("ras") or {}).items():
        if cnt.get("ue", 0) > 0:
            issues.append(f"{block}: {cnt['ue']} uncorrectable error(s)")
    t = g.get("temperature_c")
    if t is not None and t >= limit:
        issues.append(f"temperature {t:.0f}C >= {limit}C")
    if g.get("vram_total") in (None, 0):
        issues.append("VRAM not reported (device lost?)")
    return issues


def gpu_metrics(root: str = DRM_ROOT) -> List[Dict[str, Any]]:
    gpus = []
    for i, card in enumerate(amd_gpu_cards(root)):
        dev = os.path.join(card, "device")
        g: Dict[str, Any] = {
            "index": i,
            "card": os.path.basename(card),
            "busy_percent": _read_int(os.path.join(dev, "gpu_busy_percent")),
            "vram_used": _read_int(os.path.join(dev, "mem_info_vram_used")),
            "vram_total": _read_int(os.path.join(dev, "mem_info_vram_total")),
            "pci": os.path.basename(os.path.realpath(dev)),
        }
        hw = sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*")))
        if hw:
            t = _read_int(os.path.join(hw[0], "temp1_input"))
            pw = _read_int(os.path.join(hw[0], "power1_average")) or _read_int(os.path.join(hw[0], "power1_input"))
            g["temperature_c"] = t / 1000.0 if t is not None else None
            g["power_w"] = pw / 1e6 if pw is not None else None
            # the hottest sensor (junction / HBM) when the driver exposes several
            temps = [_read_int(p) for p in glob.glob(os.path.join(hw[0], "temp*_input"))]
            temps = [v for v in temps if v is not None]
            if temps:
                g["temperature_max_c"] = max(temps) / 1000.0
        g["ras"] = ras_counts(dev)
        g["health_issues"] = gpu_health(dict(g, temperature_c=g.get("temperature_max_c", g.get("temperature_c"))))
        g["healthy"] = not g["health_issues"]
        gpus.append(g)
    return gpus


def _dpm_current_mhz(path: str) -> Optional[int]:
    """The active level of an amdgpu ``pp_dpm_*`` table ("1: 2100Mhz *")."""
    for line in (_read(path) or "").splitlines():
        if line.rstrip().endswith("*"):
            tok = line.split(":", 1)[-1].strip().split()[0].lower()
            try:
                return int(float(tok.replace("mhz", "")))
            except ValueError:
                return None
    return None


def pci_device_dir(domain: int, bus: int, device: int, root: str = DRM_ROOT) -> Optional[str]:
    """sysfs directory of the GPU at PCI ``domain:bus:device.0``
    (``torch.cuda.get_device_properties`` gives the three numbers), or None.  Looked up
    through the amdgpu DRM cards (a container may not expose /sys/bus/pci); when exactly
    one AMD card is visible and nothing matches, that card."""
    want = f"{bus:02x}:{device:02x}.0"
    d = f"/sys/bus/pci/devices/{domain:04x}:{want}"
    if os.path.isdir(d):
        return d
    cards = amd_gpu_cards(root)
    for card in cards:
        dev = os.path.realpath(os.path.join(card, "device"))
        if os.path.basename(dev).endswith(want):
            return dev
    if len(cards) == 1:
        return os.path.realpath(os.path.join(cards[0], "device"))
    return None


def gpu_clock_snapshot(dev: Optional[str] = None, root: str = DRM_ROOT) -> Dict[str, Any]:
    """Clock / power / temperature of one GPU right now, from amdgpu sysfs: the state that
    decides an MFMA-bound benchmark's speed on a given box (the chip lowers its clock under
    load; MI355X_MICROARCH.md 'DVFS give-back').  ``dev`` is the PCI device directory (default:
    the first AMD card).  Keys absent when the driver does not expose them."""
    if dev is None:
        cards = amd_gpu_cards(root)
        if not cards:
            return {}
        dev = os.path.realpath(os.path.join(cards[0], "device"))
    out: Dict[str, Any] = {"pci": os.path.basename(os.path.realpath(dev))}
    s = _dpm_current_mhz(os.path.join(dev, "pp_dpm_sclk"))
    m = _dpm_current_mhz(os.path.join(dev, "pp_dpm_mclk"))
    if s is not None:
        out["sclk_mhz"] = s
    if m is not None:
        out["mclk_mhz"] = m
    hw = sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*")))
    if hw:
        h = hw[0]
        pw = _read_int(os.path.join(h, "power1_average")) or _read_int(os.path.join(h, "power1_input"))
        if pw is not None:
            out["power_w"] = round(pw / 1e6, 1)
        cap = _read_int(os.path.join(h, "power1_cap"))
        if cap:
            out["power_cap_w"] = round(cap / 1e6, 1)
        for f in sorted(glob.glob(os.path.join(h, "freq*_input"))):
            lab = (_read(f.replace("_input", "_label")) or os.path.basename(f)[:-6]).lower()
            v = _read_int(f)
            if v is not None:
                out[f"{lab}_mhz"] = int(v / 1e6)
        for f in sorted(glob.glob(os.path.join(h, "temp*_input"))):
            lab = (_read(f.replace("_input", "_label")) or os.path.basename(f)[:-6]).lower()
            v = _read_int(f)
            if v is not None:
                out[f"temp_{lab}_c"] = v / 1000.0
    return out


class NodeMetricsCollector:
    def __init__(self, drm_root: str = DRM_ROOT):
        self.drm_root = drm_root
        self._last_net = None
        psutil.cpu_percent(interval=None)

    def collect(self) -> Dict[str, Any]:
        vm = psutil.virtual_memory()
        now = time.time()
        net = psutil.net_io_counters()
        rx_rate = tx_rate = 0.0
        if self._last_net is not None:
            dt = max(1e-3, now - self._last_net[0])
            rx_rate = (net.bytes_recv - self._last_net[1]) / dt
            tx_rate = (net.bytes_sent - self._last_net[2]) / dt
        self._last_net = (now, net.bytes_recv, net.bytes_sent)
        try:
            load = os.getloadavg()
        except OSError:
            load = (0.0, 0.0, 0.0)
        disk = psutil.disk_usage(os.path.expanduser("~"))
        gpus = gpu_metrics(self.drm_root)
        return {
            "time": now,
            "cpu_count": psutil.cpu_count(),
            "cpu_percent": psutil.cpu_percent(interval=None),
            "load_avg": list(load),
            "memory_total": vm.total,
            "memory_used": vm.total - vm.available,
            "disk_total": disk.total,
            "disk_used": disk.used,
            "network_rx_bytes_per_s": rx_rate,
            "network_tx_bytes_per_s": tx_rate,
            "gpus": gpus,
            "gpu_busy_percent_avg": (sum(g["busy_percent"] or 0 for g in gpus) / len(gpus)) if gpus else None,
            "gpu_healthy": all(g["healthy"] for g in gpus),
            "gpu_health_issues": [f"gpu{g['index']}: {i}" for g in gpus for i in g["health_issues"]],
        }
