"""Measured collective tuning for one node: the gradient-bucket size and the one-shot P2P
all-reduce crossover that ``bench/comm_bench.py --write-tuning`` measured at a given world
size, read back by the data-parallel path (``bench.py --bucket-mb auto``,
``parallel/p2p.from_env``).

Nothing here is assumed: an entry exists only for a world size that was measured on a node,
and without one the callers keep their built-in defaults (64 MiB BERT / 8 MiB ResNet buckets,
P2P off).  The P2P path is switched on by a measured crossover only when it was measured with
at least 2 ranks (the kernel's whole point is reading the xGMI peers at once; a 1-rank
measurement says nothing about that).

File: ``CLOUDTIK_COMM_TUNING`` or ``cloudtik_amd/parallel/comm_tuning.json``:
``{"<world>": {"bucket_bytes": int, "p2p_crossover_bytes": int|null, "rccl": str,
"gpu": str, "measured": "<iso time>"}}``.
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, Optional

MiB = 1 << 20
DEFAULT_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "comm_tuning.json")


def path() -> str:
    return os.environ.get("CLOUDTIK_COMM_TUNING") or DEFAULT_PATH


def load_all(p: Optional[str] = None) -> Dict[str, Any]:
    try:
        with open(p or path()) as f:
            d = json.load(f)
        return d if isinstance(d, dict) else {}
    except (OSError, ValueError):
        return {}


def entry(world: int, p: Optional[str] = None) -> Optional[Dict[str, Any]]:
    return load_all(p).get(str(int(world)))


def record(world: int, bucket_bytes: Optional[int], p2p_crossover_bytes: Optional[int],
           p: Optional[str] = None, **extra) -> Dict[str, Any]:
    """Store the measurement of one world size (other sizes' entries are kept)."""
    target = p or path()
    d = load_all(target)
    d[str(int(world))] = dict({"bucket_bytes": bucket_bytes, "p2p_crossover_bytes": p2p_crossover_bytes,
                               "measured": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}, **extra)
    tmp = target + ".tmp"
    with open(tmp, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    os.replace(tmp, target)
    return d


def bucket_mb(world: int, default: float, lo: float = 4.0, hi: float = 256.0) -> float:
    """The measured bucket size for ``world`` ranks in MiB (clamped to [lo, hi]), or
    ``default`` when this world size was never measured."""
    e = entry(world)
    b = (e or {}).get("bucket_bytes")
    if not b:
        return default
    return float(min(hi, max(lo, b / MiB)))


def p2p_bytes(world: int) -> int:
    """Measured crossover below which the one-shot P2P all-reduce beats RCCL, for >= 2 ranks
    (0 = not measured / never faster: P2P stays off)."""
    if world < 2:
        return 0
    e = entry(world)
    return int((e or {}).get("p2p_crossover_bytes") or 0)
