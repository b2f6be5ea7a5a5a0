"""Checkpoint / resume (reference: the transfer-learning models' checkpoint saving and
BERT's (commented-out) resume path, SURVEY.md §5 "checkpoint/resume").

* one directory per step: ``<dir>/step-<N>/`` with ``model.pt`` (rank 0), ``optim-rank<R>.pt``
  (every rank: flat fp32 master + moments, so ZeRO-style sharded optimizer state round-trips),
  ``meta.json`` (step, epoch, world size, user metadata) and ``rng-rank<R>.pt``;
* writes go to ``step-<N>.tmp`` and are renamed only after every rank finished (barrier),
  so a crash never leaves a half-written "latest" checkpoint;
* ``load_latest`` restores model, optimizer, scheduler and RNG (torch CPU/GPU + the
  dropout Philox stream of cloudtik_amd.ops) and returns the metadata;
* only tensors / numbers / strings are stored, loaded with ``weights_only=True``.
"""
from __future__ import annotations

import json
import os
import re
import shutil
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist


def _rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


class Checkpointer:
    def __init__(self, directory: str, keep: int = 3):
        self.dir = os.path.abspath(os.path.expanduser(directory))
        self.keep = keep
        os.makedirs(self.dir, exist_ok=True)

    # ------------------------------------------------------------------ listing
    def steps(self):
        out = []
        for name in os.listdir(self.dir):
            m = re.fullmatch(r"step-(\d+)", name)
            if m and os.path.exists(os.path.join(self.dir, name, "meta.json")):
                out.append(int(m.group(1)))
        return sorted(out)

    def latest_step(self) -> Optional[int]:
        s = self.steps()
        return s[-1] if s else None

    # ------------------------------------------------------------------ save
    def save(self, step: int, model: torch.nn.Module, optimizer=None, scheduler=None, epoch: int = 0,
             extra: Optional[Dict[str, Any]] = None) -> str:
        rank, world = _rank_world()
        final = os.path.join(self.dir, f"step-{step}")
        tmp = final + ".tmp"
        if rank == 0:
            shutil.rmtree(tmp, ignore_errors=True)
            os.makedirs(tmp, exist_ok=True)
        _barrier()
        if rank == 0:
            torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()}, os.path.join(tmp, "model.pt"))
            if scheduler is not None and hasattr(scheduler, "state_dict"):
                torch.save(scheduler.state_dict(), os.path.join(tmp, "scheduler.pt"))
        if optimizer is not None:
            torch.save(_to_cpu(optimizer.state_dict()), os.path.join(tmp, f"optim-rank{rank}.pt"))
        torch.save(_rng_state(), os.path.join(tmp, f"rng-rank{rank}.pt"))
        _barrier()
        if rank == 0:
            with open(os.path.join(tmp, "meta.json"), "w") as f:
                json.dump({"step": step, "epoch": epoch, "world_size": world, "extra": extra or {}}, f)
            if os.path.exists(final):
                shutil.rmtree(final)
            os.replace(tmp, final)
            for old in self.steps()[:-self.keep] if self.keep else []:
                shutil.rmtree(os.path.join(self.dir, f"step-{old}"), ignore_errors=True)
        _barrier()
        return final

    # ------------------------------------------------------------------ load
    def load(self, step: int, model: torch.nn.Module, optimizer=None, scheduler=None,
             map_location="cpu", strict: bool = True) -> Dict[str, Any]:
        rank, world = _rank_world()
        d = os.path.join(self.dir, f"step-{step}")
        with open(os.path.join(d, "meta.json")) as f:
            meta = json.load(f)
        sd = torch.load(os.path.join(d, "model.pt"), map_location=map_location, weights_only=True)
        model.load_state_dict(sd, strict=strict)
        if optimizer is not None:
            p = os.path.join(d, f"optim-rank{rank}.pt")
            if not os.path.exists(p):
                if meta["world_size"] != world:
                    raise RuntimeError(f"checkpoint written by {meta['world_size']} ranks; resuming with {world} "
                                       "needs an unsharded optimizer state")
                raise FileNotFoundError(p)
            optimizer.load_state_dict(torch.load(p, map_location=map_location, weights_only=True))
        if scheduler is not None and os.path.exists(os.path.join(d, "scheduler.pt")):
            scheduler.load_state_dict(torch.load(os.path.join(d, "scheduler.pt"), weights_only=True))
        rp = os.path.join(d, f"rng-rank{rank}.pt")
        if os.path.exists(rp):
            _set_rng_state(torch.load(rp, weights_only=True))
        return meta

    def load_latest(self, model, optimizer=None, scheduler=None, **kw) -> Optional[Dict[str, Any]]:
        s = self.latest_step()
        if s is None:
            return None
        return self.load(s, model, optimizer, scheduler, **kw)


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def _rng_state():
    st = {"torch": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state()
    try:
        from cloudtik_amd import ops
        r = ops.rng_state()
        st["ops_seed"] = int(r["seed"])
        st["ops_offset"] = int(r["offset"])
    except Exception:  # noqa: BLE001
        pass
    return st


def _set_rng_state(st):
    torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])
    if "ops_seed" in st:
        from cloudtik_amd import ops
        ops.set_rng_state({"seed": st["ops_seed"], "offset": st["ops_offset"]})
