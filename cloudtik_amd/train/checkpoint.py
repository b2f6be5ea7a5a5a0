"""Checkpoint / resume (reference: the transfer-learning models' checkpoint saving and
BERT's (commented-out) resume path, SURVEY.md §5 "checkpoint/resume").

* one directory per step: ``<dir>/step-<N>/`` with ``model.pt`` (rank 0), ``optim.pt`` (rank 0:
  the flat fp32 master + moments in the global layout -- ZeRO-1 shards are gathered -- which
  restores at any world size) or ``optim-rank<R>.pt`` (per-rank shard-layout state),
  ``meta.json`` (step, epoch, world size, user metadata) and ``rng-rank<R>.pt``;
* writes go to ``step-<N>.tmp`` and are renamed only after every rank finished (barrier),
  so a crash never leaves a half-written "latest" checkpoint;
* ``load_latest`` restores model, optimizer, scheduler and RNG (torch CPU/GPU + the
  dropout hash stream of cloudtik_amd.ops) and returns the metadata;
* only tensors / numbers / strings are stored, loaded with ``weights_only=True``;
* ``save_async``: the device state is copied into reused pinned host buffers on a side HIP
  stream (the compute stream waits on that copy only, not on the host), and a writer thread
  serialises the files.  Completion is agreed through per-rank marker files instead of a
  collective, so no collective ever runs off the main thread; rank 0 commits (meta.json +
  rename) once every rank's marker is present.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import threading
import time
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
            osd = optimizer.state_dict()          # collective under ZeRO-1: every rank calls it
            name = _optim_file(osd, rank)
            if name is not None:
                torch.save(_to_cpu(osd), os.path.join(tmp, name))
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

    # ------------------------------------------------------------------ async save
    def _pinned_copy(self, obj, stream, key=""):
        if isinstance(obj, torch.Tensor):
            t = obj.detach()
            if t.device.type != "cuda":
                return t.clone()
            buf = self._pinned.get(key)
            if buf is None or buf.shape != t.shape or buf.dtype != t.dtype:
                buf = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                self._pinned[key] = buf
            with torch.cuda.stream(stream):
                buf.copy_(t, non_blocking=True)
            return buf
        if isinstance(obj, dict):
            return {k: self._pinned_copy(v, stream, f"{key}/{k}") for k, v in obj.items()}
        if isinstance(obj, (list, tuple)):
            return type(obj)(self._pinned_copy(v, stream, f"{key}/{i}") for i, v in enumerate(obj))
        return obj

    def save_async(self, step: int, model: torch.nn.Module, optimizer=None, scheduler=None, epoch: int = 0,
                   extra: Optional[Dict[str, Any]] = None, timeout: float = 1800.0) -> "PendingSave":
        prev = getattr(self, "_inflight", None)
        if prev is not None:
            prev.wait()                         # pinned buffers are reused: one save in flight
        if not hasattr(self, "_pinned"):
            self._pinned = {}
        rank, world = _rank_world()
        final = os.path.join(self.dir, f"step-{step}")
        tmp = final + ".tmp"
        if rank == 0:
            shutil.rmtree(tmp, ignore_errors=True)
            os.makedirs(tmp, exist_ok=True)
        _barrier()
        event = None
        cuda = torch.cuda.is_available() and torch.cuda.is_initialized()
        stream = None
        if cuda:
            stream = torch.cuda.Stream()
            stream.wait_stream(torch.cuda.current_stream())
        osd = optimizer.state_dict() if optimizer is not None else None   # collective under ZeRO-1
        if osd is not None and _optim_file(osd, rank) is None:
            osd = None                          # rank 0 writes the global-layout state
        snap = {"model": model.state_dict() if rank == 0 else None, "optim": osd}
        if stream is not None:
            snap = self._pinned_copy(snap, stream, "s")
            event = torch.cuda.Event()
            event.record(stream)
            # later optimizer steps must not overwrite the tensors while they are copied
            torch.cuda.current_stream().wait_event(event)
        else:
            snap = self._pinned_copy(snap, None, "s")
        sched = scheduler.state_dict() if (rank == 0 and scheduler is not None
                                           and hasattr(scheduler, "state_dict")) else None
        rng = _rng_state()
        meta = {"step": step, "epoch": epoch, "world_size": world, "extra": extra or {}}
        pending = PendingSave(final)

        def write():
            try:
                if event is not None:
                    event.synchronize()
                if rank == 0:
                    torch.save(snap["model"], os.path.join(tmp, "model.pt"))
                    if sched is not None:
                        torch.save(sched, os.path.join(tmp, "scheduler.pt"))
                if snap["optim"] is not None:
                    name = _optim_file(snap["optim"], rank)
                    if name is not None:
                        torch.save(snap["optim"], os.path.join(tmp, name))
                torch.save(rng, os.path.join(tmp, f"rng-rank{rank}.pt"))
                open(os.path.join(tmp, f"done-rank{rank}"), "w").close()
                if rank == 0:
                    deadline = time.time() + timeout
                    while not all(os.path.exists(os.path.join(tmp, f"done-rank{r}")) for r in range(world)):
                        if time.time() > deadline:
                            raise TimeoutError(f"ranks did not finish checkpoint {final}")
                        time.sleep(0.05)
                    for r in range(world):
                        os.remove(os.path.join(tmp, f"done-rank{r}"))
                    with open(os.path.join(tmp, "meta.json"), "w") as f:
                        json.dump(meta, f)
                    if os.path.exists(final):
                        shutil.rmtree(final)
                    os.replace(tmp, final)
                    for old in self.steps()[:-self.keep] if self.keep else []:
                        shutil.rmtree(os.path.join(self.dir, f"step-{old}"), ignore_errors=True)
            except BaseException as e:  # noqa: BLE001 - surfaced by wait()
                pending.error = e
            finally:
                pending.done.set()

        pending.thread = threading.Thread(target=write, name=f"ckpt-{step}", daemon=True)
        pending.thread.start()
        self._inflight = pending
        return pending

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
            p = os.path.join(d, "optim.pt")          # global layout: one file for any world size
            if not os.path.exists(p):
                p = os.path.join(d, f"optim-rank{rank}.pt")
                if meta["world_size"] != world:
                    raise RuntimeError(f"checkpoint written by {meta['world_size']} ranks holds per-rank "
                                       f"(shard-layout) optimizer state; it cannot resume at {world} ranks")
                if not os.path.exists(p):
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


class PendingSave:
    """Handle of an in-flight ``save_async``; ``wait()`` re-raises a writer error.  On
    rank != 0 it completes when this rank's files are written (rank 0 commits)."""

    def __init__(self, path: str):
        self.path = path
        self.done = threading.Event()
        self.error: Optional[BaseException] = None
        self.thread: Optional[threading.Thread] = None

    def wait(self, timeout: Optional[float] = None) -> str:
        self.done.wait(timeout)
        if self.error is not None:
            raise self.error
        return self.path


def _optim_file(osd, rank: int) -> Optional[str]:
    """File name of this rank's optimizer state, or None when another rank writes it: a
    global-layout flat state (identical on every rank) is written once, by rank 0."""
    if isinstance(osd, dict) and osd.get("flat_layout") == "global":
        return "optim.pt" if rank == 0 else None
    return f"optim-rank{rank}.pt"


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
