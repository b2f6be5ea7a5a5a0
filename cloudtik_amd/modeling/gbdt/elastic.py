"""Elastic / fault-tolerant distributed GBDT training.

The reference trains XGBoost through xgboost_ray with ``RayParams`` (num_actors,
elastic_training, max_failed_actors, max_actor_restarts, checkpoint_frequency; reference
classical_ml/.../xgboost/modeling/run.py:90-106): actors that die are restarted, and with
elastic training the job goes on with the surviving actors instead of failing.

Here an actor is one process (one GPU each when training on GPUs) in a ``torch.distributed``
group (gloo on CPU, RCCL on GPUs) that trains on its row shard, the per-level histograms being
all-reduced (booster.py).  The driver (``train_elastic``):

* launches every live actor with a fresh rendezvous (127.0.0.1, a new port per attempt);
* rank 0 writes a checkpoint -- the whole model, which includes the rounds done -- every
  ``checkpoint_frequency`` rounds, atomically (temp file + rename);
* watches the processes; the first actor that exits non-zero (or the attempt running past
  ``attempt_timeout_s``) ends the attempt: the others are terminated (the exact processes
  it started);
* a failed actor with restarts left is restarted; one without restarts is dropped if
  ``elastic_training`` and at most ``max_failed_actors`` actors are gone, otherwise training
  fails;
* the next attempt resumes from the latest checkpoint with the live actors.  The data of a
  dropped actor is not used from then on (the xgboost_ray elastic semantics); the booster
  re-seeds its row / feature sampling from the global round index, so a resumed run with the
  same actors reproduces an uninterrupted one exactly.

``shard_fn(actor_id, num_actors)`` builds an actor's ``DMatrix`` inside the actor process and
must be picklable (a module-level function).  ``fail_at`` = {actor_id: round} makes that actor
exit abruptly after finishing the round, on the first attempt only (fault injection for tests).
"""
from __future__ import annotations

import json
import os
import socket
import tempfile
import time
from dataclasses import dataclass, field
from datetime import timedelta
from typing import Any, Callable, Dict, List, Optional

import torch.multiprocessing as mp


@dataclass
class ElasticParams:
    num_actors: int = 2
    elastic_training: bool = False
    max_failed_actors: int = 0
    max_actor_restarts: int = 0
    checkpoint_frequency: int = 5
    checkpoint_dir: Optional[str] = None
    device: str = "cpu"                  # "cuda": actor rank r uses cuda:(r % device_count)
    attempt_timeout_s: float = 3600.0
    collective_timeout_s: float = 120.0
    fail_at: Dict[int, int] = field(default_factory=dict)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _latest_checkpoint(d: str) -> Optional[str]:
    p = os.path.join(d, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        name = f.read().strip()
    path = os.path.join(d, name)
    return path if os.path.exists(path) else None


def _write_checkpoint(booster, d: str, rounds_done: int) -> str:
    name = f"checkpoint-{rounds_done:06d}.json"
    tmp = os.path.join(d, f".{name}.tmp")
    booster.save_model(tmp)
    os.replace(tmp, os.path.join(d, name))
    ptr = os.path.join(d, ".latest.tmp")
    with open(ptr, "w") as f:
        f.write(name)
    os.replace(ptr, os.path.join(d, "latest"))
    return name


def _actor_main(actor_id: int, rank: int, world: int, port: int, attempt: int, num_actors: int,
                shard_fn: Callable, params: Dict[str, Any], rounds: int, ep: ElasticParams, ckpt_dir: str,
                out_path: str):
    import torch
    import torch.distributed as dist
    from cloudtik_amd.modeling.gbdt.booster import Booster
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if ep.device.startswith("cuda"):
        torch.cuda.set_device(rank % torch.cuda.device_count())
        device = f"cuda:{rank % torch.cuda.device_count()}"
        backend = "nccl"
    else:
        device, backend = "cpu", "gloo"
    dist.init_process_group(backend, rank=rank, world_size=world,
                            timeout=timedelta(seconds=ep.collective_timeout_s))
    try:
        dm = shard_fn(actor_id, num_actors)
        ck = _latest_checkpoint(ckpt_dir)
        booster = Booster.load_model(ck, device=device) if ck else Booster(params, device=device)
        K = booster.objective.n_outputs
        done = booster.num_trees // K
        fail_round = ep.fail_at.get(actor_id) if attempt == 0 else None

        def on_round(rnd, _scores):
            if fail_round is not None and rnd == fail_round:
                os._exit(17)                       # abrupt death: no cleanup, peers see a dead socket

        freq = max(1, int(ep.checkpoint_frequency))
        while done < rounds:
            n = min(freq - done % freq, rounds - done)
            booster.train(dm, n, callback=on_round)
            done += n
            if rank == 0 and done < rounds:
                _write_checkpoint(booster, ckpt_dir, done)
            dist.barrier()                           # nobody runs ahead of a checkpoint being written
        if rank == 0:
            booster.save_model(out_path)
    finally:
        dist.destroy_process_group()


def train_elastic(params: Dict[str, Any], shard_fn: Callable[[int, int], Any], num_boost_round: int,
                  ep: ElasticParams, log: Callable[[str], None] = lambda m: None):
    """Train with fault tolerance; returns (Booster, report).  ``report`` has the attempts
    (live actors, failed actors, rounds resumed from) and the final actor set."""
    from cloudtik_amd.modeling.gbdt.booster import Booster
    own_dir = ep.checkpoint_dir is None
    ckpt_dir = ep.checkpoint_dir or tempfile.mkdtemp(prefix="gbdt-elastic-")
    os.makedirs(ckpt_dir, exist_ok=True)
    out_path = os.path.join(ckpt_dir, "final-model.json")
    if os.path.exists(out_path):
        os.remove(out_path)
    ctx = mp.get_context("spawn")
    alive: List[int] = list(range(ep.num_actors))
    restarts = {a: ep.max_actor_restarts for a in alive}
    dropped: List[int] = []
    attempts: List[Dict[str, Any]] = []
    attempt = 0
    while True:
        ck = _latest_checkpoint(ckpt_dir)
        resumed = 0
        if ck:
            with open(ck) as f:
                doc = json.load(f)
            resumed = len((doc.get("trees") or {}).get("feat", []))
        port = _free_port()
        procs = {}
        for rank, a in enumerate(alive):
            p = ctx.Process(target=_actor_main, args=(a, rank, len(alive), port, attempt, ep.num_actors, shard_fn,
                                                      params, num_boost_round, ep, ckpt_dir, out_path),
                            daemon=True)
            p.start()
            procs[a] = p
        log(f"attempt {attempt}: actors {alive}, resuming with {resumed} trees")
        failed: List[int] = []
        deadline = time.time() + ep.attempt_timeout_s
        while True:
            codes = {a: p.exitcode for a, p in procs.items()}
            failed = [a for a, c in codes.items() if c not in (None, 0)]
            if failed or all(c == 0 for c in codes.values()):
                break
            if time.time() > deadline:
                failed = [a for a, c in codes.items() if c is None]
                break
            time.sleep(0.05)
        if failed:
            # take the rest of the group down: they are blocked in (or heading for) a collective
            # with a dead peer
            for a, p in procs.items():
                if p.is_alive():
                    p.terminate()
            for p in procs.values():
                p.join(10)
                if p.is_alive():
                    p.kill()
                    p.join(5)
        attempts.append({"actors": list(alive), "failed": list(failed), "resumed_trees": resumed})
        if not failed:
            break
        for a in failed:
            if restarts[a] > 0:
                restarts[a] -= 1
                log(f"actor {a} failed: restarting ({restarts[a]} restarts left)")
            else:
                alive.remove(a)
                dropped.append(a)
                log(f"actor {a} failed with no restarts left")
        if dropped and not ep.elastic_training:
            raise RuntimeError(f"actors {dropped} failed and elastic_training is off")
        if len(dropped) > ep.max_failed_actors or not alive:
            raise RuntimeError(f"{len(dropped)} actors lost (max_failed_actors={ep.max_failed_actors})")
        attempt += 1
    booster = Booster.load_model(out_path, device="cpu" if not ep.device.startswith("cuda") else None)
    report = {"attempts": attempts, "final_actors": list(alive), "dropped_actors": dropped,
              "checkpoint_dir": None if own_dir else ckpt_dir}
    if own_dir:
        import shutil
        shutil.rmtree(ckpt_dir, ignore_errors=True)
    return booster, report
