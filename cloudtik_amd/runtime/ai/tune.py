"""Hyper-parameter trial parallelism (reference: Hyperopt ``SparkTrials`` in the AI examples,
examples/runtime/ai/basics/**/*hyperopt*; SURVEY.md §2.14 "Hyperparameter-trial
parallelism").

On an MI355X node the natural unit of trial parallelism is the GPU: ``tune`` runs up to
``max_concurrent`` trials at once (default: one per visible GPU), each in its own process
pinned to one GPU through ``HIP_VISIBLE_DEVICES``, and feeds finished results back into the
search (random search or TPE-style refinement around the best trials so far).

    def objective(params):                      # runs in a worker process on ONE GPU
        acc = train_and_eval(lr=params["lr"], width=params["width"])
        return {"loss": -acc}

    best = tune(objective, {"lr": loguniform(1e-4, 1e-1), "width": choice([128, 256, 512])},
                num_trials=32)

A trial that raises is recorded as failed and does not stop the search.
"""
from __future__ import annotations

import math
import multiprocessing as mp
import os
import random
import time
import traceback
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence


# ------------------------------------------------------------------------- search space
@dataclass
class uniform:
    low: float
    high: float

    def sample(self, rng, around=None, width=1.0):
        if around is not None:
            span = (self.high - self.low) * 0.25 * width
            return min(self.high, max(self.low, rng.gauss(around, span)))
        return rng.uniform(self.low, self.high)


@dataclass
class loguniform:
    low: float
    high: float

    def sample(self, rng, around=None, width=1.0):
        lo, hi = math.log(self.low), math.log(self.high)
        if around is not None:
            v = rng.gauss(math.log(around), (hi - lo) * 0.25 * width)
            return math.exp(min(hi, max(lo, v)))
        return math.exp(rng.uniform(lo, hi))


@dataclass
class choice:
    options: Sequence[Any]

    def sample(self, rng, around=None, width=1.0):
        if around is not None and rng.random() < 0.6:
            return around
        return rng.choice(list(self.options))


@dataclass
class Trial:
    tid: int
    params: Dict[str, Any]
    gpu: Optional[int] = None
    result: Optional[Dict[str, Any]] = None
    error: Optional[str] = None
    seconds: float = 0.0

    @property
    def loss(self) -> float:
        if self.result is None or "loss" not in self.result:
            return float("inf")
        return float(self.result["loss"])


@dataclass
class TuneResult:
    trials: List[Trial] = field(default_factory=list)

    @property
    def best(self) -> Trial:
        ok = [t for t in self.trials if t.error is None]
        if not ok:
            raise RuntimeError("every trial failed")
        return min(ok, key=lambda t: t.loss)


def _visible_gpus() -> List[int]:
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") \
        or os.environ.get("CUDA_VISIBLE_DEVICES")
    if env:
        return [int(x) for x in env.split(",") if x.strip()]
    try:
        from cloudtik_amd.core.node.metrics import amd_gpu_cards
        n = len(amd_gpu_cards())
    except Exception:  # noqa: BLE001
        n = 0
    return list(range(n))


def _worker(fn, params, gpu, q, tid):
    if gpu is not None:
        os.environ["HIP_VISIBLE_DEVICES"] = str(gpu)
    t0 = time.time()
    try:
        res = fn(params)
        if not isinstance(res, dict):
            res = {"loss": float(res)}
        q.put((tid, res, None, time.time() - t0))
    except Exception:  # noqa: BLE001
        q.put((tid, None, traceback.format_exc(), time.time() - t0))


def _propose(space, rng, history: List[Trial], n_startup: int):
    done = [t for t in history if t.error is None and t.result is not None]
    if len(done) < n_startup:
        return {k: d.sample(rng) for k, d in space.items()}
    # refine around one of the best quarter (TPE-flavoured exploitation with exploration)
    done.sort(key=lambda t: t.loss)
    elite = done[:max(1, len(done) // 4)]
    base = rng.choice(elite).params
    if rng.random() < 0.2:
        return {k: d.sample(rng) for k, d in space.items()}
    return {k: d.sample(rng, around=base[k], width=0.5) for k, d in space.items()}


def tune(fn: Callable[[Dict[str, Any]], Any], space: Dict[str, Any], num_trials: int = 16,
         max_concurrent: Optional[int] = None, seed: int = 0, n_startup: Optional[int] = None,
         timeout_s: Optional[float] = None) -> TuneResult:
    """Run ``num_trials`` trials of ``fn`` with up to ``max_concurrent`` at a time, one per GPU.

    ``fn`` must be picklable (module-level function).  Without GPUs trials run as CPU
    processes."""
    gpus = _visible_gpus()
    slots: List[Optional[int]] = list(gpus) if gpus else [None]
    if max_concurrent:
        slots = (slots * max_concurrent)[:max_concurrent] if gpus else [None] * max_concurrent
    rng = random.Random(seed)
    n_startup = n_startup if n_startup is not None else max(2, len(slots))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    res = TuneResult()
    running: Dict[int, Any] = {}
    free = list(range(len(slots)))
    slot_of: Dict[int, int] = {}
    deadline = time.time() + timeout_s if timeout_s else None
    next_tid = 0
    while next_tid < num_trials or running:
        while free and next_tid < num_trials:
            s = free.pop(0)
            t = Trial(next_tid, _propose(space, rng, res.trials, n_startup), slots[s])
            res.trials.append(t)
            p = ctx.Process(target=_worker, args=(fn, t.params, t.gpu, q, t.tid), daemon=True)
            p.start()
            running[t.tid], slot_of[t.tid] = p, s
            next_tid += 1
        try:
            tid, out, err, secs = q.get(timeout=1.0)
        except Exception:  # noqa: BLE001 - queue.Empty: check for dead workers / timeout
            for tid, p in list(running.items()):
                if not p.is_alive() and p.exitcode not in (0, None):
                    t = res.trials[tid]
                    t.error = f"worker exited with code {p.exitcode}"
                    running.pop(tid)
                    free.append(slot_of.pop(tid))
            if deadline and time.time() > deadline:
                for p in running.values():
                    p.terminate()
                for tid in list(running):
                    res.trials[tid].error = "timeout"
                break
            continue
        t = res.trials[tid]
        t.result, t.error, t.seconds = out, err, secs
        p = running.pop(tid, None)
        if p is not None:
            p.join(5)
        free.append(slot_of.pop(tid))
    return res
