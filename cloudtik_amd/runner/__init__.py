"""Distributed job runner (``cloudtik-run``) and the function-call API.

``run_command(cmd, nnodes=..., nproc_per_node=..., hosts=...)`` launches a command on every
rank exactly as ``cloudtik-run`` would (reference runtime/ai/runner/__init__.py:139-187) and
returns its exit code.  ``run(fn, args, num_proc=...)`` runs a Python function on every rank
of a local or multi-host job and returns the per-rank results (reference runtime/ai/runner/util/
func_call.py + run_func.py + codec.py: the function is serialized with cloudpickle,
each rank executes it under the launcher's env:// rank environment and writes its result
back).  Only files this process wrote are deserialized.
"""
from __future__ import annotations

import argparse
import os
import shutil
import sys
import tempfile
from typing import Any, Callable, List, Optional

from cloudtik_amd.runner.distributor import Distributor


def run_command(command, num_proc: int = 0, nnodes: int = 0, nproc_per_node: int = 0, hosts: Optional[str] = None,
                hostfile: Optional[str] = None, launcher: Optional[str] = None, master_addr: Optional[str] = None,
                master_port: int = 29500, module: bool = False, no_python: bool = False,
                max_restarts: int = 0, env: Optional[dict] = None, extra_args: Optional[List[str]] = None) -> int:
    """Run ``command`` (a script / module and its arguments, list or string) on every rank;
    same launcher selection, rank environment and restarts as the ``cloudtik-run`` CLI."""
    import shlex
    from cloudtik_amd.runner.launch import main as launch_main
    cmd = shlex.split(command) if isinstance(command, str) else [str(c) for c in command]
    if not cmd:
        raise ValueError("empty command")
    argv = ["--num-proc", str(num_proc), "--nnodes", str(nnodes), "--nproc-per-node", str(nproc_per_node),
            "--master-port", str(master_port), "--max-restarts", str(max_restarts)]
    if hosts:
        argv += ["--hosts", hosts]
    if hostfile:
        argv += ["--hostfile", hostfile]
    if launcher:
        argv += ["--launcher", launcher]
    if master_addr:
        argv += ["--master-addr", master_addr]
    if module:
        argv.append("-m")
    if no_python:
        argv.append("--no-python")
    argv += list(extra_args or [])
    old = dict(os.environ)
    os.environ.update({k: str(v) for k, v in (env or {}).items()})
    try:
        return launch_main(argv + cmd)
    finally:
        os.environ.clear()
        os.environ.update(old)


def run(fn: Callable, args: tuple = (), kwargs: Optional[dict] = None, num_proc: int = 0,
        nproc_per_node: int = 0, hosts: Optional[str] = None, master_port: int = 29500,
        bind_cpus: bool = True, env: Optional[dict] = None) -> List[Any]:
    import cloudpickle
    from cloudtik_amd.runner.launch import build_parser
    from cloudtik_amd.runner.launchers import create_launcher
    work = tempfile.mkdtemp(prefix="cloudtik-run-func-")
    try:
        with open(os.path.join(work, "func.pkl"), "wb") as f:
            cloudpickle.dump((fn, args, kwargs or {}), f)
        argv = ["--num-proc", str(num_proc), "--nproc-per-node", str(nproc_per_node),
                "--master-port", str(master_port), "-m"]
        if hosts:
            argv += ["--hosts", hosts]
        if not bind_cpus:
            argv.append("--no-bind-cpus")
        argv += ["cloudtik_amd.runner.run_func", work]
        a = build_parser().parse_args(argv)
        d = Distributor(a.num_proc, a.nnodes, a.nproc_per_node, a.hosts or None, None)
        a.launcher = "distributed" if d.nnodes > 1 else "local"
        old = dict(os.environ)
        os.environ.update(env or {})
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        os.environ["PYTHONPATH"] = root + (os.pathsep + old["PYTHONPATH"] if old.get("PYTHONPATH") else "")
        try:
            rc = create_launcher(a.launcher, a, d).run()
        finally:
            os.environ.clear()
            os.environ.update(old)
        if rc != 0:
            raise RuntimeError(f"distributed function failed with exit code {rc}")
        out = []
        for r in range(d.num_proc):
            with open(os.path.join(work, f"result_{r}.pkl"), "rb") as f:
                out.append(cloudpickle.load(f))
        return out
    finally:
        shutil.rmtree(work, ignore_errors=True)
