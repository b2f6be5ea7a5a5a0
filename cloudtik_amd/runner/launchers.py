"""Process launchers behind ``cloudtik-run`` (reference runtime/ai/runner/launcher.py,
cpu/local_launcher.py, cpu/distributed_launcher.py, rsh/rsh_launcher.py,
mpi/mpi_launcher.py, horovod/horovod_launcher.py).

* ``local``       -- N ranks on this node, one per GPU: ``RANK / LOCAL_RANK / WORLD_SIZE /
  LOCAL_WORLD_SIZE / NODE_RANK / MASTER_ADDR / MASTER_PORT`` (the ``torch.distributed``
  env:// contract), each rank pinned to the cores of its GPU's NUMA node and given
  ``OMP_NUM_THREADS`` = its core count.  If any rank fails the others are terminated
  (exactly the process groups this launcher started) and its exit code is returned.
* ``distributed`` -- multi-node: runs the local launcher on every host (directly on this
  host, over ssh elsewhere) with its node rank; rank 0's host is the rendezvous master.
* ``rsh``         -- same as distributed with a configurable remote shell (``--rsh``).
* ``mpi``         -- ``mpirun -np N -H host:slots,...`` with the rank environment exported.
* ``horovod``     -- distributed, plus ``HOROVOD_*`` variables for Horovod-style scripts
  (served by cloudtik_amd.parallel.horovod on RCCL).
"""
from __future__ import annotations

import os
import shlex
import shutil
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

from cloudtik_amd.runner.affinity import rank_cpu_sets
from cloudtik_amd.runner.distributor import Distributor


def cloudtik_rsh_agent(rsh: Optional[str]) -> Optional[str]:
    """``--rsh cloudtik`` selects the ``cloudtik-rsh`` agent (remote commands through
    ``cloudtik head exec --node-ip``; reference runtime/ai/scripts/cloudtik-rsh.sh)."""
    if rsh in ("cloudtik", "cloudtik-rsh"):
        return shutil.which("cloudtik-rsh") or os.path.join(
            os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "bin", "cloudtik-rsh")
    return None


def _is_local(host: str) -> bool:
    if host in ("localhost", "127.0.0.1", socket.gethostname()):
        return True
    from cloudtik_amd.core.executor import local_ips
    return host in local_ips()


class Launcher:
    def __init__(self, args, distributor: Distributor):
        self.args = args
        self.d = distributor

    def program(self) -> List[str]:
        a = self.args
        prog = [a.program] + list(a.program_args)
        if a.no_python:
            return prog
        py = [sys.executable, "-u"]
        if a.module:
            return py + ["-m"] + prog
        return py + prog

    def base_env(self) -> Dict[str, str]:
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env["MASTER_ADDR"] = self.args.master_addr or "127.0.0.1"
        env["MASTER_PORT"] = str(self.args.master_port)
        env["WORLD_SIZE"] = str(self.d.num_proc)
        return env

    def run(self) -> int:
        raise NotImplementedError


class LocalLauncher(Launcher):
    """Spawns this node's ranks."""

    def __init__(self, args, distributor, node_rank: int = 0, first_rank: int = 0,
                 local_world: Optional[int] = None):
        super().__init__(args, distributor)
        self.node_rank = node_rank
        self.first_rank = first_rank
        self.local_world = local_world or min(distributor.nproc_per_node, distributor.num_proc)
        self.procs: List[subprocess.Popen] = []
        self._stopping = False

    def rank_env(self, local_rank: int, cpus: Optional[List[int]]) -> Dict[str, str]:
        env = self.base_env()
        env.update(RANK=str(self.first_rank + local_rank), LOCAL_RANK=str(local_rank),
                   LOCAL_WORLD_SIZE=str(self.local_world), NODE_RANK=str(self.node_rank),
                   GROUP_RANK=str(self.node_rank))
        if "OMP_NUM_THREADS" not in os.environ:
            # the rank's pinned cores, or a fair share of the node without GPU affinity
            share = len(cpus) if cpus else (os.cpu_count() or 1) // max(1, self.local_world)
            env["OMP_NUM_THREADS"] = str(max(1, share))
        if self.args.launcher == "horovod":
            env.update(HOROVOD_RANK=env["RANK"], HOROVOD_SIZE=env["WORLD_SIZE"],
                       HOROVOD_LOCAL_RANK=str(local_rank), HOROVOD_LOCAL_SIZE=str(self.local_world))
        return env

    def _terminate_all(self, sig=signal.SIGTERM):
        self._stopping = True
        for p in self.procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except (ProcessLookupError, PermissionError):
                    pass

    def rank_plan(self):
        """[(argv prefix, extra env, cpus)] per local rank: GPU ranks pinned to their GPU's
        NUMA-node cores."""
        cpu_sets = rank_cpu_sets(self.local_world) if self.args.bind_cpus else {}
        return [([], {}, cpu_sets.get(lr)) for lr in range(self.local_world)]

    def run(self) -> int:
        plan = self.rank_plan()
        prog = self.program()
        log_dir = self.args.log_dir
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)
        # if this launcher is killed outright, the reaper still ends the ranks (and frees GPUs)
        from cloudtik_amd.core.node.reaper import Reaper
        reaper = Reaper()
        for lr in range(self.local_world):
            prefix, extra_env, cpus = plan[lr]
            env = self.rank_env(lr, cpus)
            env.update(extra_env)
            argv = prefix + prog
            if getattr(self.args, "profile", ""):
                # rocprofv3 per rank; the program follows '--' directly (no shell/env hop)
                from cloudtik_amd.utils.profiling import rocprof_command
                argv = rocprof_command(prog, os.path.join(os.path.abspath(self.args.profile),
                                                          f"rank{self.first_rank + lr}"))
            out = None
            if log_dir:
                rank = self.first_rank + lr
                out = open(os.path.join(log_dir, f"{self.args.log_file_prefix}_{rank}.log"), "ab")

            def pre(c=None if prefix else cpus):
                if c:
                    try:
                        os.sched_setaffinity(0, c)
                    except OSError:
                        pass
            if self.args.verbose:
                print(f"[cloudtik-run] rank {env['RANK']} (local {lr}) cpus={cpus}: {' '.join(argv)}",
                      file=sys.stderr)
            self.procs.append(subprocess.Popen(argv, env=env, stdout=out, stderr=subprocess.STDOUT if out else None,
                                               preexec_fn=pre, start_new_session=True))
            reaper.watch(self.procs[-1].pid)          # the rank leads its own process group
        prev = {s: signal.getsignal(s) for s in (signal.SIGINT, signal.SIGTERM)}
        if threading.current_thread() is threading.main_thread():
            for s in prev:
                signal.signal(s, lambda *_: self._terminate_all())
        rc = 0
        try:
            alive = set(range(len(self.procs)))
            while alive:
                for i in list(alive):
                    r = self.procs[i].poll()
                    if r is None:
                        continue
                    alive.discard(i)
                    if r != 0 and rc == 0:
                        rc = r
                        if not self._stopping:
                            print(f"[cloudtik-run] rank {self.first_rank + i} exited with {r}: stopping the job",
                                  file=sys.stderr)
                            self._terminate_all()
                time.sleep(0.05)
        finally:
            if threading.current_thread() is threading.main_thread():
                for s, h in prev.items():
                    signal.signal(s, h)
            self._terminate_all(signal.SIGKILL)
            reaper.release()
        return rc if rc >= 0 else 128 - rc


class CpuLauncher(LocalLauncher):
    """CPU processes on this node placed by the core-pool scheduler (runner/cpu.py): per
    process a core list, a numactl / taskset prefix, OMP_NUM_THREADS and the allocator /
    OpenMP-runtime preloads (reference runtime/ai/runner/cpu/local_launcher.py:222-352)."""

    def rank_plan(self):
        from cloudtik_amd.runner.cpu import cpu_plan
        a = self.args
        if a.local_world:
            # a remote node launcher: its share of the job is fixed by the driver
            a.num_proc = a.local_world
        plan = cpu_plan(a)
        self.local_world = len(plan)
        if self.node_rank == 0 and self.first_rank == 0 and self.d.nnodes <= 1:
            self.d.num_proc = len(plan)
        if a.verbose:
            for i, (prefix, env, cpus) in enumerate(plan):
                print(f"[cloudtik-run] cpu process {i}: {' '.join(prefix) or '(affinity mask)'} "
                      f"OMP_NUM_THREADS={env.get('OMP_NUM_THREADS')} LD_PRELOAD={env.get('LD_PRELOAD', '')}",
                      file=sys.stderr)
        return [(prefix, env, cpus) for prefix, env, cpus in plan]


class DistributedLauncher(Launcher):
    """Runs the local launcher on every host of the job."""

    rsh_default = "ssh -o StrictHostKeyChecking=no -o UserKnownHostsFile=/dev/null"

    def remote_command(self, host: str, node_rank: int, local_world: int, first_rank: int) -> str:
        a = self.args
        local = "horovod-local" if a.launcher == "horovod" else ("cpu" if getattr(a, "cpu", False) else "local")
        parts = ["cloudtik-run", "--launcher", local,
                 "--node-rank", str(node_rank), "--first-rank", str(first_rank),
                 "--local-world", str(local_world), "--num-proc", str(self.d.num_proc),
                 "--nproc-per-node", str(self.d.nproc_per_node),
                 "--master-addr", a.master_addr, "--master-port", str(a.master_port)]
        if a.module:
            parts.append("-m")
        if a.no_python:
            parts.append("--no-python")
        if a.log_dir:
            parts += ["--log-dir", a.log_dir, "--log-file-prefix", a.log_file_prefix]
        if not a.bind_cpus:
            parts.append("--no-bind-cpus")
        if getattr(a, "profile", ""):
            parts += ["--profile", a.profile]
        if getattr(a, "cpu", False):
            from cloudtik_amd.runner.cpu import cpu_flags_argv
            parts += cpu_flags_argv(a)
        parts += [a.program] + list(a.program_args)
        keep = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_", "HSA_", "HIP_", "CLOUDTIK_",
                                                                       "TORCH_", "PYTHONPATH", "MIOPEN_"))}
        exports = " ".join(f"{k}={shlex.quote(v)}" for k, v in keep.items())
        return f"cd {shlex.quote(os.getcwd())} && env {exports} " + " ".join(shlex.quote(p) for p in parts)

    def run(self) -> int:
        """Start the local launcher on every host; the first host that fails stops the job
        everywhere (reference rsh/rsh_exec.py:196-263 terminate-all), so no rank is left
        blocked in an RCCL collective until the communicator timeout.

        Each remote launcher runs as the leader of its own process group (``setsid``) and
        writes its pid to a per-job file; terminate-all signals that whole group over the
        same remote shell, then ends the local ssh clients."""
        import uuid
        placements = self.d.host_ranks()
        if not self.args.master_addr:
            first = placements[0][0] if placements else "127.0.0.1"
            self.args.master_addr = "127.0.0.1" if _is_local(first) and len(placements) == 1 else first
        agent = cloudtik_rsh_agent(getattr(self.args, "rsh", None))
        rsh = [agent] if agent else shlex.split(getattr(self.args, "rsh", None) or self.rsh_default)
        job = uuid.uuid4().hex[:12]
        codes: Dict[str, int] = {}
        remote: Dict[str, subprocess.Popen] = {}
        locals_: Dict[str, LocalLauncher] = {}
        lock = threading.Lock()
        failed = threading.Event()

        def pidfile(node_rank):
            return f"/tmp/cloudtik-job-{job}-{node_rank}.pid"

        def run_host(host, node_rank, n, first):
            if _is_local(host):
                ll = LocalLauncher(self.args, self.d, node_rank, first, n)
                with lock:
                    locals_[host] = ll
                rc = ll.run()
            else:
                inner = self.remote_command(host, node_rank, n, first)
                wrapped = (f"setsid sh -c {shlex.quote(f'echo $$ > {pidfile(node_rank)}; exec sh -c {shlex.quote(inner)}')}"
                           f"; rc=$?; rm -f {pidfile(node_rank)}; exit $rc")
                p = subprocess.Popen(rsh + [host, wrapped])
                with lock:
                    remote[host] = p
                rc = p.wait()
            with lock:
                codes[host] = rc
            if rc != 0:
                failed.set()

        threads = []
        for host, node_rank, n, first in placements:
            t = threading.Thread(target=run_host, args=(host, node_rank, n, first), daemon=True)
            t.start()
            threads.append(t)
        ranks = {h: nr for h, nr, _, _ in placements}
        while any(t.is_alive() for t in threads):
            if failed.wait(0.2):
                bad = {h: c for h, c in codes.items() if c != 0}
                print(f"[cloudtik-run] host(s) {sorted(bad)} failed ({bad}): terminating the job on every host",
                      file=sys.stderr)
                self.terminate_all(rsh, remote, locals_, ranks, pidfile, lock)
                break
        for t in threads:
            t.join(timeout=60)
        bad = [c for c in codes.values() if c != 0]
        return bad[0] if bad else 0

    @staticmethod
    def terminate_all(rsh, remote, locals_, ranks, pidfile, lock):
        with lock:
            rem, loc = dict(remote), dict(locals_)
        for host, p in rem.items():
            if p.poll() is None:
                kill = f"[ -f {pidfile(ranks[host])} ] && kill -TERM -- -$(cat {pidfile(ranks[host])}) 2>/dev/null; true"
                subprocess.call(rsh + [host, kill], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        for ll in loc.values():
            ll._terminate_all()
        deadline = time.time() + 30
        for p in rem.values():
            try:
                p.wait(max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()


class MPILauncher(Launcher):
    def run(self) -> int:
        mpirun = shutil.which("mpirun")
        if mpirun is None:
            raise RuntimeError("mpirun not found: use --launcher distributed (RCCL does not need MPI)")
        hosts = ",".join(f"{h}:{n}" for h, _, n, _ in self.d.host_ranks())
        cmd = [mpirun, "-np", str(self.d.num_proc), "-H", hosts, "--bind-to", "none"]
        agent = cloudtik_rsh_agent(getattr(self.args, "rsh", None))
        if agent:
            # OpenMPI spawns its remote daemons through the agent (reference mpi_launcher.py:81)
            cmd += ["-mca", "plm_rsh_agent", agent]
        env = self.base_env()
        for k in ("MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "HSA_ENABLE_IPC_MODE_LEGACY"):
            cmd += ["-x", k]
        cmd += self.program()
        return subprocess.call(cmd, env=env)


def create_launcher(name: str, args, distributor: Distributor) -> Launcher:
    if name == "cpu" or (name == "local" and getattr(args, "cpu", False)):
        args.cpu = True
        return CpuLauncher(args, distributor, args.node_rank, args.first_rank, args.local_world or None)
    if name in ("local", "horovod-local"):
        if name == "horovod-local":
            args.launcher = "horovod"
        return LocalLauncher(args, distributor, args.node_rank, args.first_rank, args.local_world or None)
    if name in ("distributed", "rsh", "horovod"):
        return DistributedLauncher(args, distributor)
    if name == "mpi":
        return MPILauncher(args, distributor)
    raise ValueError(f"unknown launcher {name!r}")
