"""CPU-side launching: core pools, process placement, memory allocator and OpenMP runtime
(reference runtime/ai/runner/cpu/cpu_pool.py:97-384, cpu_launcher.py:48-296,
local_launcher.py:98-431).

On an MI355X node the GPU ranks are pinned by ``runner.affinity`` (the cores of each GPU's
NUMA node).  This module covers the CPU-only jobs the reference's CPU launcher serves --
data preprocessing, CPU inference / benchmarking, GBDT training -- and CPU-heavy helper
processes next to the GPU ranks:

* ``cpu_topology()`` reads ``lscpu -p`` (or sysfs) into (cpu, core, socket, node) records;
* ``CpuPoolScheduler.schedule()`` splits the physical (or logical) cores into per-process
  core lists: one process per socket (throughput mode), 4 cores per process (latency mode),
  N processes, N cores per process, optionally restricted to NUMA nodes / core ids and
  never straddling a node when asked;
* ``allocator_env()`` / ``omp_env()`` build the LD_PRELOAD + MALLOC_CONF / KMP_* / GOMP_*
  environment for jemalloc / tcmalloc and the Intel or GNU OpenMP runtime;
* ``CpuLauncher`` starts the processes, each under ``numactl -C cores -m node`` or
  ``taskset -c cores`` (or a plain affinity mask), with OMP_NUM_THREADS = its core count.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from cloudtik_amd.runner.affinity import parse_cpulist


@dataclass(frozen=True)
class CpuCore:
    cpu: int          # logical CPU id
    core: int         # physical core id (unique over the machine)
    socket: int
    node: int         # NUMA node
    physical: bool    # the first hardware thread of its core


def _parse_lscpu(text: str) -> List[CpuCore]:
    rows = []
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        f = line.split(",")
        cpu, core, sock = int(f[0]), int(f[1] or 0), int(f[2] or 0)
        node = int(f[3]) if len(f) > 3 and f[3] != "" else sock
        rows.append((cpu, core, sock, node))
    seen = set()
    out = []
    for cpu, core, sock, node in sorted(rows):
        key = (sock, core)
        out.append(CpuCore(cpu, core, sock, node, key not in seen))
        seen.add(key)
    return out


def _sysfs_topology(root: str = "/sys/devices/system") -> List[CpuCore]:
    rows = []
    node_of = {}
    for nd in glob.glob(os.path.join(root, "node", "node[0-9]*")):
        try:
            with open(os.path.join(nd, "cpulist")) as f:
                for c in parse_cpulist(f.read()):
                    node_of[c] = int(os.path.basename(nd)[4:])
        except OSError:
            pass
    for cd in glob.glob(os.path.join(root, "cpu", "cpu[0-9]*")):
        cpu = int(os.path.basename(cd)[3:])
        try:
            with open(os.path.join(cd, "topology", "core_id")) as f:
                core = int(f.read())
            with open(os.path.join(cd, "topology", "physical_package_id")) as f:
                sock = int(f.read())
        except OSError:
            continue
        rows.append(f"{cpu},{sock * 100000 + core},{sock},{node_of.get(cpu, sock)}")
    return _parse_lscpu("\n".join(rows))


def cpu_topology(lscpu_text: Optional[str] = None) -> List[CpuCore]:
    """Every logical CPU of this machine (restricted to the current affinity mask), or of the
    given ``lscpu -p=CPU,Core,Socket,Node`` text."""
    text = lscpu_text
    if text is None and shutil.which("lscpu"):
        try:
            text = subprocess.run(["lscpu", "-p=CPU,Core,Socket,Node"], capture_output=True, text=True,
                                  timeout=10).stdout
        except (OSError, subprocess.SubprocessError):
            text = None
    live = lscpu_text is None
    cores = _parse_lscpu(text) if text else _sysfs_topology()
    if not cores:
        n = os.cpu_count() or 1
        cores = [CpuCore(i, i, 0, 0, True) for i in range(n)]
    if live:
        try:                                  # a container / cgroup may allow only part of the machine
            allowed = os.sched_getaffinity(0)
            cores = [c for c in cores if c.cpu in allowed] or cores
        except AttributeError:
            pass
    return cores


class CpuPoolScheduler:
    def __init__(self, cores: Optional[Sequence[CpuCore]] = None, lscpu_text: Optional[str] = None):
        self.pool: List[CpuCore] = list(cores) if cores is not None else cpu_topology(lscpu_text)

    def num_sockets(self) -> int:
        return len({c.socket for c in self.pool}) or 1

    def num_nodes(self) -> int:
        return len({c.node for c in self.pool}) or 1

    def physical_cores(self) -> List[CpuCore]:
        return [c for c in self.pool if c.physical]

    def schedule(self, num_proc: int = 0, ncores_per_proc: int = 0, use_logical_cores: bool = False,
                 skip_cross_node_cores: bool = False, nodes_list: Optional[Sequence[int]] = None,
                 cores_list: Optional[Sequence[int]] = None) -> List[List[CpuCore]]:
        """Per-process core lists.  Defaults: one process per NUMA node over its physical cores."""
        pool = self.pool if use_logical_cores else self.physical_cores()
        if nodes_list:
            pool = [c for c in pool if c.node in set(nodes_list)]
        if cores_list:
            want = set(cores_list)
            pool = [c for c in self.pool if c.cpu in want]       # explicit ids win over physical-only
        if not pool:
            raise ValueError("no CPU cores left after applying the node / core filters")
        # physical cores first, then their sibling threads, grouped by node in id order
        pool = sorted(pool, key=lambda c: (c.node, not c.physical, c.cpu))
        by_node: Dict[int, List[CpuCore]] = {}
        for c in pool:
            by_node.setdefault(c.node, []).append(c)
        if num_proc <= 0 and ncores_per_proc <= 0:
            return [cs for _, cs in sorted(by_node.items())]
        if ncores_per_proc <= 0:
            ncores_per_proc = max(1, len(pool) // num_proc)
        chunks: List[List[CpuCore]] = []
        if skip_cross_node_cores:
            for _, cs in sorted(by_node.items()):
                for i in range(0, len(cs) - ncores_per_proc + 1, ncores_per_proc):
                    chunks.append(cs[i:i + ncores_per_proc])
        else:
            for i in range(0, len(pool) - ncores_per_proc + 1, ncores_per_proc):
                chunks.append(pool[i:i + ncores_per_proc])
        if num_proc > 0:
            if len(chunks) < num_proc:
                raise ValueError(f"{num_proc} processes x {ncores_per_proc} cores do not fit in "
                                 f"{len(pool)} cores")
            chunks = chunks[:num_proc]
        if not chunks:
            raise ValueError(f"{ncores_per_proc} cores per process exceed the {len(pool)} available")
        return chunks


def ranges(ids: Sequence[int]) -> str:
    """[0,1,2,3,8,9] -> '0-3,8-9' (numactl / taskset / GOMP_CPU_AFFINITY syntax)."""
    ids = sorted(set(ids))
    out = []
    i = 0
    while i < len(ids):
        j = i
        while j + 1 < len(ids) and ids[j + 1] == ids[j] + 1:
            j += 1
        out.append(str(ids[i]) if i == j else f"{ids[i]}-{ids[j]}")
        i = j + 1
    return ",".join(out)


# ----------------------------------------------------------------------------- libraries
def library_dirs() -> List[str]:
    dirs = [d for d in os.environ.get("LD_LIBRARY_PATH", "").split(":") if d]
    for var in ("CONDA_PREFIX", "VIRTUAL_ENV"):
        if os.environ.get(var):
            dirs.append(os.path.join(os.environ[var], "lib"))
    dirs += [os.path.join(sys.prefix, "lib"), os.path.expanduser("~/.local/lib"), "/usr/local/lib",
             "/usr/local/lib64", "/usr/lib/x86_64-linux-gnu", "/usr/lib64", "/usr/lib"]
    seen, out = set(), []
    for d in dirs:
        if d not in seen:
            seen.add(d)
            out.append(d)
    return out


def find_library(names: Sequence[str], dirs: Optional[Sequence[str]] = None) -> Optional[str]:
    for d in (dirs if dirs is not None else library_dirs()):
        for n in names:
            hits = sorted(glob.glob(os.path.join(d, n)))
            if hits:
                return hits[0]
    return None


ALLOCATORS = ("auto", "default", "jemalloc", "tcmalloc")
_ALLOC_LIBS = {"jemalloc": ("libjemalloc.so", "libjemalloc.so.*"),
               "tcmalloc": ("libtcmalloc.so", "libtcmalloc.so.*", "libtcmalloc_minimal.so.*")}
# jemalloc: large allocations straight to dedicated extents, purging in a background thread;
# benchmark mode keeps freed pages (no decay) for steady-state latency at the price of RSS
_JEMALLOC_CONF = "oversize_threshold:1,background_thread:true,metadata_thp:auto"
_JEMALLOC_BENCH = ",dirty_decay_ms:-1,muzzy_decay_ms:-1"


def allocator_env(kind: str = "auto", benchmark: bool = False,
                  dirs: Optional[Sequence[str]] = None) -> Tuple[List[str], Dict[str, str], str]:
    """(LD_PRELOAD entries, env vars, allocator actually used)."""
    if kind not in ALLOCATORS:
        raise ValueError(f"memory allocator must be one of {ALLOCATORS}")
    if kind == "default":
        return [], {}, "default"
    order = ["jemalloc", "tcmalloc"] if kind == "auto" else [kind]
    for k in order:
        lib = find_library(_ALLOC_LIBS[k], dirs)
        if lib:
            env = {}
            if k == "jemalloc":
                env["MALLOC_CONF"] = _JEMALLOC_CONF + (_JEMALLOC_BENCH if benchmark else "")
            return [lib], env, k
    if kind != "auto":
        print(f"[cloudtik-run] {kind} not found in {list(dirs or library_dirs())[:4]}...: using the default "
              f"allocator", file=sys.stderr)
    return [], {}, "default"


OMP_RUNTIMES = ("auto", "default", "intel")


def omp_env(kind: str, cores: Sequence[int], set_affinity: bool = True,
            dirs: Optional[Sequence[str]] = None) -> Tuple[List[str], Dict[str, str], str]:
    """(LD_PRELOAD entries, env vars, runtime used) for one process running on ``cores``."""
    if kind not in OMP_RUNTIMES:
        raise ValueError(f"OpenMP runtime must be one of {OMP_RUNTIMES}")
    env = {"OMP_NUM_THREADS": str(max(1, len(cores)))}
    if kind in ("auto", "intel"):
        lib = find_library(("libiomp5.so",), dirs)
        if lib:
            env["KMP_BLOCKTIME"] = "1"
            if set_affinity:
                env["KMP_AFFINITY"] = "granularity=fine,compact,1,0"
            return [lib], env, "intel"
        if kind == "intel":
            print("[cloudtik-run] libiomp5.so not found: using the GNU OpenMP runtime", file=sys.stderr)
    if set_affinity and cores:
        env["GOMP_CPU_AFFINITY"] = " ".join(str(c) for c in cores)
        env["OMP_PROC_BIND"] = "true"
    return [], env, "default"


TASK_MANAGERS = ("auto", "none", "numactl", "taskset")


def task_prefix(manager: str, cores: Sequence[CpuCore]) -> Tuple[List[str], str]:
    """Command prefix pinning a process to ``cores`` (and, with numactl, its memory to their
    node when they all share one)."""
    if manager not in TASK_MANAGERS:
        raise ValueError(f"task manager must be one of {TASK_MANAGERS}")
    ids = ranges([c.cpu for c in cores])
    cand = ["numactl", "taskset"] if manager == "auto" else [manager]
    for m in cand:
        if m == "none":
            break
        if not shutil.which(m):
            if manager != "auto":
                print(f"[cloudtik-run] {m} not found: pinning with the affinity mask only", file=sys.stderr)
            continue
        if m == "numactl":
            nodes = {c.node for c in cores}
            return (["numactl", "-C", ids] + (["-m", str(nodes.pop())] if len(nodes) == 1 else [])), "numactl"
        return ["taskset", "-c", ids], "taskset"
    return [], "none"


def apply_mode(args, scheduler: CpuPoolScheduler) -> None:
    """--latency-mode: 4 physical cores per process over all cores; --throughput-mode: one
    process per socket.  Both override --num-proc / --ncores-per-proc / --nodes-list."""
    if args.latency_mode and args.throughput_mode:
        raise ValueError("--latency-mode and --throughput-mode are exclusive")
    if args.latency_mode:
        args.ncores_per_proc, args.num_proc, args.use_logical_cores, args.nodes_list = 4, 0, False, ""
    elif args.throughput_mode:
        args.num_proc, args.ncores_per_proc, args.use_logical_cores, args.nodes_list = \
            scheduler.num_sockets(), 0, False, ""


def cpu_plan(args, scheduler: Optional[CpuPoolScheduler] = None, dirs: Optional[Sequence[str]] = None):
    """[(argv prefix, env, cores)] for every process of a CPU job."""
    scheduler = scheduler or CpuPoolScheduler()
    apply_mode(args, scheduler)
    sched = scheduler.schedule(num_proc=args.num_proc, ncores_per_proc=args.ncores_per_proc,
                               use_logical_cores=args.use_logical_cores,
                               skip_cross_node_cores=args.skip_cross_node_cores,
                               nodes_list=parse_cpulist(args.nodes_list) if args.nodes_list else None,
                               cores_list=parse_cpulist(args.cores_list) if args.cores_list else None)
    pre_a, env_a, _ = allocator_env(args.memory_allocator, args.benchmark, dirs)
    out = []
    all_cores = {c.cpu for p in sched for c in p}
    for cores in sched:
        ids = [c.cpu for c in cores]
        # pinning every logical CPU of the machine: leave the OpenMP runtime's own placement
        set_aff = not (args.use_logical_cores and len(all_cores) == len(scheduler.pool))
        pre_o, env_o, _ = omp_env(args.omp_runtime, ids, set_aff, dirs)
        env = dict(env_a)
        env.update(env_o)
        preload = [p for p in os.environ.get("LD_PRELOAD", "").split(":") if p] + pre_a + pre_o
        if preload:
            env["LD_PRELOAD"] = ":".join(dict.fromkeys(preload))
        prefix, _ = task_prefix(args.task_manager, cores)
        out.append((prefix, env, ids))
    return out


def add_cpu_args(p) -> None:
    g = p.add_argument_group("CPU launching (--launcher cpu)")
    g.add_argument("--ncores-per-proc", "--ncores_per_proc", type=int, default=0)
    g.add_argument("--nodes-list", "--nodes_list", default="", help="NUMA nodes, e.g. 0,1 or 0-1")
    g.add_argument("--cores-list", "--cores_list", default="", help="logical CPU ids, e.g. 0-15,32-47")
    g.add_argument("--use-logical-cores", "--use_logical_cores", action="store_true")
    g.add_argument("--skip-cross-node-cores", "--skip_cross_node_cores", action="store_true")
    g.add_argument("--task-manager", "--task_manager", default="auto", choices=TASK_MANAGERS)
    g.add_argument("--latency-mode", "--latency_mode", action="store_true")
    g.add_argument("--throughput-mode", "--throughput_mode", action="store_true")
    g.add_argument("--memory-allocator", "--memory_allocator", default="auto", choices=ALLOCATORS)
    g.add_argument("--omp-runtime", "--omp_runtime", default="auto", choices=OMP_RUNTIMES)
    g.add_argument("--benchmark", action="store_true",
                   help="jemalloc tuned for steady-state latency (freed pages are kept)")


CPU_FLAGS = ("ncores_per_proc", "nodes_list", "cores_list", "use_logical_cores", "skip_cross_node_cores",
             "task_manager", "latency_mode", "throughput_mode", "memory_allocator", "omp_runtime", "benchmark")


def cpu_flags_argv(args) -> List[str]:
    """The CPU flags of ``args`` as command-line arguments (for remote node launchers)."""
    out = []
    for k in CPU_FLAGS:
        v = getattr(args, k, None)
        flag = "--" + k.replace("_", "-")
        if isinstance(v, bool):
            if v:
                out.append(flag)
        elif v not in (None, "", 0):
            out += [flag, str(v)]
    return out
