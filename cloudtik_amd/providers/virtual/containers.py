"""Container nodes for the virtual provider (reference providers/_private/virtual/
virtual_container_scheduler.py + virtual_docker_command_executor.py: one docker container
per node on a bridge network, CPU / memory limits, data disks, shared data dirs).

MI355X-first layout: a node is a container that owns an exclusive slice of the host --

* **GPUs**: whole devices, passed through as ``/dev/kfd`` + the device's own render node
  ``/dev/dri/renderD<minor>`` (minor from the KFD topology, so the container's HIP device 0
  is the allocated GPU -- no ``HIP_VISIBLE_DEVICES`` games, the container cannot see the
  other GPUs at all);
* **CPUs**: a ``--cpuset-cpus`` taken from the NUMA node the node's first GPU hangs off (the
  xGMI-attached socket), so host-side data loading runs next to its GPU;
* **memory**: ``--memory`` from the node type, ``--shm-size`` a fraction of it (RCCL and
  DataLoader workers live in /dev/shm);
* **disks**: per-node host directories bind-mounted as ``/mnt/cloudtik/data_disk_<k>``
  (deleted with the node unless ``permanent_data_volumes``), shared ``data_dirs`` under
  ``/cloudtik/data/<name>``, and the cluster state dir under ``/cloudtik/state``.

Every container joins the workspace's user-defined bridge network (``cloudtik-<workspace>``),
so nodes reach each other by address and name; labels carry the node tags.  Allocations are
recorded in the provider's state file, so a second ``cloudtik up`` on the same host never
hands out a GPU or core twice.  ``docker`` is driven through an injectable runner (tests use a
fake).
"""
from __future__ import annotations

import json
import os
import shlex
import subprocess
from typing import Any, Callable, Dict, List, Optional, Tuple

from cloudtik_amd.core.node_provider import NodeLaunchException

DATA_DISK_MOUNT = "/mnt/cloudtik/data_disk_{}"
DATA_DIR_MOUNT = "/cloudtik/data/{}"
STATE_MOUNT = "/cloudtik/state"

Runner = Callable[[List[str]], Tuple[int, str, str]]


def _subprocess_runner(cmd: List[str]) -> Tuple[int, str, str]:
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    return r.returncode, r.stdout, r.stderr


def host_gpus(kfd_root: str = "/sys/class/kfd/kfd/topology/nodes", drm_root: str = "/sys/class/drm") \
        -> List[Dict[str, int]]:
    """[{index, render_minor, numa}] of the host's AMD GPUs in HIP device order."""
    from cloudtik_amd.core.resources import kfd_gpu_nodes
    out = []
    for i, kv in enumerate(kfd_gpu_nodes(kfd_root)):
        minor = kv.get("drm_render_minor", 128 + i)
        numa = 0
        try:
            with open(os.path.join(drm_root, f"renderD{minor}", "device", "numa_node")) as f:
                numa = max(0, int(f.read().strip()))
        except (OSError, ValueError):
            pass
        out.append({"index": i, "render_minor": int(minor), "numa": numa})
    return out


def host_numa_cpus() -> Dict[int, List[int]]:
    from cloudtik_amd.runner.affinity import parse_cpulist
    out = {}
    root = "/sys/devices/system/node"
    try:
        for d in sorted(os.listdir(root)):
            if d.startswith("node") and d[4:].isdigit():
                with open(os.path.join(root, d, "cpulist")) as f:
                    out[int(d[4:])] = parse_cpulist(f.read())
    except OSError:
        pass
    return out or {0: list(range(os.cpu_count() or 1))}


def _mem_mb(v) -> int:
    if v is None:
        return 0
    if isinstance(v, (int, float)):
        return int(v) // (1024 * 1024) if v > 1 << 20 else int(v)
    from cloudtik_amd.core.resources import parse_memory
    return parse_memory(v) // (1024 * 1024)


class ContainerScheduler:
    """Allocates whole GPUs and NUMA-local cores to container nodes; the allocation table lives
    in the provider's state (``st['alloc'] = {node_id: {gpus, cpus}}``)."""

    def __init__(self, gpus: List[Dict[str, int]], numa_cpus: Dict[int, List[int]], reserve_cpus: int = 0):
        self.gpus = gpus
        self.numa_cpus = numa_cpus
        self.reserve = set(sorted(c for cs in numa_cpus.values() for c in cs)[:reserve_cpus])

    def allocate(self, alloc: Dict[str, Dict[str, List[int]]], n_gpu: int, n_cpu: int) -> Dict[str, List[int]]:
        used_g = {g for a in alloc.values() for g in a.get("gpus", [])}
        used_c = {c for a in alloc.values() for c in a.get("cpus", [])} | self.reserve
        free_g = [g for g in self.gpus if g["index"] not in used_g]
        if n_gpu > len(free_g):
            raise NodeLaunchException("InsufficientGPUs", f"{n_gpu} GPUs requested, {len(free_g)} free on the host")
        # GPUs: prefer a set on one NUMA node (one socket's xGMI neighbourhood)
        by_numa: Dict[int, List[Dict[str, int]]] = {}
        for g in free_g:
            by_numa.setdefault(g["numa"], []).append(g)
        pick = next((gs[:n_gpu] for _, gs in sorted(by_numa.items()) if len(gs) >= n_gpu), free_g[:n_gpu])
        # CPUs: from the first GPU's NUMA node first, then the others
        home = pick[0]["numa"] if pick else None
        order = ([home] if home in self.numa_cpus else []) + [n for n in sorted(self.numa_cpus) if n != home]
        cpus: List[int] = []
        for n in order:
            for c in self.numa_cpus[n]:
                if len(cpus) == n_cpu:
                    break
                if c not in used_c:
                    cpus.append(c)
        if len(cpus) < n_cpu:
            raise NodeLaunchException("InsufficientCPUs", f"{n_cpu} cores requested, {len(cpus)} free on the host")
        return {"gpus": [g["index"] for g in pick], "cpus": sorted(cpus)}


def _ranges(cpus: List[int]) -> str:
    out, start, prev = [], None, None
    for c in sorted(cpus):
        if start is None:
            start = prev = c
        elif c == prev + 1:
            prev = c
        else:
            out.append(f"{start}-{prev}" if start != prev else str(start))
            start = prev = c
    if start is not None:
        out.append(f"{start}-{prev}" if start != prev else str(start))
    return ",".join(out)


class DockerNodes:
    """docker container lifecycle for virtual nodes."""

    def __init__(self, provider_config: Dict[str, Any], cluster_name: str, workspace_name: str, state_dir: str,
                 runner: Optional[Runner] = None, gpus: Optional[List[Dict[str, int]]] = None,
                 numa_cpus: Optional[Dict[int, List[int]]] = None):
        self.cfg = provider_config
        self.cluster = cluster_name
        self.network = provider_config.get("docker_network") or f"cloudtik-{workspace_name}"
        self.docker = list(provider_config.get("docker_cmd", ["docker"]))
        self.runner = runner or _subprocess_runner
        self.state_dir = state_dir
        self.disk_root = provider_config.get("data_disk_root") or os.path.join(state_dir, "disks")
        self.scheduler = ContainerScheduler(gpus if gpus is not None else host_gpus(),
                                            numa_cpus if numa_cpus is not None else host_numa_cpus(),
                                            int(provider_config.get("reserved_host_cpus", 0)))

    def _d(self, *args, check: bool = True) -> str:
        rc, out, err = self.runner(self.docker + list(args))
        if check and rc != 0:
            raise RuntimeError(f"docker {' '.join(args[:2])} failed: {err.strip()[:400]}")
        return out

    def ensure_network(self):
        rc, _, _ = self.runner(self.docker + ["network", "inspect", self.network])
        if rc != 0:
            self._d("network", "create", "--driver", "bridge", "--label", "cloudtik-managed=true", self.network)

    def run_args(self, node_id: str, node_config: Dict[str, Any], tags: Dict[str, str],
                 alloc: Dict[str, List[int]], gpus: List[Dict[str, int]], seq: int) -> List[str]:
        it = node_config.get("instance_type") if isinstance(node_config.get("instance_type"), dict) else {}
        mem = _mem_mb(it.get("memory") or node_config.get("memory"))
        args = ["run", "-d", "--name", node_id, "--hostname", node_id, "--network", self.network,
                "--restart", "unless-stopped", "--ipc", "private", "--ulimit", "memlock=-1:-1"]
        for k, v in sorted(tags.items()):
            args += ["--label", f"{k}={v}"]
        args += ["--label", f"cloudtik-virtual-node={node_id}"]
        if alloc["cpus"]:
            args += ["--cpuset-cpus", _ranges(alloc["cpus"]), "--cpus", str(len(alloc["cpus"]))]
        if mem:
            args += ["--memory", f"{mem}m",
                     "--shm-size", f"{int(mem * float(node_config.get('shared_memory_ratio', 0.3)))}m"]
        if alloc["gpus"]:
            minors = {g["index"]: g["render_minor"] for g in gpus}
            args += ["--device", "/dev/kfd"]
            for gi in alloc["gpus"]:
                args += ["--device", f"/dev/dri/renderD{minors[gi]}"]
            args += ["--group-add", "video", "--group-add", "render", "--cap-add", "SYS_PTRACE",
                     "--security-opt", "seccomp=unconfined"]
        for k, d in enumerate(self.data_disks(node_id, node_config, tags, seq), 1):
            args += ["-v", f"{d}:{DATA_DISK_MOUNT.format(k)}"]
        for d in node_config.get("data_dirs") or self.cfg.get("data_dirs") or []:
            args += ["-v", f"{d}:{DATA_DIR_MOUNT.format(os.path.basename(d.rstrip('/')))}"]
        args += ["-v", f"{self.state_dir}:{STATE_MOUNT}"]
        for hp, cp in (node_config.get("port_mappings") or {}).items():
            args += ["-p", f"{hp}:{cp}"]
        image = node_config.get("image") or self.cfg.get("image") or "rocm/pytorch:latest"
        return args + [image, "sleep", "infinity"]

    def data_disks(self, node_id: str, node_config: Dict[str, Any], tags: Dict[str, str], seq: int) -> List[str]:
        """Host directories backing the node's data disks: ``data_disks`` is either a count
        (directories under ``data_disk_root``) or, as in the reference's virtual configs, a
        list of host disk roots -- one per-node directory on each."""
        spec = node_config.get("data_disks") or 0
        owner = f"{self.cluster}-node-{seq}" if self.cfg.get("permanent_data_volumes") else node_id
        if isinstance(spec, (list, tuple)):
            return [os.path.join(os.path.expanduser(root), owner) for root in spec]
        return [os.path.join(self.disk_root, owner, f"disk_{k}") for k in range(1, int(spec) + 1)]

    def stop_disks(self, node_id: str, node_config: Optional[Dict[str, Any]]) -> List[str]:
        spec = (node_config or {}).get("data_disks")
        if isinstance(spec, (list, tuple)):
            return [os.path.join(os.path.expanduser(root), node_id) for root in spec]
        return [os.path.join(self.disk_root, node_id)]

    def start(self, node_id: str, node_config, tags, alloc, seq: int) -> str:
        self.ensure_network()
        for d in self.data_disks(node_id, node_config, tags, seq):
            os.makedirs(d, exist_ok=True)
        self._d(*self.run_args(node_id, node_config, tags, alloc, self.scheduler.gpus, seq))
        return self.ip(node_id)

    def ip(self, node_id: str) -> str:
        out = self._d("inspect", "-f", "{{json .NetworkSettings.Networks}}", node_id)
        nets = json.loads(out or "{}")
        net = nets.get(self.network) or next(iter(nets.values()), {})
        return net.get("IPAddress", "")

    def stop(self, node_id: str, node_config: Optional[Dict[str, Any]] = None, seq: int = 0):
        self._d("rm", "-f", node_id, check=False)
        if not self.cfg.get("permanent_data_volumes") and self.cfg.get("data_disks.delete_on_termination", True):
            import shutil
            for d in self.stop_disks(node_id, node_config):
                shutil.rmtree(d, ignore_errors=True)

    def running(self) -> Dict[str, Dict[str, str]]:
        out = self._d("ps", "--filter", f"label=cloudtik-cluster-name={self.cluster}", "--format", "{{.Names}}",
                      check=False)
        return {n: {} for n in out.split()}


class ContainerExecutor:
    """Runs node commands inside the node's container (``docker exec``); file transfer with
    ``docker cp``.  Wraps the host executor so ``run_env='host'`` still reaches the host."""

    def __init__(self, host, container: str, docker_cmd: str = "docker"):
        self.host = host
        self.container = container
        self.docker = docker_cmd

    def __getattr__(self, name):
        return getattr(self.host, name)

    def run(self, cmd=None, timeout=120, exit_on_fail=False, port_forward=None, with_output=False,
            environment_variables=None, run_env="auto", ssh_options_override_ssh_key="",
            shutdown_after_run=False, cmd_to_print=None, silent=False):
        if not cmd:
            return None
        if run_env == "host":
            return self.host.run(cmd, timeout, exit_on_fail, port_forward, with_output, environment_variables,
                                 run_env, ssh_options_override_ssh_key, shutdown_after_run, cmd_to_print, silent)
        from cloudtik_amd.core.executor import run_cmd_with_runner, with_environment_variables
        inner = with_environment_variables(cmd, environment_variables or {})
        return run_cmd_with_runner(self.host.process_runner,
                                   [self.docker, "exec", self.container, "bash", "-lc", inner],
                                   with_output=with_output, silent=silent)

    def run_rsync_up(self, source, target, options=None):
        self.host.process_runner.check_call([self.docker, "exec", self.container, "mkdir", "-p",
                                             os.path.dirname(target.rstrip("/")) or "/"])
        self.host.process_runner.check_call([self.docker, "cp", source, f"{self.container}:{target}"])

    def run_rsync_down(self, source, target, options=None):
        self.host.process_runner.check_call([self.docker, "cp", f"{self.container}:{source}", target])

    def remote_shell_command_str(self):
        return f"{self.docker} exec -it {shlex.quote(self.container)} bash\n"
