"""``cloudtik cluster-dump`` / ``cloudtik head cluster-dump`` / ``cloudtik node dump``: collect
what is needed to debug a cluster into one tarball (reference
core/_private/cluster/cluster_dump.py:42-77 parameters, :227-360 local collection,
:546-758 remote collection).

Per node (``collect_local``, run ON the node by ``cloudtik node dump``):

* ``logs/``            -- the session logs (+ the runtimes' log directories, ``Runtime.get_logs``);
* ``debug_state.txt``  -- the controller's last scaler state (written each round on the head);
* ``pip_packages.txt`` -- installed Python distributions (importlib.metadata; no pip internals);
* ``meta/process_info.txt`` -- the CloudTik daemons and the runtimes' processes from the
  process table (``--processes-verbose``: full command lines);
* ``gpu/``             -- AMD GPU state, the MI355X replacement of the reference's nvidia
  probes: ``amd-smi static/metric --json`` (``rocm-smi`` as fallback), the KFD topology of
  every GPU node and the RAS error counters from sysfs.

Cluster level (``dump_cluster``): the nodes are picked by ``--hosts`` (IPs or node ids) or
``--head-only``; the local node is collected in-process, every other node runs ``cloudtik
node dump`` through its command executor and the archive is copied back -- in parallel
(``MAX_PARALLEL_DUMP_WORKERS`` threads), one failing node never stops the rest (its error
goes to ``dump_failures.txt``).  Each node lands under ``head_<ip>/`` or ``worker_<ip>/``.
From the CLI host the whole collection runs ON THE HEAD (``cloudtik head cluster-dump``,
which reaches the workers on the cluster network) and only the result is copied back.
"""
from __future__ import annotations

import json
import logging
import os
import shlex
import shutil
import subprocess
import tarfile
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

logger = logging.getLogger(__name__)

MAX_PARALLEL_DUMP_WORKERS = 16
DEBUG_STATE_FILE = "debug_state.txt"


@dataclass
class DumpParameters:
    logs: bool = True
    debug_state: bool = True
    pip: bool = True
    processes: bool = True
    processes_verbose: bool = True
    gpu: bool = True
    runtimes: List[str] = field(default_factory=list)

    def node_flags(self) -> List[str]:
        out = []
        for name in ("logs", "debug_state", "pip", "processes", "processes_verbose", "gpu"):
            flag = name.replace("_", "-")
            out.append(f"--{flag}" if getattr(self, name) else f"--no-{flag}")
        if self.runtimes:
            out.append(f"--runtimes={shlex.quote(','.join(self.runtimes))}")
        return out


# ------------------------------------------------------------------------------ local node
def _write(root: str, rel: str, text: str):
    path = os.path.join(root, rel)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


def _copy_tree(src: str, dst: str):
    src = os.path.expanduser(src)
    if not os.path.isdir(src):
        return
    for base, _, files in os.walk(src):
        for fn in files:
            s = os.path.join(base, fn)
            d = os.path.join(dst, os.path.relpath(s, src))
            os.makedirs(os.path.dirname(d), exist_ok=True)
            try:
                shutil.copy2(s, d)
            except OSError:
                pass


def pip_packages() -> str:
    from importlib import metadata
    names = sorted({f"{d.metadata['Name']}=={d.version}" for d in metadata.distributions() if d.metadata['Name']},
                   key=str.lower)
    return "\n".join(names) + "\n"


def _process_keywords(runtimes: List[str]) -> List[Tuple[str, bool]]:
    from cloudtik_amd.core import constants as C
    kws = [(p, False) for p in (C.PROCESS_TYPE_STATE_SERVER, C.PROCESS_TYPE_CLUSTER_CONTROLLER,
                                C.PROCESS_TYPE_NODE_MONITOR, C.PROCESS_TYPE_LOG_MONITOR, C.PROCESS_TYPE_REAPER,
                                "cloudtik-state-server", "cloudtik_amd.core")]
    if runtimes:
        from cloudtik_amd.core import runtime_factory as rf
        for t in runtimes:
            try:
                for p in rf.get_runtime(t, {}).get_processes() or []:
                    kws.append((p[0], bool(p[1])))
            except Exception:  # noqa: BLE001 - unknown runtime: skip its processes
                continue
    return kws


def process_table(runtimes: List[str], verbose: bool) -> List[Dict[str, Any]]:
    import psutil
    kws = _process_keywords(runtimes)
    out = []
    for p in psutil.process_iter(["pid", "name", "cmdline", "status", "create_time", "memory_info"]):
        try:
            info = p.info
            cmd = info.get("cmdline") or []
            line = subprocess.list2cmdline(cmd)
            if not any((kw in (info.get("name") or "")) if by_name else (kw in line) for kw, by_name in kws):
                continue
            rss = info.get("memory_info").rss if info.get("memory_info") else None
            out.append({"pid": info["pid"], "name": info.get("name"), "status": info.get("status"),
                        "executable": line if verbose else (cmd[0] if cmd else ""), "rss_bytes": rss,
                        "started": info.get("create_time")})
        except (psutil.NoSuchProcess, psutil.AccessDenied):
            continue
    return out


def _run(cmd: List[str], timeout: float = 30.0) -> Optional[str]:
    if shutil.which(cmd[0]) is None:
        return None
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
        return r.stdout if r.returncode == 0 else (r.stdout + r.stderr)
    except (OSError, subprocess.SubprocessError) as e:
        return f"{cmd[0]} failed: {e}\n"


def gpu_state(root: str, sysfs: str = "/sys") -> List[str]:
    """AMD GPU state files written under ``root``; returns the relative names written."""
    written = []
    for name, cmd in (("amd-smi-static.json", ["amd-smi", "static", "--json"]),
                      ("amd-smi-metric.json", ["amd-smi", "metric", "--json"]),
                      ("amd-smi-xgmi.txt", ["amd-smi", "xgmi"])):
        out = _run(cmd)
        if out is not None:
            _write(root, name, out)
            written.append(name)
    if not written:
        out = _run(["rocm-smi", "--showallinfo", "--json"])
        if out is not None:
            _write(root, "rocm-smi.json", out)
            written.append("rocm-smi.json")
    topo = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    if os.path.isdir(topo):
        rows = []
        for n in sorted(os.listdir(topo), key=lambda x: int(x) if x.isdigit() else 0):
            try:
                with open(os.path.join(topo, n, "properties")) as f:
                    props = dict(ln.split(None, 1) for ln in f.read().splitlines() if " " in ln)
            except OSError:
                continue
            if props.get("simd_count", "0").strip() != "0":
                rows.append({"node": n, **{k: v.strip() for k, v in props.items()}})
        _write(root, "kfd_topology.json", json.dumps(rows, indent=1))
        written.append("kfd_topology.json")
    drm = os.path.join(sysfs, "class", "drm")
    ras = {}
    if os.path.isdir(drm):
        for card in sorted(os.listdir(drm)):
            d = os.path.join(drm, card, "device", "ras")
            if not card.startswith("card") or "-" in card or not os.path.isdir(d):
                continue
            ras[card] = {}
            for fn in sorted(os.listdir(d)):
                if fn.endswith("_err_count"):
                    try:
                        with open(os.path.join(d, fn)) as f:
                            ras[card][fn] = f.read().strip()
                    except OSError:
                        pass
    if ras:
        _write(root, "ras_errors.json", json.dumps(ras, indent=1))
        written.append("ras_errors.json")
    return written


def collect_local(params: DumpParameters, output: Optional[str] = None, sysfs: str = "/sys") -> str:
    """This node's data as a .tar.gz (path returned)."""
    from cloudtik_amd.core import services
    output = output or os.path.join(tempfile.gettempdir(), f"cloudtik-node-dump-{os.getpid()}-{time.time_ns()}.tar.gz")
    tmp = tempfile.mkdtemp(prefix="cloudtik-node-dump-")
    try:
        notes = []
        if params.logs:
            _copy_tree(services.logs_dir(), os.path.join(tmp, "logs"))
            if params.runtimes:
                from cloudtik_amd.core import runtime_factory as rf
                for t in params.runtimes:
                    try:
                        for name, path in (rf.get_runtime(t, {}).get_logs() or {}).items():
                            _copy_tree(os.path.expandvars(path), os.path.join(tmp, "logs", "runtimes", t, name))
                    except Exception as e:  # noqa: BLE001
                        notes.append(f"runtime {t} logs: {e}")
        if params.debug_state:
            src = os.path.join(services.logs_dir(), DEBUG_STATE_FILE)
            if os.path.exists(src):
                shutil.copy2(src, os.path.join(tmp, DEBUG_STATE_FILE))
        if params.pip:
            _write(tmp, "pip_packages.txt", pip_packages())
        if params.processes:
            import yaml
            rows = process_table(params.runtimes, params.processes_verbose)
            _write(tmp, os.path.join("meta", "process_info.txt"), yaml.safe_dump_all(rows) if rows else "")
        if params.gpu:
            gpu_state(os.path.join(tmp, "gpu"), sysfs=sysfs)
        if notes:
            _write(tmp, "notes.txt", "\n".join(notes) + "\n")
        with tarfile.open(output, "w:gz") as tar:
            for name in sorted(os.listdir(tmp)):
                tar.add(os.path.join(tmp, name), arcname=name)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return output


def write_debug_state(summary: Dict[str, Any]):
    """Head: the controller's latest scaler state (reference debug_state.txt)."""
    from cloudtik_amd.core import services
    path = os.path.join(services.logs_dir(), DEBUG_STATE_FILE)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(summary, f, indent=1, default=str, sort_keys=True)
    os.replace(tmp, path)


# ------------------------------------------------------------------------------ cluster
def select_nodes(config: Dict[str, Any], provider, hosts: Optional[str] = None,
                 head_only: bool = False) -> List[Tuple[str, str, bool]]:
    """(node id, ip, is head) of the nodes to dump: the head + workers, only the head, or the
    nodes named in ``hosts`` (IPs or node ids, comma separated)."""
    from cloudtik_amd.core import tags as T
    from cloudtik_amd.core.cluster_utils import get_head_node, get_worker_nodes
    head = get_head_node(provider, config["cluster_name"])
    nodes = []
    if head is not None:
        nodes.append((head, provider.internal_ip(head) or head, True))
    if not head_only:
        nodes += [(w, provider.internal_ip(w) or w, False) for w in get_worker_nodes(provider, config["cluster_name"])]
    if hosts:
        want = {h.strip() for h in hosts.split(",") if h.strip()}
        nodes = [n for n in nodes if n[0] in want or n[1] in want]
        missing = want - {n[0] for n in nodes} - {n[1] for n in nodes}
        if missing:
            logger.warning("no cluster node matches %s", sorted(missing))
    _ = T
    return nodes


def _is_local(ip: str) -> bool:
    from cloudtik_amd.core.executor import local_ips
    return ip in set(local_ips())


def _extract_into(tar_path: str, root: str, subdir: str):
    dst = os.path.join(root, subdir)
    os.makedirs(dst, exist_ok=True)
    with tarfile.open(tar_path, "r:gz") as t:
        for m in t.getmembers():
            # never write outside the node's directory (archives come from remote nodes)
            target = os.path.realpath(os.path.join(dst, m.name))
            if not target.startswith(os.path.realpath(dst) + os.sep) and target != os.path.realpath(dst):
                continue
            if m.issym() or m.islnk():
                continue
            t.extract(m, dst)


def dump_node(config, provider, node: Tuple[str, str, bool], params: DumpParameters, root: str,
              executor_fn=None):
    """Collect one node into ``root/<head|worker>_<ip>/``."""
    node_id, ip, is_head = node
    sub = f"{'head' if is_head else 'worker'}_{ip}"
    if _is_local(ip):
        path = collect_local(params)
        try:
            _extract_into(path, root, sub)
        finally:
            os.remove(path)
        return sub
    if executor_fn is None:
        from cloudtik_amd.core.cluster_operator import _executor as executor_fn  # noqa: N813
    ex = executor_fn(config, provider, node_id)
    remote = f"/tmp/cloudtik_dump_{'head' if is_head else 'worker'}_{ip.replace(':', '_')}_{os.getpid()}.tar.gz"
    ex.run(" ".join(["cloudtik", "node", "dump", "--silent", "--output", remote] + params.node_flags()), timeout=600)
    fd, local = tempfile.mkstemp(prefix=f"cloudtik_dump_{ip}_", suffix=".tar.gz")
    os.close(fd)
    try:
        ex.run_rsync_down(remote, local)
        _extract_into(local, root, sub)
    finally:
        os.remove(local)
        try:
            ex.run(f"rm -f {shlex.quote(remote)}", timeout=60)
        except Exception:  # noqa: BLE001 - a leftover temp file on the node is harmless
            pass
    return sub


def dump_cluster(config: Dict[str, Any], provider, params: DumpParameters, output: Optional[str] = None,
                 hosts: Optional[str] = None, head_only: bool = False, executor_fn=None,
                 parallel: int = MAX_PARALLEL_DUMP_WORKERS) -> str:
    """Collect the selected nodes in parallel into one archive (run where the nodes are
    reachable: the head, or a CLI host of a local / on-premise cluster)."""
    from cloudtik_amd.core.cluster_operator import get_cluster_info
    nodes = select_nodes(config, provider, hosts, head_only)
    name = config["cluster_name"]
    output = os.path.expanduser(output or os.path.join(os.getcwd(), f"{name}_{time.strftime('%Y-%m-%d_%H-%M-%S')}.tar.gz"))
    root = tempfile.mkdtemp(prefix="cloudtik-cluster-dump-")
    failures = {}
    try:
        try:
            _write(root, "cluster_info.json", json.dumps(get_cluster_info(config), indent=1, default=str))
        except Exception as e:  # noqa: BLE001
            failures["cluster_info"] = repr(e)
        from cloudtik_amd.core.cluster_config import get_runtime_types

        def one(n):
            p = DumpParameters(**{**params.__dict__, "runtimes": list(params.runtimes or get_runtime_types(config))})
            return dump_node(config, provider, n, p, root, executor_fn)

        with ThreadPoolExecutor(max_workers=max(1, min(parallel, len(nodes) or 1))) as pool:
            futs = {n[1]: pool.submit(one, n) for n in nodes}
            for ip, f in futs.items():
                try:
                    f.result()
                except Exception as e:  # noqa: BLE001 - one node never stops the rest
                    failures[ip] = repr(e)
                    logger.error("dump of node %s failed: %s", ip, e)
        if failures:
            _write(root, "dump_failures.txt", "".join(f"{k}: {v}\n" for k, v in sorted(failures.items())))
        base = os.path.basename(output).split(".tar")[0]
        with tarfile.open(output, "w:gz") as tar:
            tar.add(root, arcname=base)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return output
