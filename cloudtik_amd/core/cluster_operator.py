"""Cluster lifecycle operations behind the ``cloudtik`` CLI and the Python API
(reference core/_private/cluster/cluster_operator.py: create_or_update_cluster:228,
get_or_create_head_node:869, teardown_cluster:375, exec / rsync / attach:1210-1556,
get_head_node_ip:1731, show_cluster_info:2146, scale_cluster:3821,
submit_and_exec:4189, wait_for_ready:4432, health_check:4483, resource metrics:4752,
cluster_dump, monitor).

The CLI side launches / updates the head node and copies the bootstrapped config onto it;
everything about workers (launch, setup, recovery, scale-down) is done by the head's
cluster controller.  State queries go to the head's state service.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import shlex
import subprocess
import sys
import tarfile
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, List, Optional

import yaml

from cloudtik_amd.core import constants as C
from cloudtik_amd.core import tags as T
from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.core.cluster_config import get_runtime_types, load_cluster_config
from cloudtik_amd.core.cluster_utils import (BOOTSTRAP_CONFIG_REMOTE, create_updater, get_head_node,
                                             get_worker_nodes, launch_hash, node_environment, node_tags)
from cloudtik_amd.core.executor import CallContext, ProcessRunnerError
from cloudtik_amd.core.provider_factory import get_node_provider, get_workspace_provider

logger = logging.getLogger(__name__)


class ClusterError(RuntimeError):
    pass


def _config(config_or_file, override_cluster_name=None, no_config_cache=False) -> Dict[str, Any]:
    if isinstance(config_or_file, dict):
        return config_or_file
    return load_cluster_config(config_or_file, override_cluster_name, no_config_cache=no_config_cache)


def _provider(config):
    return get_node_provider(config["provider"], config["cluster_name"], use_cache=False)


def _executor(config, provider, node_id, call_context=None):
    is_head = provider.node_tags(node_id).get(T.CLOUDTIK_TAG_NODE_KIND) == T.NODE_KIND_HEAD
    return provider.get_command_executor(
        call_context or CallContext(), f"{node_id}: ", node_id, config.get("auth", {}), config["cluster_name"],
        subprocess, not is_head or config["provider"].get("use_internal_ips", False), config.get("docker"))


def state_password(config) -> str:
    return (config.get("runtime", {}).get("state", {}) or {}).get("password") or C.CLOUDTIK_STATE_PASSWORD


def head_state_client(config):
    from cloudtik_amd.core.state.state_client import StateClient
    ip = get_head_node_ip(config)
    return StateClient.create(f"{ip}:{C.CLOUDTIK_DEFAULT_PORT}", state_password(config), timeout=5.0)


# ---------------------------------------------------------------------- create / update
def create_or_update_cluster(config_file, overrides: Optional[Dict[str, Any]] = None, no_restart: bool = False,
                             restart_only: bool = False, yes: bool = True,
                             override_cluster_name: Optional[str] = None, no_config_cache: bool = False,
                             call_context: Optional[CallContext] = None) -> Dict[str, Any]:
    if no_restart and restart_only:
        raise ValueError("--no-restart and --restart-only are mutually exclusive")
    if isinstance(config_file, dict):
        config = config_file
    else:
        config = load_cluster_config(config_file, override_cluster_name, overrides, no_config_cache)
    get_or_create_head_node(config, no_restart=no_restart, restart_only=restart_only,
                            call_context=call_context)
    _publish_services(config)
    return config


def _write_remote_config(config, provider) -> str:
    remote = copy.deepcopy(config)
    remote = provider.prepare_config_for_head(config, remote) or remote
    remote.setdefault("file_mounts", {})
    fd, path = tempfile.mkstemp(prefix="cloudtik-bootstrap-", suffix=".yaml")
    with os.fdopen(fd, "w") as f:
        yaml.safe_dump(remote, f, sort_keys=False)
    return path


def get_or_create_head_node(config: Dict[str, Any], no_restart: bool = False, restart_only: bool = False,
                            call_context: Optional[CallContext] = None) -> str:
    from cloudtik_amd.core.event_system import CreateClusterEvent as Ev, global_event_system as events
    ev = {"cluster_name": config["cluster_name"]}
    events.execute_callback(Ev.up_started, ev)
    try:
        head = _get_or_create_head_node(config, no_restart, restart_only, call_context, events, ev)
    except Exception as e:
        events.execute_callback(Ev.cluster_booting_failed, dict(ev, error=str(e)))
        raise
    events.execute_callback(Ev.cluster_booting_completed, dict(ev, node_id=head))
    return head


def _get_or_create_head_node(config, no_restart, restart_only, call_context, events, ev) -> str:
    from cloudtik_amd.core.event_system import CreateClusterEvent as Ev
    provider = _provider(config)
    head_type = config["head_node_type"]
    head = get_head_node(provider, config["cluster_name"])
    want_hash = launch_hash(config, head_type, provider)
    if head is not None and provider.node_tags(head).get(T.CLOUDTIK_TAG_LAUNCH_CONFIG) != want_hash:
        logger.info("head node %s has an outdated launch config: replacing it", head)
        _run_stop_commands(config, provider, head, is_head=True)
        provider.terminate_node(head)
        head = None
    if head is None:
        events.execute_callback(Ev.acquiring_new_head_node, ev)
        tags = node_tags(config, head_type, T.NODE_KIND_HEAD, T.CLOUDTIK_TAG_HEAD_NODE_SEQ_ID, provider)
        nt = config["available_node_types"][head_type]
        provider.create_node_with_resources(nt.get("node_config", {}), tags, 1, nt.get("resources", {}))
        deadline = time.time() + 300
        while head is None and time.time() < deadline:
            head = get_head_node(provider, config["cluster_name"])
            if head is None:
                time.sleep(1)
        if head is None:
            raise ClusterError("head node did not come up")
    head_ip = provider.internal_ip(head)
    events.execute_callback(Ev.head_node_acquired, dict(ev, node_id=head, head_ip=head_ip))
    remote_cfg = _write_remote_config(config, provider)
    try:
        updater = create_updater(config, provider, head, is_head=True, head_ip=head_ip,
                                 restart_only=restart_only and not no_restart,
                                 file_mounts={BOOTSTRAP_CONFIG_REMOTE: remote_cfg}, call_context=call_context)
        if no_restart:
            updater.start_commands = []
        stage_events = {"sync_files": Ev.ssh_control_acquired, "initialization": Ev.run_initialization_cmd,
                        "setup": Ev.run_setup_cmd, "start": Ev.start_cloudtik_runtime}
        updater.stage_callback = lambda st: st in stage_events and events.execute_callback(
            stage_events[st], dict(ev, node_id=head))
        updater.run()
    finally:
        os.unlink(remote_cfg)
    if updater.exitcode != 0:
        raise ClusterError(f"failed to set up the head node: {updater.error}")
    for t in get_runtime_types(config):
        rf.get_runtime(t, config["runtime"].get(t, {}) or {}).cluster_booting_completed(config, head)
    return head


def _publish_services(config):
    """Register the cluster's runtime services as workspace global variables (reference
    cluster_operator._publish_runtime_services / service discovery)."""
    from cloudtik_amd.core import service_discovery as sd
    try:
        wp = get_workspace_provider(config["provider"], config.get("workspace_name", "default"))
    except Exception:  # noqa: BLE001 -- providers without a workspace provider
        return
    head_ip = get_head_node_ip(config)
    worker_ips = None
    gv = {}
    for t in get_runtime_types(config):
        rt = rf.get_runtime(t, config["runtime"].get(t, {}) or {})
        for name, svc in (rt.get_runtime_services(config) or {}).items():
            if svc.get("scope") == sd.SERVICE_SCOPE_LOCAL:
                continue                      # cluster-internal: not visible to the workspace
            hosts = None
            if svc.get("node_kind") in (sd.SERVICE_DISCOVERY_NODE_KIND_WORKER, sd.SERVICE_DISCOVERY_NODE_KIND_NODE):
                if worker_ips is None:
                    worker_ips = get_worker_node_ips(config)
                hosts = ([head_ip] if svc["node_kind"] == sd.SERVICE_DISCOVERY_NODE_KIND_NODE else []) + worker_ips
            gv[sd.service_global_key(config["cluster_name"], name)] = sd.encode_service_address(svc, head_ip, hosts)
    if gv:
        wp.publish_global_variables(config, gv)


# ---------------------------------------------------------------------- teardown
def _run_stop_commands(config, provider, node_id, is_head):
    from cloudtik_amd.core.cluster_config import merged_commands_for
    ex = _executor(config, provider, node_id)
    env = node_environment(config, provider, node_id, get_head_node_ip(config, provider, missing_ok=True), is_head)
    env[C.CLOUDTIK_RUNTIME_ENV_NODE_IP] = provider.internal_ip(node_id) or ""
    for cmd in merged_commands_for(config, is_head, "stop"):
        try:
            ex.run(cmd, environment_variables=env)
        except (ProcessRunnerError, OSError) as e:
            logger.warning("%s: stop command failed: %s", node_id, e)


def teardown_cluster(config_file, workers_only: bool = False, keep_min_workers: bool = False,
                     override_cluster_name: Optional[str] = None, hard: bool = False,
                     deep: bool = False) -> None:
    config = _config(config_file, override_cluster_name)
    provider = _provider(config)
    # stop the controller first so it does not relaunch the workers we terminate
    head = get_head_node(provider, config["cluster_name"])
    if head is not None and not workers_only and not hard:
        try:
            _executor(config, provider, head).run(
                _cli_cmd(config, "node stop --controller-only"), environment_variables=node_environment(
                    config, provider, head, None, True))
        except (ProcessRunnerError, OSError) as e:
            logger.warning("could not stop the controller: %s", e)
    workers = get_worker_nodes(provider, config["cluster_name"])
    if keep_min_workers:
        keep = {}
        for n in list(workers):
            nt = provider.node_tags(n).get(T.CLOUDTIK_TAG_USER_NODE_TYPE)
            mn = config["available_node_types"].get(nt, {}).get("min_workers", 0)
            if keep.get(nt, 0) < mn:
                keep[nt] = keep.get(nt, 0) + 1
                workers.remove(n)
    if not hard:
        with ThreadPoolExecutor(max_workers=max(1, min(C.MAX_PARALLEL_SHUTDOWN_WORKERS, len(workers) or 1))) as ex:
            list(ex.map(lambda n: _run_stop_commands(config, provider, n, False), workers))
    if workers:
        provider.terminate_nodes(workers)
    if workers_only:
        return
    if head is not None:
        if not hard:
            _run_stop_commands(config, provider, head, True)
        provider.terminate_node(head)
    provider.cleanup_cluster(config, deep=deep)
    try:
        get_workspace_provider(config["provider"], config.get("workspace_name", "default")).unpublish_cluster(
            config["cluster_name"])
    except Exception:  # noqa: BLE001
        pass


def _cli_cmd(config, args: str) -> str:
    return f"cloudtik {args}"


# ---------------------------------------------------------------------- node queries
def get_head_node_ip(config, provider=None, missing_ok: bool = False) -> Optional[str]:
    provider = provider or _provider(config)
    head = get_head_node(provider, config["cluster_name"])
    if head is None:
        if missing_ok:
            return None
        raise ClusterError(f"cluster {config['cluster_name']} has no running head node")
    if config["provider"].get("use_internal_ips"):
        return provider.internal_ip(head)
    return provider.external_ip(head) or provider.internal_ip(head)


def get_worker_node_ips(config, runtime: Optional[str] = None, node_status: Optional[str] = None) -> List[str]:
    provider = _provider(config)
    out = []
    for n in get_worker_nodes(provider, config["cluster_name"]):
        if node_status and provider.node_tags(n).get(T.CLOUDTIK_TAG_NODE_STATUS) != node_status:
            continue
        out.append(provider.internal_ip(n))
    return out


def _node_by_ip(config, provider, node_ip: Optional[str]) -> str:
    if node_ip is None:
        head = get_head_node(provider, config["cluster_name"])
        if head is None:
            raise ClusterError("cluster has no head node")
        return head
    for n in provider.non_terminated_nodes({T.CLOUDTIK_TAG_CLUSTER_NAME: config["cluster_name"]}):
        if node_ip in (provider.internal_ip(n), provider.external_ip(n)):
            return n
    raise ClusterError(f"no node with IP {node_ip} in cluster {config['cluster_name']}")


def get_cluster_nodes_info(config) -> List[Dict[str, Any]]:
    provider = _provider(config)
    out = []
    for n in provider.non_terminated_nodes({T.CLOUDTIK_TAG_CLUSTER_NAME: config["cluster_name"]}):
        info = provider.get_node_info(n)
        tags = provider.node_tags(n)
        info.update({"node_ip": provider.internal_ip(n), "node_type": tags.get(T.CLOUDTIK_TAG_USER_NODE_TYPE),
                     "node_kind": tags.get(T.CLOUDTIK_TAG_NODE_KIND),
                     "node_status": tags.get(T.CLOUDTIK_TAG_NODE_STATUS)})
        out.append(info)
    return sorted(out, key=lambda i: (i["node_kind"] != T.NODE_KIND_HEAD, int(i.get(T.CLOUDTIK_TAG_NODE_SEQ_ID) or 0)))


def get_cluster_info(config) -> Dict[str, Any]:
    nodes = get_cluster_nodes_info(config)
    head = [n for n in nodes if n["node_kind"] == T.NODE_KIND_HEAD]
    workers = [n for n in nodes if n["node_kind"] == T.NODE_KIND_WORKER]
    ready = [n for n in workers if n["node_status"] == T.STATUS_UP_TO_DATE]
    total = {}
    for n in ready + [h for h in head if h["node_status"] == T.STATUS_UP_TO_DATE]:
        for k, v in (config["available_node_types"].get(n["node_type"], {}).get("resources") or {}).items():
            if isinstance(v, (int, float)):
                total[k] = total.get(k, 0) + v
    status = C.CLOUDTIK_CLUSTER_STATUS_STOPPED
    if head:
        status = C.CLOUDTIK_CLUSTER_STATUS_RUNNING if head[0]["node_status"] == T.STATUS_UP_TO_DATE \
            else C.CLOUDTIK_CLUSTER_STATUS_UNHEALTHY
    endpoints = {}
    if head:
        for t in get_runtime_types(config):
            rt = rf.get_runtime(t, config["runtime"].get(t, {}) or {})
            endpoints.update(rt.get_runtime_endpoints(config, head[0]["node_ip"]) or {})
    return {"cluster_name": config["cluster_name"], "status": status,
            "head_ip": head[0]["node_ip"] if head else None, "head_status": head[0]["node_status"] if head else None,
            "total_workers": len(workers), "total_workers_ready": len(ready),
            "workers_by_status": {s: len([w for w in workers if w["node_status"] == s])
                                  for s in sorted({w["node_status"] for w in workers})},
            "resources": total, "runtimes": get_runtime_types(config), "endpoints": endpoints,
            "nodes": nodes}


def get_scaling_status(config) -> Optional[Dict[str, Any]]:
    from cloudtik_amd.core.head.scaler import KEY_SCALING_STATUS, SCALING_NAMESPACE
    try:
        v = head_state_client(config).kv_get(KEY_SCALING_STATUS, namespace=SCALING_NAMESPACE)
    except (ConnectionError, OSError, ClusterError):
        return None
    return json.loads(v) if v else None


# ---------------------------------------------------------------------- exec / rsync
def exec_cluster(config_file, cmd: str, node_ip: Optional[str] = None, all_nodes: bool = False,
                 with_output: bool = False, run_env: str = "auto", start: bool = False,
                 override_cluster_name: Optional[str] = None, env: Optional[Dict[str, Any]] = None):
    config = _config(config_file, override_cluster_name)
    if start:
        create_or_update_cluster(config, restart_only=False)
    provider = _provider(config)
    head_ip = get_head_node_ip(config, provider)
    nodes = provider.non_terminated_nodes({T.CLOUDTIK_TAG_CLUSTER_NAME: config["cluster_name"]}) if all_nodes \
        else [_node_by_ip(config, provider, node_ip)]

    def run(n):
        is_head = provider.node_tags(n).get(T.CLOUDTIK_TAG_NODE_KIND) == T.NODE_KIND_HEAD
        e = node_environment(config, provider, n, head_ip, is_head)
        e[C.CLOUDTIK_RUNTIME_ENV_NODE_IP] = provider.internal_ip(n) or ""
        e.update(env or {})
        c = cmd
        return _executor(config, provider, n).run(c, environment_variables=e, with_output=with_output,
                                                   run_env=run_env)

    if len(nodes) == 1:
        return run(nodes[0])
    with ThreadPoolExecutor(max_workers=min(C.MAX_PARALLEL_EXEC_NODES, len(nodes))) as ex:
        return list(ex.map(run, nodes))


def rsync(config_file, source: str, target: str, down: bool, node_ip: Optional[str] = None,
          all_workers: bool = False, override_cluster_name: Optional[str] = None):
    config = _config(config_file, override_cluster_name)
    provider = _provider(config)
    if all_workers:
        nodes = get_worker_nodes(provider, config["cluster_name"])
    else:
        nodes = [_node_by_ip(config, provider, node_ip)]
    for n in nodes:
        ex = _executor(config, provider, n)
        if down:
            ex.run_rsync_down(source, target)
        else:
            ex.run_rsync_up(source, target)


def attach_cluster(config_file, node_ip: Optional[str] = None, override_cluster_name: Optional[str] = None):
    config = _config(config_file, override_cluster_name)
    provider = _provider(config)
    n = _node_by_ip(config, provider, node_ip)
    ex = _executor(config, provider, n, CallContext(allow_interactive=True))
    shell = ex.remote_shell_command_str().strip()
    home = getattr(ex, "home", None)
    if home:
        shell = f"cd {shlex.quote(home)} && HOME={shlex.quote(home)} {shell}"
    return subprocess.call(["bash", "-c", shell])


RUNNERS = {".py": "python3", ".sh": "bash", ".scala": "spark-shell -i", ".sql": "spark-sql -f",
           ".ipynb": "jupyter nbconvert --execute --to notebook"}


def submit_and_exec(config_file, script: str, script_args: Optional[List[str]] = None,
                    node_ip: Optional[str] = None, job_waiter: Optional[str] = None,
                    override_cluster_name: Optional[str] = None, with_output: bool = False,
                    runtime_options: Optional[List[str]] = None):
    """Upload a local script (or reference a URL / remote path) to the head's job dir and
    run it there with the interpreter for its extension."""
    config = _config(config_file, override_cluster_name)
    provider = _provider(config)
    n = _node_by_ip(config, provider, node_ip)
    target_dir = "~/user/jobs"
    name = os.path.basename(script)
    ex = _executor(config, provider, n)
    from cloudtik_amd.core.script_registry import get_registered_script
    module = None if os.path.exists(script) else get_registered_script(script)
    args = " ".join(shlex.quote(a) for a in (script_args or []))
    if module:
        # registered alias (e.g. ai.launch): run the module with the node's interpreter
        cmd = f"mkdir -p {target_dir} && cd {target_dir} && ${{CLOUDTIK_PYTHON:-python3}} -m {module} {args}".rstrip()
    else:
        if os.path.exists(script):
            ex.run(f"mkdir -p {target_dir}")
            ex.run_rsync_up(script, f"{target_dir}/{name}")
            remote = f"{target_dir}/{name}"
        elif script.startswith(("http://", "https://")):
            ex.run(f"mkdir -p {target_dir} && wget -q -O {target_dir}/{name} {shlex.quote(script)}")
            remote = f"{target_dir}/{name}"
        else:
            remote = script
        ext = os.path.splitext(name)[1]
        runner = None
        for t in get_runtime_types(config):
            rt = rf.get_runtime(t, config["runtime"].get(t, {}) or {})
            r = rt.get_runnable_command(remote, runtime_options)
            if r:
                runner = " ".join(r[:-1])
                break
        runner = runner or RUNNERS.get(ext, "")
        cmd = f"cd {target_dir} && {runner} {remote} {args}".replace("  ", " ")
    if not job_waiter:
        return exec_cluster(config, cmd, node_ip=node_ip, with_output=with_output)
    # detached job in a named session, then wait for it with the requested waiter
    from cloudtik_amd.core.job_waiter import create_job_waiter
    session = f"cloudtik-job-{int(time.time() * 1000)}"
    kind = job_waiter.split("+")[0]
    if kind == "tmux":
        launch = f"tmux new -d -s {session} {shlex.quote(cmd)}"
    elif kind == "screen":
        launch = f"screen -dmS {session} bash -c {shlex.quote(cmd)}"
    else:
        launch = (f"mkdir -p {target_dir} && nohup bash -c {shlex.quote(cmd)} > {target_dir}/{session}.log 2>&1 "
                  f"& echo $! > {target_dir}/{session}.pid")
    exec_cluster(config, launch, node_ip=node_ip)
    create_job_waiter(config, job_waiter).wait_for_completion(n, cmd, session_name=session)
    return session


# ---------------------------------------------------------------------- scaling
def scale_cluster(config_file, cpus: Optional[int] = None, gpus: Optional[int] = None,
                  workers: Optional[int] = None, worker_type: Optional[str] = None,
                  resources: Optional[Dict[str, float]] = None, up_only: bool = False,
                  override_cluster_name: Optional[str] = None) -> Dict[str, Any]:
    """Request the cluster to have at least the given capacity (cluster requests are
    bundles the head scaler packs against the cluster's total resources)."""
    from cloudtik_amd.core.head.scaler import KEY_CLUSTER_REQUESTS, SCALING_NAMESPACE
    config = _config(config_file, override_cluster_name)
    bundles: List[Dict[str, float]] = []
    if cpus:
        bundles += [{"CPU": 1.0}] * int(cpus)
    if gpus:
        bundles += [{"GPU": 1.0}] * int(gpus)
    if resources:
        bundles.append({k: float(v) for k, v in resources.items()})
    if workers:
        types = [worker_type] if worker_type else [t for t in config["available_node_types"]
                                                   if t != config["head_node_type"]]
        res = config["available_node_types"][types[0]].get("resources") or {"CPU": 1}
        bundles += [{k: float(v) for k, v in res.items() if isinstance(v, (int, float))}] * int(workers)
    client = head_state_client(config)
    if up_only:
        cur = client.kv_get(KEY_CLUSTER_REQUESTS, namespace=SCALING_NAMESPACE)
        if cur and len(json.loads(cur).get("bundles", [])) > len(bundles):
            return json.loads(cur)
    req = {"bundles": bundles, "time": time.time()}
    client.kv_put(KEY_CLUSTER_REQUESTS, json.dumps(req), namespace=SCALING_NAMESPACE)
    return req


def kill_node(config_file, node_ip: Optional[str] = None, hard: bool = False,
              override_cluster_name: Optional[str] = None) -> Optional[str]:
    config = _config(config_file, override_cluster_name)
    provider = _provider(config)
    workers = get_worker_nodes(provider, config["cluster_name"])
    if not workers:
        return None
    n = _node_by_ip(config, provider, node_ip) if node_ip else workers[0]
    if not hard:
        _run_stop_commands(config, provider, n, False)
    provider.terminate_node(n)
    return provider.internal_ip(n)


def wait_for_ready(config_file, min_workers: Optional[int] = None, timeout: float = C.CLOUDTIK_WAIT_FOR_CLUSTER_READY_TIMEOUT_S,
                   interval: float = C.CLOUDTIK_WAIT_FOR_CLUSTER_READY_INTERVAL_S,
                   override_cluster_name: Optional[str] = None) -> int:
    config = _config(config_file, override_cluster_name)
    if min_workers is None:
        min_workers = sum(nt.get("min_workers", 0) for t, nt in config["available_node_types"].items()
                          if t != config["head_node_type"])
    deadline = time.time() + timeout
    while True:
        ready = len(get_worker_node_ips(config, node_status=T.STATUS_UP_TO_DATE))
        if ready >= min_workers:
            return ready
        if time.time() > deadline:
            raise TimeoutError(f"only {ready}/{min_workers} workers ready after {timeout}s")
        time.sleep(interval)


# ---------------------------------------------------------------------- health / metrics / dump
def cluster_process_status(config) -> Dict[str, Any]:
    from cloudtik_amd.core.state.state_client import NODE_PROCESSES_TABLE
    return head_state_client(config).table_get_all(NODE_PROCESSES_TABLE)


def cluster_resource_metrics(config) -> Dict[str, Any]:
    from cloudtik_amd.core.state.state_client import NODE_METRICS_TABLE
    return head_state_client(config).table_get_all(NODE_METRICS_TABLE)


def health_check(config, with_details: bool = False) -> Dict[str, Any]:
    """Head daemons alive, every up-to-date node heart-beating, no node failed."""
    from cloudtik_amd.core.state.state_client import NODE_PROCESSES_TABLE, NODE_TABLE
    problems: List[str] = []
    try:
        client = head_state_client(config)
        hb = client.table_get_all(NODE_TABLE)
        procs = client.table_get_all(NODE_PROCESSES_TABLE)
    except (ConnectionError, OSError, ClusterError) as e:
        return {"healthy": False, "problems": [f"state service unreachable: {e}"]}
    now = time.time()
    info = get_cluster_info(config)
    for n in info["nodes"]:
        ip = n["node_ip"]
        nid = n["node_id"]
        beat = hb.get(nid) or hb.get(ip)
        if n["node_status"] == T.STATUS_UPDATE_FAILED:
            problems.append(f"{ip}: setup failed")
        elif n["node_status"] == T.STATUS_UP_TO_DATE:
            if beat is None:
                problems.append(f"{ip}: no heartbeat")
            elif now - beat.get("last_heartbeat_time", 0) > C.CLOUDTIK_HEARTBEAT_TIMEOUT_S:
                problems.append(f"{ip}: heartbeat lost {now - beat['last_heartbeat_time']:.0f}s ago")
        p = (procs.get(nid) or procs.get(ip) or {}).get("processes", {})
        for name, st in p.items():
            if not st.get("alive"):
                problems.append(f"{ip}: process {name} is not running")
    out = {"healthy": not problems, "problems": problems}
    if with_details:
        out["heartbeats"] = hb
        out["processes"] = procs
    return out


def cluster_dump(config_file, output: Optional[str] = None, include_logs: bool = True,
                 override_cluster_name: Optional[str] = None, hosts: Optional[str] = None,
                 head_only: bool = False, params=None, on_head: bool = False) -> str:
    """Collect logs, debug state, pip packages, processes and GPU state of the cluster's nodes
    into one tarball (core/cluster_dump.py).  ``on_head`` (``cloudtik head cluster-dump``), or
    a head that is this very host: collect here.  Otherwise the collection runs on the head
    (``cloudtik head cluster-dump``, which reaches the workers) and its archive is copied back
    (reference cluster_operator.py dump_cluster -> get_archive_from_head_node)."""
    from cloudtik_amd.core import cluster_dump as cd
    config = _config(config_file, override_cluster_name)
    provider = _provider(config)
    params = params or cd.DumpParameters(logs=include_logs)
    head = get_head_node(provider, config["cluster_name"])
    if on_head or head is None or cd._is_local(provider.internal_ip(head) or ""):
        return cd.dump_cluster(config, provider, params, output, hosts=hosts, head_only=head_only)
    name = config["cluster_name"]
    output = os.path.expanduser(output or os.path.join(os.getcwd(), f"{name}_{time.strftime('%Y-%m-%d_%H-%M-%S')}.tar.gz"))
    remote = f"/tmp/cloudtik_cluster_dump_{name}_{os.getpid()}.tar.gz"
    cmd = ["cloudtik", "head", "cluster-dump", "--silent", "--output", remote] + params.node_flags()
    if hosts:
        cmd += ["--hosts", shlex.quote(hosts)]
    if head_only:
        cmd.append("--head-only")
    ex = _executor(config, provider, head)
    ex.run(" ".join(cmd), timeout=1800, environment_variables=node_environment(config, provider, head, None, True))
    ex.run_rsync_down(remote, output)
    try:
        ex.run(f"rm -f {shlex.quote(remote)}", timeout=60)
    except (ProcessRunnerError, OSError):
        pass
    return output


def monitor_cluster(config_file, lines: int = 100, follow: bool = False, timeout: Optional[float] = None,
                    override_cluster_name: Optional[str] = None, out=sys.stdout):
    """Print the head's controller log tail; with ``follow`` stream every node's new log
    lines from the state service's log channel."""
    from cloudtik_amd.core.state.state_client import LOG_CHANNEL
    config = _config(config_file, override_cluster_name)
    try:
        tail = exec_cluster(config, f"tail -n {int(lines)} ~/.cloudtik/session/logs/{C.PROCESS_TYPE_CLUSTER_CONTROLLER}.err "
                                    f"2>/dev/null || true", with_output=True)
        out.write(tail.decode(errors="replace") if isinstance(tail, bytes) else str(tail or ""))
    except (ProcessRunnerError, OSError):
        pass
    if not follow:
        return
    ps = head_state_client(config).subscribe(LOG_CHANNEL)
    end = time.time() + timeout if timeout else None
    try:
        while end is None or time.time() < end:
            m = ps.get_message(1.0)
            if m is None:
                continue
            data = json.loads(m[1])
            for fn, line in data.get("lines", []):
                out.write(f"({data.get('ip')}:{fn}) {line}\n")
            out.flush()
    finally:
        ps.close()


# ---------------------------------------------------------------------- built-in scripts / runtime services
def get_cluster_metrics(config) -> Dict[str, Any]:
    """Per-node resource metrics rows (alias of cluster_resource_metrics for the head CLI)."""
    return cluster_resource_metrics(config)


def _builtin_script_command(script: str, args: List[str]) -> str:
    """A registered alias -> ``python -m module``; ``<runtime>/<file>.sh|.py`` -> the script
    shipped in that runtime package on the node; anything else is not built in."""
    from cloudtik_amd.core.script_registry import get_registered_script
    qargs = " ".join(shlex.quote(a) for a in args)
    module = get_registered_script(script)
    if module:
        return f"${{CLOUDTIK_PYTHON:-python3}} -m {module} {qargs}".rstrip()
    parts = script.split("/")
    if len(parts) == 2 and parts[1].endswith((".sh", ".py")):
        rt, name = parts
        here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "runtime", rt)
        for sub in ("scripts", ""):
            if os.path.exists(os.path.join(here, sub, name)):
                root = ("$(${CLOUDTIK_PYTHON:-python3} -c 'import cloudtik_amd, os; "
                        "print(os.path.dirname(cloudtik_amd.__file__))')")
                path = f"{root}/runtime/{rt}/{sub + '/' if sub else ''}{name}"
                runner = "bash" if name.endswith(".sh") else "${CLOUDTIK_PYTHON:-python3}"
                return f"{runner} \"{path}\" {qargs}".rstrip()
    raise ValueError(f"{script!r} is not a built-in script (a registered alias or <runtime>/<script>); "
                     f"use `cloudtik exec` or `cloudtik submit` for your own commands")


def run_script(config_file, script: str, script_args: Optional[List[str]] = None, node_ip: Optional[str] = None,
               job_waiter: Optional[str] = None, override_cluster_name: Optional[str] = None,
               with_output: bool = False):
    """``cloudtik run``: run a built-in script on the head (or a node) of the cluster
    (reference scripts.py:678 run / _run_script)."""
    config = _config(config_file, override_cluster_name)
    cmd = _builtin_script_command(script, list(script_args or []))
    if not job_waiter:
        return exec_cluster(config, cmd, node_ip=node_ip, with_output=with_output)
    from cloudtik_amd.core.job_waiter import create_job_waiter
    session = f"cloudtik-run-{int(time.time() * 1000)}"
    exec_cluster(config, f"tmux new -d -s {session} {shlex.quote(cmd)}", node_ip=node_ip)
    waiter = create_job_waiter(config, job_waiter)
    provider = _provider(config)
    return waiter.wait_for_completion(_node_by_ip(config, provider, node_ip), cmd, session)


def runtime_services(config_file, command: str, runtimes: Optional[List[str]] = None,
                     node_ip: Optional[str] = None, workers_only: bool = False,
                     override_cluster_name: Optional[str] = None):
    """Start / stop the services of (some of) the cluster's runtimes on its nodes, head first
    on start and last on stop (reference head_scripts.py:925-1036 `cloudtik head runtime`)."""
    if command not in ("start", "stop"):
        raise ValueError("command must be start or stop")
    config = _config(config_file, override_cluster_name)
    types = get_runtime_types(config)
    sel = [t for t in types if not runtimes or t in runtimes]
    unknown = set(runtimes or []) - set(types)
    if unknown:
        raise ValueError(f"runtimes {sorted(unknown)} are not configured on this cluster")
    provider = _provider(config)
    head = get_head_node(provider, config["cluster_name"])
    if node_ip:
        nodes = [_node_by_ip(config, provider, node_ip)]
    else:
        workers = get_worker_nodes(provider, config["cluster_name"])
        nodes = list(workers) if workers_only or head is None else \
            ([head] + list(workers) if command == "start" else list(workers) + [head])
    order = sel if command == "start" else list(reversed(sel))
    done = []
    for n in nodes:
        is_head = provider.node_tags(n).get(T.CLOUDTIK_TAG_NODE_KIND) == T.NODE_KIND_HEAD
        flag = " --head" if is_head else ""
        cmd = " && ".join(f"cloudtik runtime services {t} {command}{flag}" for t in order)
        if not cmd:
            continue
        exec_cluster(config, cmd, node_ip=provider.internal_ip(n))
        done.append(provider.internal_ip(n))
    return done
