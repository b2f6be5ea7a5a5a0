"""In-memory provider + process runner for unit tests (reference tests use a MockProvider
and MockProcessRunner the same way): nodes get fake IPs, commands are
recorded instead of executed, and launch / command failures can be injected."""
from __future__ import annotations

import threading
from typing import Any, Dict, List, Optional

from cloudtik_amd.core.executor import CommandExecutor, ProcessRunnerError
from cloudtik_amd.core.node_provider import NodeLaunchException, NodeProvider


class MockProcessRunner:
    """Records commands; ``fail_cmds`` substrings make a command fail; ``respond_to_call``
    gives canned outputs to commands that capture output (reference test_cloudtik.py:91-205)."""

    def __init__(self, fail_cmds: Optional[List[str]] = None):
        self.calls: List[str] = []
        self.fail_cmds = list(fail_cmds or [])
        self.lock = threading.Lock()
        self.responses: Dict[str, List[str]] = {}

    def respond_to_call(self, pattern: str, outputs: List[str]):
        """The next commands containing ``pattern`` that capture output get ``outputs`` in order
        (the last one repeats)."""
        self.responses[pattern] = list(outputs)

    def output_for(self, cmd: str) -> bytes:
        with self.lock:
            for pat, outs in self.responses.items():
                if pat in cmd and outs:
                    return (outs.pop(0) if len(outs) > 1 else outs[0]).encode()
        return b""

    def clear_history(self):
        with self.lock:
            self.calls.clear()

    def record(self, node_id: str, cmd: str):
        with self.lock:
            self.calls.append(f"{node_id}: {cmd}")
        for f in self.fail_cmds:
            if f in cmd:
                raise ProcessRunnerError("injected failure", "cmd_failed", code=1, command=cmd)

    def commands_for(self, node_id: str) -> List[str]:
        return [c.split(": ", 1)[1] for c in self.calls if c.startswith(f"{node_id}: ")]


class MockCommandExecutor(CommandExecutor):
    def __init__(self, call_context, node_id: str, runner: MockProcessRunner):
        super().__init__(call_context)
        self.node_id, self.runner = node_id, runner

    def run(self, cmd=None, timeout=120, exit_on_fail=False, port_forward=None, with_output=False,
            environment_variables=None, run_env="auto", ssh_options_override_ssh_key="",
            shutdown_after_run=False, cmd_to_print=None, silent=False):
        if cmd:
            self.runner.record(self.node_id, cmd)
        return self.runner.output_for(cmd or "") if with_output else None

    def run_rsync_up(self, source, target, options=None):
        self.runner.record(self.node_id, f"rsync-up {source} {target}")

    def run_rsync_down(self, source, target, options=None):
        self.runner.record(self.node_id, f"rsync-down {source} {target}")


class MockProvider(NodeProvider):
    # shared across instances keyed by cluster so the scaler and the test see one world
    _worlds: Dict[str, Dict[str, Any]] = {}

    def __init__(self, provider_config, cluster_name):
        super().__init__(provider_config, cluster_name)
        w = MockProvider._worlds.setdefault(cluster_name, {"nodes": {}, "next": 0, "lock": threading.RLock(),
                                                           "runner": MockProcessRunner(), "fail_launch": set()})
        self.world = w
        # stop instead of terminate, reuse stopped nodes on launch (the reference MockProvider's
        # cache_stopped, test_cloudtik.py:207)
        self.cache_stopped = bool(provider_config.get("cache_stopped_nodes", False))

    @classmethod
    def reset(cls, cluster_name: Optional[str] = None):
        if cluster_name is None:
            cls._worlds.clear()
        else:
            cls._worlds.pop(cluster_name, None)

    def workspace_head_nodes(self, workspace_name):
        from cloudtik_amd.core import tags as T
        out = {}
        for cname, w in sorted(MockProvider._worlds.items()):
            with w["lock"]:
                for nid, n in w["nodes"].items():
                    t = n["tags"]
                    if n["state"] not in ("terminated", "stopped") and t.get(T.CLOUDTIK_TAG_NODE_KIND) == "head" \
                            and t.get(T.CLOUDTIK_TAG_WORKSPACE_NAME) == workspace_name:
                        out[f"{cname}/{nid}"] = dict(t)
        return out

    @property
    def runner(self) -> MockProcessRunner:
        return self.world["runner"]

    def fail_launches_of(self, instance_type: str):
        self.world["fail_launch"].add(instance_type)

    # ------------------------------------------------------------------ NodeProvider
    def non_terminated_nodes(self, tag_filters):
        with self.world["lock"]:
            return sorted((nid for nid, n in self.world["nodes"].items()
                           if n["state"] not in ("terminated", "stopped")
                           and all(n["tags"].get(k) == v for k, v in tag_filters.items())),
                          key=lambda x: int(x.split("-")[-1]))

    def is_running(self, node_id):
        return self.world["nodes"].get(node_id, {}).get("state") == "running"

    def is_terminated(self, node_id):
        return self.world["nodes"].get(node_id, {}).get("state", "terminated") in ("terminated", "stopped")

    def node_tags(self, node_id):
        return dict(self.world["nodes"].get(node_id, {}).get("tags", {}))

    def internal_ip(self, node_id):
        n = self.world["nodes"].get(node_id)
        return n["ip"] if n else None

    def external_ip(self, node_id):
        return self.internal_ip(node_id)

    def create_node(self, node_config, tags, count):
        itype = node_config.get("instance_type", "mock")
        if itype in self.world["fail_launch"]:
            raise NodeLaunchException("InsufficientCapacity", f"no capacity for {itype}")
        out = {}
        with self.world["lock"]:
            if self.cache_stopped:
                from cloudtik_amd.core import tags as T
                keys = (T.CLOUDTIK_TAG_NODE_KIND, T.CLOUDTIK_TAG_LAUNCH_CONFIG, T.CLOUDTIK_TAG_USER_NODE_TYPE)
                for nid in sorted(self.world["nodes"], key=lambda x: int(x.split("-")[-1])):
                    n = self.world["nodes"][nid]
                    if count <= 0:
                        break
                    if n["state"] == "stopped" and all(n["tags"].get(k) == tags.get(k) for k in keys):
                        n["state"] = "running"
                        n["tags"].update(tags)
                        out[nid] = n
                        count -= 1
            for _ in range(count):
                i = self.world["next"]
                self.world["next"] += 1
                nid = f"mock-{i}"
                self.world["nodes"][nid] = {"state": "running", "tags": dict(tags), "ip": f"10.9.{i // 250}.{i % 250 + 1}",
                                            "instance_type": itype}
                out[nid] = self.world["nodes"][nid]
        return out

    def set_node_tags(self, node_id, tags):
        with self.world["lock"]:
            self.world["nodes"][node_id]["tags"].update(tags)

    def terminate_node(self, node_id):
        with self.world["lock"]:
            if node_id in self.world["nodes"]:
                self.world["nodes"][node_id]["state"] = "stopped" if self.cache_stopped else "terminated"

    def get_command_executor(self, call_context, log_prefix, node_id, auth_config, cluster_name, process_runner,
                             use_internal_ip, docker_config=None):
        host = MockCommandExecutor(call_context, node_id, self.runner)
        if docker_config and docker_config.get("enabled") and (
                docker_config.get("image") or docker_config.get("head_image") or docker_config.get("worker_image")):
            from cloudtik_amd.core.executor import DockerCommandExecutor
            return DockerCommandExecutor(call_context, host, docker_config, cluster_name)
        return host
