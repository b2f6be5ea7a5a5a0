"""Per-node setup pipeline (reference core/_private/node/node_updater.py:41-800).

A :class:`NodeUpdater` brings one node to the configured state:

1. ``waiting-for-ssh``  -- wait until the node answers a trivial command;
2. ``syncing-files``    -- push ``file_mounts`` / ``cluster_synced_files``;
3. ``setting-up``       -- run the merged initialization, setup, bootstrap and start
   command lists (or only the start commands when the node's runtime hash tag already
   matches -- a restart -- or ``restart_only`` is requested);
4. ``up-to-date`` / ``update-failed`` + the launch/runtime hash tags.

Every command runs with the node environment (``CLOUDTIK_NODE_IP``, ``CLOUDTIK_HEAD_IP``,
``CLOUDTIK_NODE_TYPE``, ``CLOUDTIK_RUNTIMES``...) plus the runtimes' and provider's own
variables, through the provider's command executor (local shell / SSH / docker /
kubectl).  :class:`NodeUpdaterThread` runs it in the background for the scaler.
"""
from __future__ import annotations

import logging
import subprocess
import threading
import time
from typing import Any, Dict, List, Optional

from cloudtik_amd.core import constants as C
from cloudtik_amd.core import tags as T
from cloudtik_amd.core.executor import CallContext, ProcessRunnerError

logger = logging.getLogger(__name__)

READY_CHECK_INTERVAL = C.CLOUDTIK_NODE_SSH_INTERVAL_S


class NodeUpdateError(Exception):
    pass


class NodeUpdater:
    def __init__(self, node_id: str, provider_config: Dict[str, Any], provider, auth_config,
                 cluster_name: str, file_mounts: Dict[str, str],
                 initialization_commands: List[str], setup_commands: List[str],
                 bootstrap_commands: List[str], start_commands: List[str],
                 runtime_hash: Optional[str], file_mounts_contents_hash: Optional[str],
                 is_head_node: bool, node_resources: Optional[Dict[str, Any]] = None,
                 cluster_synced_files: Optional[List[str]] = None,
                 process_runner=subprocess, use_internal_ip: bool = False,
                 docker_config: Optional[Dict[str, Any]] = None, restart_only: bool = False,
                 for_recovery: bool = False, environment_variables: Optional[Dict[str, Any]] = None,
                 call_context: Optional[CallContext] = None, ready_timeout: float = None,
                 command_timeout: Optional[float] = None, shared_memory_ratio: float = 0.0):
        self.node_id = node_id
        self.provider = provider
        self.provider_config = provider_config
        self.cluster_name = cluster_name
        self.file_mounts = dict(file_mounts or {})
        self.cluster_synced_files = list(cluster_synced_files or [])
        self.initialization_commands = list(initialization_commands or [])
        self.setup_commands = list(setup_commands or [])
        self.bootstrap_commands = list(bootstrap_commands or [])
        self.start_commands = list(start_commands or [])
        self.runtime_hash = runtime_hash
        self.file_mounts_contents_hash = file_mounts_contents_hash
        self.is_head_node = is_head_node
        self.node_resources = node_resources
        self.restart_only = restart_only
        self.for_recovery = for_recovery
        self.environment_variables = dict(environment_variables or {})
        self.call_context = call_context or CallContext()
        self.ready_timeout = ready_timeout if ready_timeout is not None else C.CLOUDTIK_NODE_START_WAIT_S
        self.command_timeout = command_timeout
        self.shared_memory_ratio = shared_memory_ratio
        self.log_prefix = f"NodeUpdater: {node_id}: "
        self.executor = provider.get_command_executor(
            self.call_context, self.log_prefix, node_id, auth_config, cluster_name, process_runner,
            use_internal_ip, docker_config)
        self.exitcode = -1
        self.error: Optional[BaseException] = None
        self.update_time: Optional[float] = None
        self.stage_times: Dict[str, float] = {}

    # ------------------------------------------------------------------ driver
    def run(self):
        t0 = time.time()
        try:
            self.do_update()
        except Exception as e:  # noqa: BLE001 -- recorded in tags + exitcode
            self.error = e
            logger.error("%supdate failed: %s", self.log_prefix, e)
            try:
                self.provider.set_node_tags(self.node_id, {T.CLOUDTIK_TAG_NODE_STATUS: T.STATUS_UPDATE_FAILED})
            except Exception:  # noqa: BLE001
                pass
            self.exitcode = 1
            return
        tags = {T.CLOUDTIK_TAG_NODE_STATUS: T.STATUS_UP_TO_DATE}
        if self.runtime_hash is not None:
            tags[T.CLOUDTIK_TAG_RUNTIME_CONFIG] = self.runtime_hash
        if self.file_mounts_contents_hash is not None:
            tags[T.CLOUDTIK_TAG_FILE_MOUNTS_CONTENTS] = self.file_mounts_contents_hash
        self.provider.set_node_tags(self.node_id, tags)
        self.update_time = time.time() - t0
        self.exitcode = 0

    def _set_status(self, status: str):
        self.provider.set_node_tags(self.node_id, {T.CLOUDTIK_TAG_NODE_STATUS: status})

    stage_callback = None       # optional fn(stage_name), e.g. cluster-creation events

    def _stage(self, name):
        self.stage_times[name] = time.time()
        if self.stage_callback is not None:
            self.stage_callback(name)

    # ------------------------------------------------------------------ stages
    def wait_ready(self, deadline: float):
        while time.time() < deadline:
            if self.provider.is_terminated(self.node_id):
                raise NodeUpdateError("node terminated while waiting for it to become ready")
            try:
                self.executor.run("uptime >/dev/null 2>&1 || true", timeout=10, silent=True)
                return
            except (ProcessRunnerError, OSError, subprocess.SubprocessError) as e:
                logger.debug("%snot ready yet: %s", self.log_prefix, e)
                time.sleep(READY_CHECK_INTERVAL)
        raise NodeUpdateError("timed out waiting for the node to become ready")

    def sync_file_mounts(self):
        for remote, local in self.file_mounts.items():
            self.executor.run_rsync_up(local, remote)
        for path in self.cluster_synced_files:
            self.executor.run_rsync_up(path, path)

    def get_update_environment_variables(self) -> Dict[str, Any]:
        tags = self.provider.node_tags(self.node_id)
        env = {
            C.CLOUDTIK_RUNTIME_ENV_CLUSTER: self.cluster_name,
            C.CLOUDTIK_RUNTIME_ENV_NODE_ID: self.node_id,
            C.CLOUDTIK_RUNTIME_ENV_NODE_IP: self.provider.internal_ip(self.node_id) or "",
            C.CLOUDTIK_RUNTIME_ENV_NODE_TYPE: tags.get(T.CLOUDTIK_TAG_USER_NODE_TYPE, ""),
            C.CLOUDTIK_RUNTIME_ENV_NODE_SEQ_ID: tags.get(T.CLOUDTIK_TAG_NODE_SEQ_ID, ""),
            C.CLOUDTIK_RUNTIME_ENV_PROVIDER_TYPE: self.provider_config.get("type", ""),
            "CLOUDTIK_HEAD": "true" if self.is_head_node else "false",
        }
        if self.node_resources:
            env["CLOUDTIK_NODE_RESOURCES"] = self.node_resources
        env.update(self.environment_variables)
        return env

    def do_update(self):
        self._stage("wait_ready")
        self._set_status(T.STATUS_WAITING_FOR_SSH)
        self.wait_ready(time.time() + self.ready_timeout)

        tags = self.provider.node_tags(self.node_id)
        runtime_unchanged = (self.runtime_hash is not None
                             and tags.get(T.CLOUDTIK_TAG_RUNTIME_CONFIG) == self.runtime_hash)
        if runtime_unchanged:
            # a node resumed from the stopped-node cache keeps its runtime hash, but its
            # container is gone: a container (re)start invalidates the hash, so the
            # initialization and setup commands run again inside the new container
            # (reference node_updater.py:456-466)
            if self.executor.run_init(as_head=self.is_head_node, file_mounts=self.file_mounts,
                                      shared_memory_ratio=self.shared_memory_ratio, sync_run_yet=False):
                runtime_unchanged = False
                self.restart_only = False
        mounts_unchanged = (self.file_mounts_contents_hash is None
                            or tags.get(T.CLOUDTIK_TAG_FILE_MOUNTS_CONTENTS) == self.file_mounts_contents_hash)
        env = self.get_update_environment_variables()

        if runtime_unchanged and mounts_unchanged and not self.for_recovery:
            # Nothing changed: only restart the services when asked to
            if self.restart_only:
                self._set_status(T.STATUS_SETTING_UP)
                self.exec_commands("start", self.start_commands, env)
            return

        self._stage("data_disks")
        self._set_status(T.STATUS_BOOTSTRAPPING_DATA_DISKS)
        self.executor.bootstrap_data_disks()
        self._stage("sync_files")
        self._set_status(T.STATUS_SYNCING_FILES)
        self.sync_file_mounts()
        if runtime_unchanged and not self.for_recovery and not self.restart_only:
            return  # only file contents changed
        self._set_status(T.STATUS_SETTING_UP)
        if not runtime_unchanged or self.for_recovery:
            # a changed runtime hash always re-runs the initialization commands and starts the
            # container (after the files are synced); restart_only drops only the setup /
            # bootstrap commands (reference node_updater.py:467-537)
            self._stage("initialization")
            self.exec_commands("initialization", self.initialization_commands, env)
            self.executor.run_init(as_head=self.is_head_node, file_mounts=self.file_mounts,
                                   shared_memory_ratio=self.shared_memory_ratio, sync_run_yet=True)
            if not self.restart_only or self.for_recovery:
                self._stage("setup")
                self.exec_commands("setup", self.setup_commands, env)
                self._stage("bootstrap")
                self.exec_commands("bootstrap", self.bootstrap_commands, env)
        self._stage("start")
        self.exec_commands("start", self.start_commands, env)

    def exec_commands(self, action: str, commands: List[str], env: Dict[str, Any]):
        for cmd in commands:
            logger.info("%s[%s] %s", self.log_prefix, action, cmd)

            try:
                self.executor.run(cmd, environment_variables=env, timeout=self.command_timeout,
                                  run_env="auto")
            except ProcessRunnerError as e:
                raise NodeUpdateError(f"{action} command failed (exit {e.code}): {cmd}") from e


class NodeUpdaterThread(NodeUpdater, threading.Thread):
    def __init__(self, *args, **kwargs):
        NodeUpdater.__init__(self, *args, **kwargs)
        threading.Thread.__init__(self, name=f"updater-{self.node_id}", daemon=True)
