"""Command executors: how the control plane runs commands on (and syncs files to) nodes.

Contract: reference ``core/command_executor.py:27-186``.  Implementations:

* ``LocalCommandExecutor``  -- the node is this host (local provider head = CLI host).
* ``SSHCommandExecutor``    -- ssh with ControlMaster/ControlPersist multiplexing, optional
                               proxy command, rsync over ssh (ssh_command_executor.py:25-268).
* ``DockerCommandExecutor`` -- wraps a host executor and runs everything inside the node's
                               container.  ROCm-first: ``run_init`` starts the container with
                               ``--device=/dev/kfd --device=/dev/dri --group-add video
                               --ipc=host`` when the host has AMD GPUs (replacing the
                               reference's nvidia-container-runtime detection,
                               docker_command_executor.py:475-497), plus auto shm sizing.
* ``KubernetesCommandExecutor`` -- ``kubectl exec`` / ``kubectl cp``.

All executors route process creation through an injectable ``process_runner`` (the
``subprocess`` module by default) so tests can substitute a recording fake runner, as the
reference test-suite does with MockProcessRunner.
"""
from __future__ import annotations

import hashlib
import json
import re
import logging
import os
import shlex
import socket
import subprocess
import time
from typing import Any, Dict, List, Optional

logger = logging.getLogger(__name__)

CHECK_DOCKER_RUNTIME_NUMBER_OF_RETRIES = 5
SSH_CONTROL_PATH_MAX = 70


class CallContext:
    """Per-invocation output settings (reference core/_private/call_context.py)."""

    def __init__(self, verbosity: int = 0, output_redirected: bool = False, allow_interactive: bool = False):
        self.verbosity = verbosity
        self.output_redirected = output_redirected
        self.allow_interactive = allow_interactive

    def is_output_redirected(self):
        return self.output_redirected

    def new_call_context(self):
        return CallContext(self.verbosity, self.output_redirected, self.allow_interactive)


class ProcessRunnerError(Exception):
    def __init__(self, msg, msg_type, code=None, command=None, special_case=None):
        super().__init__(f"{msg} (type={msg_type}, code={code}, cmd={command})")
        self.msg_type = msg_type
        self.code = code
        self.command = command
        self.special_case = special_case


# environment variables whose values never appear in printed / logged commands or errors
# (reference command_executor.py:23-70 is_key_with_privacy)
_PRIVACY_KEY = re.compile(r"(PASSWORD|PASSWD|SECRET|TOKEN|CREDENTIAL|PRIVATE|ACCESS_KEY|API_KEY|AUTH|_KEY$)",
                          re.IGNORECASE)
PRIVACY_MASK = "<hidden>"


def is_key_with_privacy(key: str) -> bool:
    return bool(_PRIVACY_KEY.search(key or ""))


def with_environment_variables(cmd: str, env: Optional[Dict[str, Any]], for_print: bool = False) -> str:
    """``export K=V; ... cmd``; with ``for_print`` the values of privacy keys are masked."""
    if not env:
        return cmd
    parts = []
    for k, v in env.items():
        if not isinstance(v, str):
            v = json.dumps(v, separators=(",", ":"))
        if for_print and is_key_with_privacy(k):
            v = PRIVACY_MASK
        parts.append(f"export {k}={shlex.quote(v)};")
    if "CLOUDTIK_BIN_DIR" in env:
        # same-host nodes run this checkout's `cloudtik` / `cloudtik-run` wrappers
        parts.append('export PATH="$CLOUDTIK_BIN_DIR:$PATH";')
    return " ".join(parts) + " " + cmd


def printable_command(cmd: str, env: Optional[Dict[str, Any]], cmd_to_print: Optional[str] = None) -> str:
    return with_environment_variables(cmd_to_print or cmd, env, for_print=True)


def run_cmd_with_runner(process_runner, final_cmd, with_output=False, silent=False, timeout=None,
                        shell=False, printable=None):
    """Run ``final_cmd``; errors and debug logs carry ``printable`` (secrets masked), never
    the real command line."""
    shown = printable if printable is not None else final_cmd
    logger.debug("running: %s", shown)
    try:
        if with_output:
            return process_runner.check_output(final_cmd, shell=shell, timeout=timeout) \
                if timeout else process_runner.check_output(final_cmd, shell=shell)
        kw = {}
        if silent:
            kw["stdout"] = subprocess.DEVNULL
            kw["stderr"] = subprocess.DEVNULL
        if timeout:
            kw["timeout"] = timeout
        return process_runner.check_call(final_cmd, shell=shell, **kw)
    except subprocess.CalledProcessError as e:
        raise ProcessRunnerError("Command failed", "cmd_failed", code=e.returncode, command=shown) from None


class CommandExecutor:
    def __init__(self, call_context: CallContext = None):
        self.call_context = call_context or CallContext()

    def run(self, cmd: str = None, timeout: int = 120, exit_on_fail: bool = False,
            port_forward=None, with_output: bool = False, environment_variables=None,
            run_env: str = "auto", ssh_options_override_ssh_key: str = "",
            shutdown_after_run: bool = False, cmd_to_print: str = None, silent: bool = False):
        raise NotImplementedError

    def run_with_retry(self, cmd: str = None, timeout: int = 120, exit_on_fail=False,
                       port_forward=None, with_output=False, environment_variables=None,
                       run_env="auto", ssh_options_override_ssh_key="",
                       shutdown_after_run=False, cmd_to_print=None, silent=False,
                       number_of_retries=30, retry_interval=1):
        last = None
        for i in range(max(1, number_of_retries)):
            try:
                return self.run(cmd, timeout=timeout, exit_on_fail=exit_on_fail,
                                port_forward=port_forward, with_output=with_output,
                                environment_variables=environment_variables, run_env=run_env,
                                ssh_options_override_ssh_key=ssh_options_override_ssh_key,
                                shutdown_after_run=shutdown_after_run, cmd_to_print=cmd_to_print,
                                silent=silent)
            except Exception as e:  # noqa: BLE001
                last = e
                if i + 1 < number_of_retries:
                    time.sleep(retry_interval)
        raise last

    def run_rsync_up(self, source: str, target: str, options: Optional[Dict[str, Any]] = None):
        raise NotImplementedError

    def run_rsync_down(self, source: str, target: str, options: Optional[Dict[str, Any]] = None):
        raise NotImplementedError

    def remote_shell_command_str(self) -> str:
        return "true"

    def run_init(self, *, as_head: bool, file_mounts: Dict[str, str], shared_memory_ratio: float,
                 sync_run_yet: bool) -> Optional[bool]:
        return None

    def run_terminate(self):
        return None

    def bootstrap_data_disks(self) -> None:
        return None


# ---------------------------------------------------------------------------------- local
class LocalCommandExecutor(CommandExecutor):
    def __init__(self, call_context, log_prefix, auth_config, cluster_name, process_runner,
                 node_id=None, provider=None, use_internal_ip=True):
        super().__init__(call_context)
        self.log_prefix = log_prefix
        self.process_runner = process_runner
        self.node_id = node_id
        self.provider = provider

    def run(self, cmd=None, timeout=120, exit_on_fail=False, port_forward=None, with_output=False,
            environment_variables=None, run_env="auto", ssh_options_override_ssh_key="",
            shutdown_after_run=False, cmd_to_print=None, silent=False):
        if not cmd:
            return None
        shown = printable_command(cmd, environment_variables, cmd_to_print)
        cmd = with_environment_variables(cmd, environment_variables)
        final = ["bash", "-c", cmd]
        return run_cmd_with_runner(self.process_runner, final, with_output=with_output, silent=silent,
                                   printable=["bash", "-c", shown])

    def run_rsync_up(self, source, target, options=None):
        target = os.path.expanduser(target)
        os.makedirs(os.path.dirname(target.rstrip("/")) or ".", exist_ok=True)
        self._copy(source, target)

    def run_rsync_down(self, source, target, options=None):
        self._copy(os.path.expanduser(source), target)

    def _copy(self, source, target):
        if os.path.abspath(source.rstrip("/")) == os.path.abspath(target.rstrip("/")):
            return
        if os.path.isdir(source):
            src = source.rstrip("/") + "/."
            os.makedirs(target, exist_ok=True)
            run_cmd_with_runner(self.process_runner, ["cp", "-a", src, target])
        else:
            run_cmd_with_runner(self.process_runner, ["cp", "-a", source, target])

    def remote_shell_command_str(self):
        return "bash"


# ---------------------------------------------------------------------------------- ssh
class SSHOptions:
    def __init__(self, ssh_key, control_path=None, **kwargs):
        self.ssh_key = ssh_key
        self.arg_dict = {
            "StrictHostKeyChecking": "no",
            "UserKnownHostsFile": os.devnull,
            "IdentitiesOnly": "yes",
            "ExitOnForwardFailure": "yes",
            "ServerAliveInterval": 5,
            "ServerAliveCountMax": 3,
        }
        if control_path:
            self.arg_dict.update({"ControlMaster": "auto", "ControlPath": f"{control_path}/%C",
                                  "ControlPersist": "10s"})
        self.arg_dict.update(kwargs)

    def to_ssh_options_list(self, *, timeout=60):
        self.arg_dict["ConnectTimeout"] = f"{timeout}s"
        opts = ["-i", self.ssh_key] if self.ssh_key else []
        return opts + [x for y in (["-o", f"{k}={v}"] for k, v in self.arg_dict.items() if v is not None) for x in y]


class SSHCommandExecutor(CommandExecutor):
    def __init__(self, call_context, log_prefix, node_id, provider, auth_config, cluster_name,
                 process_runner, use_internal_ip):
        super().__init__(call_context)
        ssh_control_hash = hashlib.md5(cluster_name.encode()).hexdigest()
        ssh_user_hash = hashlib.md5(os.environ.get("USER", "user").encode()).hexdigest()
        self.ssh_control_path = f"/tmp/cloudtik_ssh_{ssh_user_hash[:10]}/{ssh_control_hash[:10]}"
        self.log_prefix = log_prefix
        self.node_id = node_id
        self.provider = provider
        self.use_internal_ip = use_internal_ip
        self.ssh_user = auth_config.get("ssh_user", "ubuntu")
        self.ssh_private_key = auth_config.get("ssh_private_key")
        self.ssh_proxy_command = auth_config.get("ssh_proxy_command")
        self.ssh_port = auth_config.get("ssh_port")
        self.process_runner = process_runner
        self.ssh_options = SSHOptions(self.ssh_private_key, self.ssh_control_path,
                                      ProxyCommand=self.ssh_proxy_command)
        self._ip = None

    def _get_node_ip(self):
        if self.use_internal_ip:
            return self.provider.internal_ip(self.node_id)
        return self.provider.external_ip(self.node_id)

    def _wait_for_ip(self, deadline=60):
        ip = self._get_node_ip()
        t0 = time.time()
        while ip is None and time.time() - t0 < deadline:
            time.sleep(2)
            ip = self._get_node_ip()
        if ip is None:
            raise RuntimeError(f"node {self.node_id} has no ip")
        return ip

    def _set_ssh_ip_if_required(self):
        if self._ip is None:
            self._ip = self._wait_for_ip()
            os.makedirs(self.ssh_control_path, mode=0o700, exist_ok=True)

    def _ssh_base(self, timeout=120):
        port = ["-p", str(self.ssh_port)] if self.ssh_port else []
        return ["ssh", "-tt" if self.call_context.allow_interactive else "-T"] + port + \
            self.ssh_options.to_ssh_options_list(timeout=timeout) + [f"{self.ssh_user}@{self._ip}"]

    def run(self, cmd=None, timeout=120, exit_on_fail=False, port_forward=None, with_output=False,
            environment_variables=None, run_env="auto", ssh_options_override_ssh_key="",
            shutdown_after_run=False, cmd_to_print=None, silent=False):
        self._set_ssh_ip_if_required()
        final = self._ssh_base(timeout)
        if port_forward:
            pf = port_forward if isinstance(port_forward, list) else [port_forward]
            for local, remote in pf:
                final += ["-L", f"{local}:localhost:{remote}"]
        shown = list(final)
        if cmd:
            printable = printable_command(cmd, environment_variables, cmd_to_print)
            cmd = with_environment_variables(cmd, environment_variables)
            if shutdown_after_run:
                cmd += "; sudo shutdown -h now"
                printable += "; sudo shutdown -h now"
            final += ["bash", "--login", "-c", "-i", shlex.quote("set -i || true; " + cmd)]
            shown += ["bash", "--login", "-c", "-i", shlex.quote("set -i || true; " + printable)]
        return run_cmd_with_runner(self.process_runner, final, with_output=with_output, silent=silent,
                                   printable=shown)

    def _rsync(self, src, dst, options):
        self._set_ssh_ip_if_required()
        ssh = " ".join(["ssh"] + self.ssh_options.to_ssh_options_list(timeout=120) +
                       (["-p", str(self.ssh_port)] if self.ssh_port else []))
        cmd = ["rsync", "--rsh", ssh, "-avz"]
        for ex in (options or {}).get("rsync_exclude", []) or []:
            cmd += ["--exclude", ex]
        for fl in (options or {}).get("rsync_filter", []) or []:
            cmd += ["--filter", f"dir-merge,- {fl}"]
        cmd += [src, dst]
        run_cmd_with_runner(self.process_runner, cmd)

    def run_rsync_up(self, source, target, options=None):
        self.run(f"mkdir -p {shlex.quote(os.path.dirname(target.rstrip('/')))}", silent=True)
        self._rsync(source, f"{self.ssh_user}@{self._ip}:{target}", options)

    def run_rsync_down(self, source, target, options=None):
        self._rsync(f"{self.ssh_user}@{self._ip}:{source}", target, options)

    def remote_shell_command_str(self):
        self._set_ssh_ip_if_required()
        key = f"-i {self.ssh_private_key} " if self.ssh_private_key else ""
        return f"ssh -o IdentitiesOnly=yes {key}{self.ssh_user}@{self._ip}\n"

    def bootstrap_data_disks(self):
        """Format and mount unmounted NVMe data disks under /mnt/cloudtik/data_disk_N."""
        script = (
            "i=1; for d in $(lsblk -dpno NAME,TYPE,MOUNTPOINT | awk '$2==\"disk\" && $3==\"\" {print $1}'); do "
            "  if ! lsblk -no MOUNTPOINT $d | grep -q .; then "
            "    (sudo blkid $d >/dev/null || sudo mkfs -t ext4 -q $d) && "
            "    sudo mkdir -p /mnt/cloudtik/data_disk_$i && sudo mount -o defaults,noatime $d /mnt/cloudtik/data_disk_$i && "
            "    sudo chmod a+w /mnt/cloudtik/data_disk_$i; i=$((i+1)); fi; done")
        self.run(script, silent=True)


# ---------------------------------------------------------------------------------- docker
# bootstrap files are copied into the container, never bind-mounted: docker bind-mounts the
# inode, so a config rewritten on the host (new file, rename) would go stale inside
BOOTSTRAP_MOUNTS = ("~/cloudtik_bootstrap_config.yaml", "~/cloudtik_bootstrap_key.pem")


def docker_host_mount_location(cluster_name: str) -> str:
    """Host directory that holds the bind-mounted file_mounts of a cluster's containers."""
    return f"/tmp/cloudtik_docker_mounts/{cluster_name}"


class DockerCommandExecutor(CommandExecutor):
    """Runs node commands inside the cluster container on a host reached by ``host_executor``
    (reference core/_private/command_executor/docker_command_executor.py, run_init :326).

    * ``run_init``: pulls the image (``pull_before_run``, default true; otherwise only when
      missing), checks a running container for drift -- a different image or file_mounts it
      does not bind-mount -- and restarts it then; a container is started only once the files
      are synced (``sync_run_yet``), with the file_mounts bind-mounted from the host mount
      location, ROCm device pass-through and /dev/shm sized from the runtime's ratio; the
      bootstrap config / key are copied in.  Returns whether a ``docker run`` was executed.
    * rsync goes to the host mount location (the bind mount makes it visible inside); paths
      that are not bind-mounted are copied into the running container.
    """

    def __init__(self, call_context, host_executor: CommandExecutor, docker_config: Dict[str, Any],
                 cluster_name: str = "default"):
        super().__init__(call_context)
        self.host = host_executor
        self.docker_config = docker_config or {}
        self.container_name = self.docker_config.get("container_name", "cloudtik-ai")
        self.docker_cmd = self.docker_config.get("docker_cmd", "docker")
        self.cluster_name = cluster_name
        self.initialized = False
        self.home_dir: Optional[str] = None
        self.bind_mounts: Dict[str, str] = {}
        self._image_homes: Dict[str, str] = {}

    # ------------------------------------------------------------------ helpers
    def _host(self, cmd, with_output=False, silent=True):
        return self.host.run(cmd, with_output=with_output, run_env="host", silent=silent)

    def image(self, as_head: bool) -> Optional[str]:
        return self.docker_config.get("head_image" if as_head else "worker_image") or self.docker_config.get("image")

    def _out(self, cmd) -> str:
        out = self._host(cmd, with_output=True)
        return out.decode() if isinstance(out, (bytes, bytearray)) else (out or "")

    def is_container_running(self) -> bool:
        out = self._out(f"{self.docker_cmd} inspect -f '{{{{.State.Running}}}}' {self.container_name} || true")
        return "true" in out.lower() and "no such object" not in out.lower()

    def image_home(self, image: str) -> str:
        """$HOME of the image's default user, read once per image BEFORE the container runs:
        ``~/`` file mounts are bind-mounted there (an image whose user is not root, e.g. the
        reference base image's /home/cloudtik, would otherwise get them under /root)."""
        if image not in self._image_homes:
            out = self._out(f"{self.docker_cmd} run --rm --entrypoint printenv {image} HOME || true")
            lines = [ln.strip() for ln in out.splitlines() if ln.strip().startswith("/")]
            self._image_homes[image] = lines[-1] if lines else "/root"
        return self._image_homes[image]

    def expand_user(self, path: str) -> str:
        if path.startswith("~"):
            if self.home_dir is None:
                self.home_dir = self._out(f"{self.docker_cmd} exec {self.container_name} printenv HOME").strip() \
                    or "/root"
            return self.home_dir + path[1:]
        return path

    @staticmethod
    def _under_home(path: str, home: str) -> str:
        if path == "~":
            return home
        if path.startswith("~/"):
            return home.rstrip("/") + "/" + path[2:]
        return path

    def host_mount_path(self, remote: str) -> str:
        return docker_host_mount_location(self.cluster_name) + "/" + remote.lstrip("~/").lstrip("/")

    def restart_needed(self, image: str, mounts: Dict[str, str]) -> bool:
        """A running container with another image or without some requested bind mounts."""
        running_image = self._out(f"{self.docker_cmd} inspect -f '{{{{.Config.Image}}}}' {self.container_name}").strip()
        if running_image and running_image != image:
            logger.warning("container %s runs image %s instead of %s: restarting it", self.container_name,
                           running_image, image)
            return True
        raw = self._out(f"{self.docker_cmd} inspect -f '{{{{json .Mounts}}}}' {self.container_name}").strip()
        try:
            active = {m["Destination"].strip("/") for m in json.loads(raw or "[]")}
        except (ValueError, KeyError, TypeError):
            return False
        # where THIS image's docker run would bind them (the same home as the -v targets)
        home = self.image_home(image) if any(r.startswith("~") for r in mounts) else None
        wanted = {self._under_home(r, home).strip("/") for r in mounts}
        missing = wanted - active
        if missing:
            logger.warning("container %s lacks file mounts %s: restarting it", self.container_name, sorted(missing))
            return True
        return False

    # ------------------------------------------------------------------ CommandExecutor
    def run(self, cmd=None, timeout=120, exit_on_fail=False, port_forward=None, with_output=False,
            environment_variables=None, run_env="auto", ssh_options_override_ssh_key="",
            shutdown_after_run=False, cmd_to_print=None, silent=False):
        if run_env == "host" or not cmd:
            return self.host.run(cmd, timeout, exit_on_fail, port_forward, with_output,
                                 environment_variables, "auto", ssh_options_override_ssh_key,
                                 shutdown_after_run, cmd_to_print, silent)
        shown = printable_command(cmd, environment_variables, cmd_to_print)
        cmd = with_environment_variables(cmd, environment_variables)
        flags = '-it' if self.call_context.allow_interactive else ''
        inner = f"{self.docker_cmd} exec {flags} {self.container_name} /bin/bash -c {shlex.quote(cmd)}"
        inner_shown = f"{self.docker_cmd} exec {flags} {self.container_name} /bin/bash -c {shlex.quote(shown)}"
        return self.host.run(inner, timeout, exit_on_fail, port_forward, with_output, None, "host",
                             ssh_options_override_ssh_key, shutdown_after_run, inner_shown, silent)

    def _bind_mounted(self, target: str) -> bool:
        t = target.rstrip("/")
        return any(t == r.rstrip("/") or t.startswith(r.rstrip("/") + "/") for r in self.bind_mounts)

    def run_rsync_up(self, source, target, options=None):
        staging = self.host_mount_path(target)
        self._host(f"mkdir -p {shlex.quote(os.path.dirname(staging.rstrip('/')))}")
        self.host.run_rsync_up(source, staging, options)
        if self.initialized and not self._bind_mounted(target) and self.is_container_running():
            dst = self.expand_user(target)
            self._host(f"{self.docker_cmd} exec {self.container_name} mkdir -p "
                       f"{shlex.quote(os.path.dirname(dst.rstrip('/')))} && "
                       f"{self.docker_cmd} cp {shlex.quote(staging)} {self.container_name}:{shlex.quote(dst)}")

    def run_rsync_down(self, source, target, options=None):
        staging = self.host_mount_path(source)
        self._host(f"mkdir -p {shlex.quote(os.path.dirname(staging.rstrip('/')))} && "
                   f"{self.docker_cmd} cp {self.container_name}:{shlex.quote(self.expand_user(source))} "
                   f"{shlex.quote(staging)}")
        self.host.run_rsync_down(staging, target, options)

    def remote_shell_command_str(self):
        return self.host.remote_shell_command_str().strip() + f" -tt -- {self.docker_cmd} exec -it {self.container_name} /bin/bash\n"

    def rocm_run_options(self, as_head: bool) -> List[str]:
        """GPU pass-through flags when the host exposes /dev/kfd (AMD ROCm); the reference's
        nvidia-container-runtime detection (docker_command_executor.py:475-497) has no role
        on MI355X."""
        if self.docker_config.get("disable_automatic_runtime_detection"):
            return []
        try:
            out = self.host.run("ls /dev/kfd /dev/dri 2>/dev/null | head -1", with_output=True, run_env="host")
            has = bool(out and out.strip())
        except Exception:  # noqa: BLE001
            has = False
        if not has:
            return []
        return ["--device=/dev/kfd", "--device=/dev/dri", "--group-add=video",
                "--cap-add=SYS_PTRACE", "--security-opt=seccomp=unconfined"]

    def shm_run_options(self, shared_memory_ratio: float) -> List[str]:
        if self.docker_config.get("disable_shm_size_detection") or shared_memory_ratio <= 0:
            return []
        try:
            out = self.host.run("cat /proc/meminfo || true", with_output=True, run_env="host").decode()
            kb = int([ln for ln in out.split("\n") if "MemAvailable" in ln][0].split()[1])
            return [f"--shm-size={int(kb * 1024 * shared_memory_ratio * 1.1)}b"]
        except Exception:  # noqa: BLE001
            return []

    def _pull(self, image: str):
        if self.docker_config.get("pull_before_run", True):
            self._host(f"{self.docker_cmd} pull {image}")
        else:
            self._host(f"{self.docker_cmd} image inspect {image} 1> /dev/null 2>&1 || {self.docker_cmd} pull {image}")

    def run_init(self, *, as_head, file_mounts, shared_memory_ratio, sync_run_yet):
        image = self.image(as_head)
        if not image:
            return None
        self._pull(image)
        mounts = {r: l for r, l in (file_mounts or {}).items() if r not in BOOTSTRAP_MOUNTS}
        self.bind_mounts = mounts
        running = self.initialized or self.is_container_running()
        restart = running and self.restart_needed(image, mounts)
        if restart:
            self._host(f"{self.docker_cmd} stop {self.container_name} > /dev/null || true")
            self.initialized = False
        docker_run = False
        if not running or restart:
            if not sync_run_yet:
                # start after the file sync: docker would create missing mount sources as root
                return True
            opts = list(self.docker_config.get("run_options", [])) + \
                list(self.docker_config.get("head_run_options" if as_head else "worker_run_options", []))
            opts += [f"--ipc={self.docker_config.get('ipc_mode') or 'host'}",
                     f"--net={self.docker_config.get('network') or 'host'}",
                     "--cap-add=NET_ADMIN", "--cap-add=SYS_NICE"]
            if self.docker_config.get("cpus"):
                opts.append(f"--cpus={self.docker_config['cpus']}")
            if self.docker_config.get("memory"):
                opts.append(f"--memory={self.docker_config['memory']}")
            opts += self.rocm_run_options(as_head) + self.shm_run_options(shared_memory_ratio)
            home = self.image_home(image) if any(r.startswith("~") for r in mounts) else None
            binds = " ".join(f"-v {shlex.quote(self.host_mount_path(r))}:{shlex.quote(self._under_home(r, home))}"
                             for r in sorted(mounts))
            labels = " ".join(f"-l {shlex.quote(f'{k}={v}')}" for k, v in
                              (self.docker_config.get("labels") or {}).items())
            self._host(f"{self.docker_cmd} run --rm --name {self.container_name} -d -it {binds} {labels} "
                       f"-e CLOUDTIK_CLUSTER_NAME={shlex.quote(self.cluster_name)} {' '.join(opts)} {image} bash")
            docker_run = True
            self.home_dir = self._image_homes.get(image)
        self.initialized = True
        # bootstrap files: copied in explicitly (see BOOTSTRAP_MOUNTS)
        for b in BOOTSTRAP_MOUNTS:
            if b in (file_mounts or {}):
                if not sync_run_yet:
                    self.host.run_rsync_up(file_mounts[b], self.host_mount_path(b))
                dst = self.expand_user(b)
                self._host(f"{self.docker_cmd} cp {shlex.quote(self.host_mount_path(b))} "
                           f"{self.container_name}:{shlex.quote(dst)}")
        return docker_run

    def run_terminate(self):
        self._host(f"{self.docker_cmd} stop {self.container_name} > /dev/null || true")
        self.initialized = False

    def bootstrap_data_disks(self):
        return self.host.bootstrap_data_disks()


# ---------------------------------------------------------------------------------- kubernetes
class KubernetesCommandExecutor(CommandExecutor):
    def __init__(self, call_context, log_prefix, namespace, node_id, auth_config, process_runner):
        super().__init__(call_context)
        self.namespace = namespace
        self.node_id = node_id
        self.process_runner = process_runner
        self.kubectl = ["kubectl"]

    def run(self, cmd=None, timeout=120, exit_on_fail=False, port_forward=None, with_output=False,
            environment_variables=None, run_env="auto", ssh_options_override_ssh_key="",
            shutdown_after_run=False, cmd_to_print=None, silent=False):
        if not cmd:
            return None
        shown = printable_command(cmd, environment_variables, cmd_to_print)
        cmd = with_environment_variables(cmd, environment_variables)
        base = self.kubectl + ["exec", "-i", "-n", self.namespace, self.node_id, "--", "bash", "-c"]
        return run_cmd_with_runner(self.process_runner, base + [cmd], with_output=with_output, silent=silent,
                                   printable=base + [shown])

    def run_rsync_up(self, source, target, options=None):
        run_cmd_with_runner(self.process_runner, self.kubectl + ["cp", source, f"{self.namespace}/{self.node_id}:{target}"])

    def run_rsync_down(self, source, target, options=None):
        run_cmd_with_runner(self.process_runner, self.kubectl + ["cp", f"{self.namespace}/{self.node_id}:{source}", target])

    def remote_shell_command_str(self):
        return f"kubectl -n {self.namespace} exec -it {self.node_id} -- bash\n"


def local_ips() -> List[str]:
    ips = {"127.0.0.1", "localhost"}
    try:
        host = socket.gethostname()
        ips.add(host)
        for a in socket.getaddrinfo(host, None):
            ips.add(a[4][0])
    except OSError:
        pass
    try:
        out = subprocess.run(["hostname", "-I"], capture_output=True, text=True, timeout=5).stdout
        ips.update(out.split())
    except Exception:  # noqa: BLE001
        pass
    return sorted(ips)


def create_default_command_executor(call_context, log_prefix, node_id, provider, auth_config,
                                    cluster_name, process_runner, use_internal_ip,
                                    docker_config=None):
    ip = provider.internal_ip(node_id) if use_internal_ip else provider.external_ip(node_id)
    if ip is not None and (ip in local_ips() or provider.provider_config.get("type") == "mock-local"):
        host = LocalCommandExecutor(call_context, log_prefix, auth_config, cluster_name, process_runner,
                                    node_id, provider, use_internal_ip)
    else:
        host = SSHCommandExecutor(call_context, log_prefix, node_id, provider, auth_config,
                                  cluster_name, process_runner, use_internal_ip)
    if docker_config and docker_config.get("enabled") and (
            docker_config.get("image") or docker_config.get("head_image") or docker_config.get("worker_image")):
        return DockerCommandExecutor(call_context, host, docker_config, cluster_name)
    return host
