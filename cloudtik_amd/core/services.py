"""Start / stop the per-node CloudTik daemons (reference core/_private/services.py:
start_redis / start_cluster_controller / start_node_monitor / start_log_monitor and
node.py's process bookkeeping).

Every daemon is a child process in its own session with its output in
``<session>/logs/<name>.{out,err}``; its pid is recorded in ``<session>/pids/<name>.pid``
so ``cloudtik node stop`` terminates exactly the processes this node started (never by
name pattern).  The session directory is ``$CLOUDTIK_SESSION_DIR`` or
``~/.cloudtik/session``.

Debug / profiling wrappers (reference services.py:246-339), keyed by the process name in
upper case (``STATE_SERVER``, ``CONTROLLER``, ``NODE_MONITOR``, ...):

* ``CLOUDTIK_<PROC>_VALGRIND=1``            valgrind memcheck (leak check, error exit code)
* ``CLOUDTIK_<PROC>_VALGRIND_PROFILER=1``   valgrind callgrind
* ``CLOUDTIK_<PROC>_PERFTOOLS_PROFILER=1``  gperftools CPU profiler (``LD_PRELOAD=$PERFTOOLS_PATH``,
  ``CPUPROFILE=<logs>/<name>.prof``)
* ``CLOUDTIK_<PROC>_GDB=1``                 run under gdb inside a detached tmux session
* ``CLOUDTIK_<PROC>_TMUX=1``                run inside a detached tmux session
* ``CLOUDTIK_JEMALLOC_PATH`` (+ ``CLOUDTIK_JEMALLOC_CONF``, ``CLOUDTIK_JEMALLOC_PROFILE=<proc>``)
  preload jemalloc (with heap profiling for the named process)

``fate_share=True`` makes the child die with its parent (``PR_SET_PDEATHSIG``).
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time
from typing import Dict, List, Optional

from cloudtik_amd.core import constants as C


def session_dir() -> str:
    d = os.environ.get("CLOUDTIK_SESSION_DIR") or os.path.join(os.path.expanduser("~"), ".cloudtik", "session")
    for sub in ("logs", "pids"):
        os.makedirs(os.path.join(d, sub), exist_ok=True)
    return d


def logs_dir() -> str:
    return os.path.join(session_dir(), "logs")


def _pid_file(name: str) -> str:
    return os.path.join(session_dir(), "pids", f"{name}.pid")


def _package_root() -> str:
    return os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _child_env() -> Dict[str, str]:
    env = dict(os.environ)
    root = _package_root()
    pp = env.get("PYTHONPATH", "")
    if root not in pp.split(os.pathsep):
        env["PYTHONPATH"] = root + (os.pathsep + pp if pp else "")
    return env


def pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    # a zombie child still answers kill(0); treat it as dead
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return True


def _flag(name: str, what: str, environ=None) -> bool:
    environ = os.environ if environ is None else environ
    return environ.get(f"CLOUDTIK_{name.upper().replace('-', '_')}_{what}", "0") not in ("", "0", "false")


def wrap_command(name: str, argv: List[str], env: Dict[str, str]) -> List[str]:
    """Apply the debug/profiling wrapper requested for process ``name`` (see module doc).
    Mutates ``env`` (preloads, profiler output) and returns the argv to execute."""
    import shutil

    def need(tool):
        path = shutil.which(tool)
        if path is None:
            raise RuntimeError(f"{name}: a {tool} wrapper was requested but {tool} is not installed")
        return path

    jemalloc = env.get("CLOUDTIK_JEMALLOC_PATH")
    if jemalloc:
        env["LD_PRELOAD"] = (jemalloc + " " + env.get("LD_PRELOAD", "")).strip()
        conf = env.get("CLOUDTIK_JEMALLOC_CONF", "")
        if env.get("CLOUDTIK_JEMALLOC_PROFILE") == name:
            conf = ",".join(x for x in (conf, f"prof:true,prof_prefix:{os.path.join(logs_dir(), name)}") if x)
        if conf:
            env["MALLOC_CONF"] = conf
    if _flag(name, "VALGRIND", env):
        argv = [need("valgrind"), "--leak-check=full", "--show-leak-kinds=definite", "--error-exitcode=1",
                f"--log-file={os.path.join(logs_dir(), name)}.valgrind.%p"] + argv
    elif _flag(name, "VALGRIND_PROFILER", env):
        argv = [need("valgrind"), "--tool=callgrind",
                f"--callgrind-out-file={os.path.join(logs_dir(), name)}.callgrind.%p"] + argv
    elif _flag(name, "PERFTOOLS_PROFILER", env):
        lib = env.get("PERFTOOLS_PATH")
        if not lib:
            raise RuntimeError(f"{name}: PERFTOOLS_PROFILER needs PERFTOOLS_PATH (libprofiler.so)")
        env["LD_PRELOAD"] = (lib + " " + env.get("LD_PRELOAD", "")).strip()
        env["CPUPROFILE"] = os.path.join(logs_dir(), f"{name}.prof")
    if _flag(name, "GDB", env):
        argv = [need("gdb"), "-ex", "run", "--args"] + argv
    if _flag(name, "GDB", env) or _flag(name, "TMUX", env):
        import shlex
        argv = [need("tmux"), "new-session", "-d", "-s", f"cloudtik_{name}",
                " ".join(shlex.quote(a) for a in argv)]
    return argv


def _pdeathsig():
    try:
        import ctypes
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)   # PR_SET_PDEATHSIG
    except OSError:
        pass


def start_process(name: str, argv: List[str], env: Optional[Dict[str, str]] = None,
                  fate_share: bool = False) -> int:
    existing = read_pid(name)
    if existing and pid_alive(existing):
        return existing
    out = open(os.path.join(logs_dir(), f"{name}.out"), "ab")
    err = open(os.path.join(logs_dir(), f"{name}.err"), "ab")
    e = _child_env()
    if env:
        e.update(env)
    argv = wrap_command(name, list(argv), e)
    p = subprocess.Popen(argv, stdout=out, stderr=err, stdin=subprocess.DEVNULL, env=e,
                         start_new_session=True, cwd=session_dir(),
                         preexec_fn=_pdeathsig if fate_share else None)
    with open(_pid_file(name), "w") as f:
        json.dump({"pid": p.pid, "argv": argv, "started": time.time()}, f)
    return p.pid


def read_pid(name: str) -> Optional[int]:
    try:
        with open(_pid_file(name)) as f:
            return int(json.load(f)["pid"])
    except (OSError, ValueError, KeyError):
        return None


def list_processes() -> Dict[str, Dict]:
    out = {}
    d = os.path.join(session_dir(), "pids")
    for fn in sorted(os.listdir(d)):
        if not fn.endswith(".pid"):
            continue
        name = fn[:-4]
        try:
            with open(os.path.join(d, fn)) as f:
                info = json.load(f)
        except (OSError, ValueError):
            continue
        info["alive"] = pid_alive(int(info["pid"]))
        out[name] = info
    return out


def stop_process(name: str, timeout: float = 10.0) -> bool:
    pid = read_pid(name)
    if pid is None:
        return False
    stopped = False
    if pid_alive(pid):
        try:
            os.killpg(pid, signal.SIGTERM)   # the daemon leads its own session/process group
        except (ProcessLookupError, PermissionError):
            try:
                os.kill(pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        deadline = time.time() + timeout
        while time.time() < deadline and pid_alive(pid):
            time.sleep(0.05)
        if pid_alive(pid):
            try:
                os.killpg(pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
        stopped = True
    try:
        os.remove(_pid_file(name))
    except OSError:
        pass
    return stopped


def stop_all() -> List[str]:
    # controller first (it may be launching nodes), state server last
    order = [C.PROCESS_TYPE_CLUSTER_CONTROLLER, C.PROCESS_TYPE_LOG_MONITOR, C.PROCESS_TYPE_NODE_MONITOR]
    names = list(list_processes())
    stopped = []
    for n in order + [n for n in names if n not in order and n != C.PROCESS_TYPE_STATE_SERVER] + \
            [C.PROCESS_TYPE_STATE_SERVER]:
        if n in names and stop_process(n):
            stopped.append(n)
    return stopped


# ------------------------------------------------------------------ daemons
def start_state_server(node_ip: str, port: int, password: Optional[str]) -> int:
    from cloudtik_amd.native.build import state_server_path
    data = os.path.join(session_dir(), "state")
    os.makedirs(data, exist_ok=True)
    argv = [state_server_path(), "--port", str(port), "--bind", "0.0.0.0" if node_ip in ("", None) else node_ip,
            "--dir", data, "--save-interval", "60"]
    if password:
        argv += ["--requirepass", password]
    pid = start_process(C.PROCESS_TYPE_STATE_SERVER, argv)
    from cloudtik_amd.core.state.state_client import StateClient
    addr = f"{node_ip or '127.0.0.1'}:{port}"
    deadline = time.time() + 15
    while time.time() < deadline:
        try:
            if StateClient.create(addr, password, timeout=1.0).ping():
                return pid
        except ConnectionError:
            time.sleep(0.1)
    raise RuntimeError(f"state server did not come up on {addr}")


def start_node_monitor(address: str, node_ip: str, head: bool, password: Optional[str],
                       resources: Optional[str] = None) -> int:
    argv = [sys.executable, "-m", "cloudtik_amd.core.node.monitor", "--address", address,
            "--node-ip", node_ip, "--logs-dir", logs_dir()]
    if head:
        argv.append("--head")
    if resources:
        argv += ["--resources", resources]
    env = {"CLOUDTIK_STATE_PASSWORD": password or ""}
    return start_process(C.PROCESS_TYPE_NODE_MONITOR, argv, env)


def start_cluster_controller(address: str, config_file: str, password: Optional[str]) -> int:
    argv = [sys.executable, "-m", "cloudtik_amd.core.head.controller", "--address", address,
            "--config", config_file]
    env = {"CLOUDTIK_STATE_PASSWORD": password or ""}
    return start_process(C.PROCESS_TYPE_CLUSTER_CONTROLLER, argv, env)
