"""Generic service daemons and periodic pull jobs (reference
core/_private/util/service/{service_runner,pull_job,service_daemon,cloudtik_service_daemon}.py,
SURVEY.md §2.8).

A runtime that needs a small long-running helper (sync a config from the state service,
refresh service-discovery records, pull a model registry, ...) declares either

* a ``ServiceRunner`` subclass (``run()`` loops until ``stop_event`` is set), or
* a pull script, run every ``interval`` seconds by ``ScriptPullJob``,

and starts it with ``cloudtik node service-daemon start <id> --service-class mod.Class``
(or ``--pull-script path``).  The daemon is an ordinary CloudTik process: pid file, logs in
the session directory, terminated exactly by ``service-daemon stop <id>``.

``PullJob`` logs a failing pull once, counts identical repeats (one summary line every
30 minutes) and logs the recovery -- the same noise control as the reference.
"""
from __future__ import annotations

import argparse
import importlib
import json
import logging
import os
import signal
import subprocess
import sys
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

logger = logging.getLogger(__name__)

DEFAULT_PULL_INTERVAL = 10
LOG_ERROR_REPEAT_SECONDS = 30 * 60


class ServiceRunner:
    def __init__(self):
        self.stop_event: Optional[threading.Event] = None

    def run(self):
        pass


class PullJob(ServiceRunner):
    def __init__(self, interval: Optional[float] = None):
        super().__init__()
        self.interval = interval or DEFAULT_PULL_INTERVAL
        self.errors = 0
        self.pulls = 0

    def pull(self):
        pass

    def run_once(self, state: Dict[str, Any]):
        repeat = max(1, int(LOG_ERROR_REPEAT_SECONDS // self.interval))
        try:
            self.pull()
            self.pulls += 1
            if state.get("last") is not None:
                if state["count"] >= repeat:
                    logger.info("recovered after %d repeated errors", state["count"])
                state["last"] = None
                state["count"] = 0
        except Exception as e:  # noqa: BLE001 - a pull job never dies on a bad pull
            self.errors += 1
            msg = str(e)
            if state.get("last") != msg:
                logger.exception("pull failed: %s", msg)
                state["last"], state["count"] = msg, 1
            else:
                state["count"] += 1
                if state["count"] % repeat == 0:
                    logger.error("pull failed %d times: %s", state["count"], msg)

    def run(self):
        state: Dict[str, Any] = {"last": None, "count": 0}
        while not (self.stop_event and self.stop_event.is_set()):
            self.run_once(state)
            if self.stop_event is not None:
                if self.stop_event.wait(self.interval):
                    break
            else:
                time.sleep(self.interval)


class ScriptPullJob(PullJob):
    """Runs ``pull_script`` (``.py`` with this interpreter, ``.sh`` with bash, anything else
    directly) every interval with the service arguments."""

    def __init__(self, interval=None, pull_script: str = None, service_args: Optional[List[str]] = None):
        super().__init__(interval)
        self.pull_script = pull_script
        self.service_args = list(service_args or [])

    def command(self) -> List[str]:
        s = self.pull_script
        if s.endswith(".py"):
            return [sys.executable, s, *self.service_args]
        if s.endswith(".sh"):
            return ["bash", s, *self.service_args]
        return [s, *self.service_args]

    def pull(self):
        subprocess.run(self.command(), check=True)


def cmd_args_to_call_args(cmd_args: Optional[List[str]]) -> Tuple[List[Any], Dict[str, Any]]:
    """``["a", "k=1", 'j={"x": 2}']`` -> (["a"], {"k": 1, "j": {"x": 2}}) (JSON-decoded when possible)."""
    args: List[Any] = []
    kwargs: Dict[str, Any] = {}
    for a in cmd_args or []:
        key, value = a.split("=", 1) if "=" in a else (None, a)
        try:
            value = json.loads(value)
        except ValueError:
            pass
        if key:
            kwargs[key] = value
        else:
            args.append(value)
    return args, kwargs


def load_class(path: str):
    mod, _, name = path.rpartition(".")
    return getattr(importlib.import_module(mod), name)


def create_runner(service_class: Optional[str], pull_script: Optional[str], interval: Optional[float],
                  service_args: Optional[List[str]]) -> ServiceRunner:
    if service_class:
        args, kwargs = cmd_args_to_call_args(service_args)
        if interval and issubclass(load_class(service_class), PullJob):
            kwargs.setdefault("interval", interval)
        return load_class(service_class)(*args, **kwargs)
    if pull_script:
        return ScriptPullJob(interval, pull_script, service_args)
    raise ValueError("a service class or a pull script is required")


def _process_name(identifier: str) -> str:
    return f"service-{identifier}"


def start_service_daemon(identifier: str, service_class: Optional[str] = None, pull_script: Optional[str] = None,
                         interval: Optional[float] = None, service_args: Optional[List[str]] = None) -> int:
    from cloudtik_amd.core import services
    if not identifier:
        raise ValueError("identifier cannot be empty")
    if not service_class and not pull_script:
        raise ValueError("a service class or a pull script is required")
    argv = [sys.executable, "-m", "cloudtik_amd.core.service_daemon", "--identifier", identifier]
    if service_class:
        argv += ["--service-class", service_class]
    if pull_script:
        argv += ["--pull-script", os.path.abspath(pull_script)]
    if interval:
        argv += ["--interval", str(interval)]
    argv += ["--", *(service_args or [])]
    return services.start_process(_process_name(identifier), argv)


def stop_service_daemon(identifier: str) -> bool:
    from cloudtik_amd.core import services
    return services.stop_process(_process_name(identifier))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="cloudtik-service-daemon")
    ap.add_argument("--identifier", required=True)
    ap.add_argument("--service-class", default=None)
    ap.add_argument("--pull-script", default=None)
    ap.add_argument("--interval", type=float, default=None)
    ap.add_argument("service_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    args = [x for x in a.service_args if x != "--"]
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s " + a.identifier + ": %(message)s")
    runner = create_runner(a.service_class, a.pull_script, a.interval, args)
    stop = threading.Event()
    runner.stop_event = stop
    for s in (signal.SIGTERM, signal.SIGINT):
        signal.signal(s, lambda *_: stop.set())
    try:
        runner.run()
    except Exception:  # noqa: BLE001
        logger.exception("service %s failed", a.identifier)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
