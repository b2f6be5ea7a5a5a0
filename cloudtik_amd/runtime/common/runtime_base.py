"""RuntimeBase: a Runtime whose defaults / commands come from YAML next to its module, and
whose node-side steps (install / configure / services) are declared as shell step lists.

Reference behaviour (runtime/common/runtime_base.py:12-35 + per-runtime scripts/*.sh):
``cloudtik runtime install|configure|services <rt>`` runs the runtime's step on a node,
with the runtime's environment exported; config files are rendered from ``conf/``
templates by ``{%placeholder%}`` substitution.
"""
from __future__ import annotations

import copy
import inspect
import os
import subprocess
from typing import Any, Dict, List, Optional

import yaml

from cloudtik_amd.core.runtime import Runtime
from cloudtik_amd.core.config.merge import merge_config

RUNTIME_PATH_ENV = "RUNTIME_PATH"


def runtime_path() -> str:
    return os.environ.get(RUNTIME_PATH_ENV, os.path.join(os.path.expanduser("~"), "runtime"))


def standard_commands(name: str) -> Dict[str, Any]:
    """The command hooks every node-installed runtime contributes (reference
    runtime/*/config/commands.yaml)."""
    return {
        "head_setup_commands": [f"cloudtik runtime install {name} --head",
                                f"cloudtik runtime configure {name} --head"],
        "worker_setup_commands": [f"cloudtik runtime install {name}",
                                  f"cloudtik runtime configure {name}"],
        "head_start_commands": [f"cloudtik runtime services {name} stop --head",
                                f"cloudtik runtime services {name} start --head"],
        "worker_start_commands": [f"cloudtik runtime services {name} stop",
                                  f"cloudtik runtime services {name} start"],
        "head_stop_commands": [f"cloudtik runtime services {name} stop --head"],
        "worker_stop_commands": [f"cloudtik runtime services {name} stop"],
    }


def render_template(text: str, values: Dict[str, Any]) -> str:
    for k, v in values.items():
        text = text.replace("{%" + k + "%}", str(v))
    return text


def render_conf_file(src: str, dst: str, values: Dict[str, Any]):
    with open(src) as f:
        text = f.read()
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst, "w") as f:
        f.write(render_template(text, values))


class RuntimeBase(Runtime):
    name: str = ""

    def _home(self) -> str:
        return os.path.dirname(inspect.getfile(self.__class__))

    def _config_object(self, cluster_config: Dict[str, Any], object_name: str) -> Dict[str, Any]:
        root = os.path.join(self._home(), "config")
        out: Dict[str, Any] = {}
        base = os.path.join(root, f"{object_name}.yaml")
        if os.path.exists(base):
            with open(base) as f:
                out = yaml.safe_load(f) or {}
        ptype = (cluster_config or {}).get("provider", {}).get("type")
        if ptype:
            p = os.path.join(root, ptype, f"{object_name}.yaml")
            if os.path.exists(p):
                with open(p) as f:
                    out = merge_config(out, yaml.safe_load(f) or {})
        return out

    def get_runtime_commands(self, cluster_config):
        cmds = self._config_object(cluster_config, "commands")
        return cmds or standard_commands(self.name)

    def get_defaults_config(self, cluster_config):
        return self._config_object(cluster_config, "defaults")

    # ------------------------------------------------------------ node-side steps
    def node_env(self, head: bool) -> Dict[str, str]:
        env = dict(os.environ)
        env.setdefault(RUNTIME_PATH_ENV, runtime_path())
        env["IS_HEAD_NODE"] = "true" if head else "false"
        # node variables are exported verbatim (never shell-expanded); resolve the runtime
        # home references like MLFLOW_HOME=$RUNTIME_PATH/mlflow here, as plain strings
        rp = env[RUNTIME_PATH_ENV]
        for k, v in list(env.items()):
            if "$RUNTIME_PATH" in v:
                env[k] = v.replace("${RUNTIME_PATH}", rp).replace("$RUNTIME_PATH", rp)
        return env

    def node_install(self, head: bool):
        return self._run_steps(self.install_steps(head), head)

    def node_configure(self, head: bool):
        return self._run_steps(self.configure_steps(head), head)

    def node_services(self, command: str, head: bool):
        steps = self.start_steps(head) if command == "start" else self.stop_steps(head)
        return self._run_steps(steps, head, ignore_errors=(command == "stop"))

    def install_steps(self, head: bool) -> List[str]:
        return []

    def configure_steps(self, head: bool) -> List[str]:
        return []

    def start_steps(self, head: bool) -> List[str]:
        return []

    def stop_steps(self, head: bool) -> List[str]:
        return []

    def _run_steps(self, steps: List[str], head: bool, ignore_errors: bool = False):
        env = self.node_env(head)
        for s in steps:
            r = subprocess.run(["bash", "-c", s], env=env)
            if r.returncode != 0 and not ignore_errors:
                raise RuntimeError(f"runtime {self.name}: step failed ({r.returncode}): {s}")
        return True

    def runtime_config_section(self, cluster_config) -> Dict[str, Any]:
        return copy.deepcopy(cluster_config.get("runtime", {}).get(self.name, {}) or {})
