"""AI runtime cluster API (reference runtime/ai/api.py:9-37): ``AICluster`` / ``ThisAICluster``
add the runtime's endpoints (MLflow tracking server) and a job launcher that runs a script
with ``cloudtik-run`` on the head (one process per GPU of every node in ``hosts``)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional

from cloudtik_amd.core.api import Cluster, ThisCluster


class _AIOps:
    def get_endpoints(self) -> Dict[str, Any]:
        return self.get_runtime_endpoints()

    def get_mlflow_uri(self) -> Optional[str]:
        ep = self.get_endpoints().get("mlflow")
        return ep.get("url") if ep else None

    def run_distributed(self, script: str, args: Optional[List[str]] = None, all_nodes: bool = True,
                        nproc_per_node: int = 0, with_output: bool = False):
        """``cloudtik-run`` the script over the head + ready workers (one rank per GPU)."""
        import shlex
        hosts = [self.get_head_node_ip()] + (self.get_worker_node_ips(node_status="up-to-date") if all_nodes else [])
        cmd = ["cloudtik-run", "--hosts", ",".join(hosts)]
        if nproc_per_node:
            cmd += ["--nproc-per-node", str(nproc_per_node)]
        cmd += [script] + list(args or [])
        return self.exec(" ".join(shlex.quote(c) for c in cmd), with_output=with_output)


class AICluster(_AIOps, Cluster):
    pass


class ThisAICluster(_AIOps, ThisCluster):
    pass
