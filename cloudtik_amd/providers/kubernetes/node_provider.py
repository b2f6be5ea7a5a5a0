"""Kubernetes provider: pods are nodes (reference providers/_private/_kubernetes/
node_provider.py + kubectl executor).

Implemented over the ``kubectl`` CLI (no client library needed): node tags are pod labels
(``cloudtik-*`` keys), ``create_node`` applies the node type's ``pod`` spec with the tags
as labels and AMD GPUs requested as ``amd.com/gpu`` (the ROCm k8s device plugin's resource
name), commands run through ``kubectl exec`` (KubernetesCommandExecutor).

    provider:
        type: kubernetes
        namespace: cloudtik
    available_node_types:
        worker.mi355x:
            node_config:
                pod: {spec: {containers: [{name: node, image: rocm/pytorch:latest}]}}
            resources: {CPU: 64, GPU: 8}
"""
from __future__ import annotations

import copy
import json
import re
import subprocess
import uuid
from typing import Any, Dict, List, Optional

from cloudtik_amd.core import tags as T
from cloudtik_amd.core.node_provider import NodeLaunchException, NodeProvider

_LABEL_OK = re.compile(r"[^A-Za-z0-9_.-]")


def _label_value(v: str) -> str:
    v = _LABEL_OK.sub("-", str(v))[:63]
    return v.strip("-_.") or "x"


class KubernetesNodeProvider(NodeProvider):
    def __init__(self, provider_config, cluster_name, kubectl: Optional[List[str]] = None):
        super().__init__(provider_config, cluster_name)
        self.namespace = provider_config.get("namespace", "cloudtik")
        self.kubectl = kubectl or list(provider_config.get("kubectl", ["kubectl"]))

    def _k(self, *args, input_obj=None, check=True) -> str:
        cmd = self.kubectl + ["-n", self.namespace] + list(args)
        r = subprocess.run(cmd, input=json.dumps(input_obj) if input_obj is not None else None,
                           capture_output=True, text=True, timeout=120)
        if check and r.returncode != 0:
            raise RuntimeError(f"{' '.join(cmd)} failed: {r.stderr.strip()}")
        return r.stdout

    def _pods(self, selector: Dict[str, str]) -> List[Dict[str, Any]]:
        sel = ",".join(f"{k}={_label_value(v)}" for k, v in selector.items())
        out = self._k("get", "pods", "-l", sel, "-o", "json")
        return json.loads(out or "{}").get("items", [])

    def _pod(self, node_id) -> Dict[str, Any]:
        return json.loads(self._k("get", "pod", node_id, "-o", "json"))

    def non_terminated_nodes(self, tag_filters):
        sel = self.cluster_filter()
        sel.update(tag_filters)
        return [p["metadata"]["name"] for p in self._pods(sel)
                if p.get("status", {}).get("phase") in ("Pending", "Running")
                and not p["metadata"].get("deletionTimestamp")]

    def is_running(self, node_id):
        return self._pod(node_id).get("status", {}).get("phase") == "Running"

    def is_terminated(self, node_id):
        try:
            return self._pod(node_id).get("status", {}).get("phase") not in ("Pending", "Running")
        except RuntimeError:
            return True

    def node_tags(self, node_id):
        p = self._pod(node_id)
        ann = p["metadata"].get("annotations", {}) or {}
        tags = {k: v for k, v in (p["metadata"].get("labels") or {}).items() if k.startswith("cloudtik")}
        # label values are sanitised; the exact values live in annotations
        tags.update({k[len("tags.cloudtik/"):]: v for k, v in ann.items() if k.startswith("tags.cloudtik/")})
        return tags

    def internal_ip(self, node_id):
        return self._pod(node_id).get("status", {}).get("podIP")

    def external_ip(self, node_id):
        return self.internal_ip(node_id)

    def create_node(self, node_config, tags, count):
        tags = dict(tags, **{T.CLOUDTIK_TAG_CLUSTER_NAME: self.cluster_name})
        created = {}
        for _ in range(count):
            pod = copy.deepcopy(node_config.get("pod") or {"spec": {"containers": [
                {"name": "node", "image": node_config.get("image", "rocm/pytorch:latest"),
                 "command": ["sleep", "infinity"]}]}})
            pod["apiVersion"], pod["kind"] = "v1", "Pod"
            md = pod.setdefault("metadata", {})
            name = f"cloudtik-{_label_value(self.cluster_name)}-{tags.get(T.CLOUDTIK_TAG_NODE_KIND, 'node')}-" \
                   f"{uuid.uuid4().hex[:6]}"
            md["name"] = name
            md.setdefault("labels", {}).update({k: _label_value(v) for k, v in tags.items()})
            md.setdefault("annotations", {}).update({f"tags.cloudtik/{k}": str(v) for k, v in tags.items()})
            gpus = node_config.get("gpus") or (node_config.get("resources") or {}).get("GPU")
            if gpus:
                for c in pod["spec"]["containers"][:1]:
                    c.setdefault("resources", {}).setdefault("limits", {})["amd.com/gpu"] = int(gpus)
            if tags.get(T.CLOUDTIK_TAG_NODE_KIND) == T.NODE_KIND_HEAD:
                spec = pod.setdefault("spec", {})
                spec.setdefault("serviceAccountName", self.provider_config.get(
                    "head_service_account", "cloudtik-head-service-account"))
                self._ensure_cluster_services()
            else:
                pod.setdefault("spec", {}).setdefault("serviceAccountName", self.provider_config.get(
                    "worker_service_account", "cloudtik-worker-service-account"))
            if self.provider_config.get("cloud_provider", {}).get("type") == "azure":
                md["labels"]["azure.workload.identity/use"] = "true"
            try:
                self._k("apply", "-f", "-", input_obj=pod)
            except RuntimeError as e:
                raise NodeLaunchException("KubernetesApplyFailed", str(e))
            created[name] = pod
        return created

    def _ensure_cluster_services(self):
        """Head / external head / headless node services of this cluster (workspace.py
        ``cluster_services``), applied once per head launch (apply is idempotent)."""
        from cloudtik_amd.providers.kubernetes.workspace import cluster_services
        for svc in cluster_services(self.namespace, self.cluster_name, self.provider_config.get("head_ports") or {},
                                    bool(self.provider_config.get("use_external_head_service"))):
            self._k("apply", "-f", "-", input_obj=svc)

    def set_node_tags(self, node_id, tags):
        self._k("label", "pod", node_id, "--overwrite", *[f"{k}={_label_value(v)}" for k, v in tags.items()])
        self._k("annotate", "pod", node_id, "--overwrite", *[f"tags.cloudtik/{k}={v}" for k, v in tags.items()])

    def terminate_node(self, node_id):
        self._k("delete", "pod", node_id, "--wait=false", check=False)

    def get_command_executor(self, call_context, log_prefix, node_id, auth_config, cluster_name, process_runner,
                             use_internal_ip, docker_config=None):
        from cloudtik_amd.core.executor import KubernetesCommandExecutor
        ex = KubernetesCommandExecutor(call_context, log_prefix, self.namespace, node_id, auth_config, process_runner)
        ex.kubectl = list(self.kubectl)
        return ex
