"""Kubernetes workspaces, with EKS / GKE / AKS cloud integration (reference
providers/_private/_kubernetes/config.py workspace half, aws_eks/config.py, gcp_gke/config.py,
azure_aks/config.py).

A Kubernetes workspace is a namespace with the head / worker service accounts and the head's
role + role binding (pods, exec, services, config maps -- what the head needs to launch and
drive worker pods).  When the cluster runs on a managed Kubernetes (``provider.cloud_provider:
{type: aws|gcp|azure, ...}``) the workspace also gives the pods a cloud identity through the
cloud's workload-identity mechanism, so runtimes reach the cloud storage without keys:

* **EKS** (IRSA): an IAM OIDC identity provider for the cluster's issuer, one IAM role per
  service account trusting ``system:serviceaccount:<ns>:<sa>`` through it (+ S3 policy), and
  the service accounts annotated ``eks.amazonaws.com/role-arn``;
* **GKE** (Workload Identity): one Google service account per Kubernetes service account
  with the storage role, ``roles/iam.workloadIdentityUser`` granted on it to
  ``<project>.svc.id.goog[<ns>/<sa>]``, and the Kubernetes accounts annotated
  ``iam.gke.io/gcp-service-account``;
* **AKS** (Azure AD workload identity): one user-assigned managed identity per service
  account with a federated credential for the AKS OIDC issuer + subject, the Storage Blob
  Data Owner role, and the service accounts annotated ``azure.workload.identity/client-id``.

Managed cloud storage (the bucket / ADLS container of the cloud workspace) is added as an
optional step when ``managed_cloud_storage`` is set.  Everything is a ``Step`` run by the
same ``WorkspaceBuilder`` as the cloud workspaces (idempotent create, reverse delete,
NOT_EXIST / IN_COMPLETED / COMPLETED).  Kubernetes is driven through ``kubectl`` (no client
library), the clouds through the same boto3 / REST transports as providers/cloud.

``cluster_services`` gives the per-cluster head service (ClusterIP, the runtimes' head
ports), the optional external head service (LoadBalancer) and the headless node service the
node provider applies when it launches a head pod.
"""
from __future__ import annotations

import json
import subprocess
from typing import Any, Callable, Dict, List, Optional, Tuple

from cloudtik_amd.providers.cloud.workspace import Step, _missing

HEAD_SA = "cloudtik-head-service-account"
WORKER_SA = "cloudtik-worker-service-account"
HEAD_ROLE = "cloudtik-head-role"
HEAD_ROLE_BINDING = "cloudtik-head-role-binding"
HEAD_RULES = [
    {"apiGroups": [""], "resources": ["pods", "pods/status", "pods/exec", "pods/log", "services", "configmaps",
                                      "secrets", "persistentvolumeclaims", "events"],
     "verbs": ["get", "watch", "list", "create", "update", "patch", "delete"]},
]


class KubectlError(RuntimeError):
    def __init__(self, msg: str, not_found: bool = False):
        super().__init__(msg)
        self.not_found = not_found


Runner = Callable[[List[str], Optional[str]], Tuple[int, str, str]]


def _subprocess_runner(cmd: List[str], stdin: Optional[str]) -> Tuple[int, str, str]:
    r = subprocess.run(cmd, input=stdin, capture_output=True, text=True, timeout=120)
    return r.returncode, r.stdout, r.stderr


class Kubectl:
    def __init__(self, kubectl: Optional[List[str]] = None, runner: Optional[Runner] = None):
        self.base = list(kubectl or ["kubectl"])
        self.runner = runner or _subprocess_runner

    def run(self, *args, input_obj=None) -> str:
        cmd = self.base + list(args)
        rc, out, err = self.runner(cmd, json.dumps(input_obj) if input_obj is not None else None)
        if rc != 0:
            raise KubectlError(f"{' '.join(cmd)}: {err.strip()}", not_found="NotFound" in err or "not found" in err)
        return out

    def get(self, kind: str, name: str, namespace: Optional[str] = None) -> Optional[Dict[str, Any]]:
        try:
            out = self.run(*(["-n", namespace] if namespace else []), "get", kind, name, "-o", "json")
        except KubectlError as e:
            if e.not_found:
                return None
            raise
        return json.loads(out)

    def apply(self, obj: Dict[str, Any]):
        ns = obj.get("metadata", {}).get("namespace")
        self.run(*(["-n", ns] if ns else []), "apply", "-f", "-", input_obj=obj)

    def delete(self, kind: str, name: str, namespace: Optional[str] = None):
        self.run(*(["-n", namespace] if namespace else []), "delete", kind, name, "--ignore-not-found=true")

    def annotate(self, kind: str, name: str, namespace: str, annotations: Dict[str, Optional[str]]):
        args = [f"{k}={v}" if v is not None else f"{k}-" for k, v in annotations.items()]
        self.run("-n", namespace, "annotate", kind, name, "--overwrite", *args)


def _obj(kind: str, name: str, namespace: Optional[str] = None, api: str = "v1", **body) -> Dict[str, Any]:
    md = {"name": name, "labels": {"cloudtik-workspace-managed": "true"}}
    if namespace:
        md["namespace"] = namespace
    return dict({"apiVersion": api, "kind": kind, "metadata": md}, **body)


class KubernetesWorkspace:
    def __init__(self, provider_config: Dict[str, Any], workspace_name: str, kubectl: Optional[Kubectl] = None,
                 cloud_transport=None):
        self.cfg = provider_config
        self.ws = workspace_name
        self.namespace = provider_config.get("namespace") or f"cloudtik-{workspace_name}"
        self.k = kubectl or Kubectl(provider_config.get("kubectl"))
        self.sa = {"head": provider_config.get("head_service_account", HEAD_SA),
                   "worker": provider_config.get("worker_service_account", WORKER_SA)}
        cp = provider_config.get("cloud_provider") or {}
        self.cloud = None
        if cp.get("type") == "aws":
            self.cloud = EKSIntegration(cp, self, cloud_transport)
        elif cp.get("type") == "gcp":
            self.cloud = GKEIntegration(cp, self, cloud_transport)
        elif cp.get("type") == "azure":
            self.cloud = AKSIntegration(cp, self, cloud_transport)

    def _exists(self, kind: str, name: str, namespaced: bool = True) -> bool:
        return self.k.get(kind, name, self.namespace if namespaced else None) is not None

    def _k8s_step(self, label: str, obj: Dict[str, Any]) -> Step:
        kind, name = obj["kind"], obj["metadata"]["name"]
        ns = obj["metadata"].get("namespace")
        return Step(label, lambda: self._exists(kind, name, ns is not None), lambda: self.k.apply(obj),
                    lambda: self.k.delete(kind, name, ns))

    def steps(self, config: Dict[str, Any]) -> List[Step]:
        ns = self.namespace
        out = [
            self._k8s_step("namespace", _obj("Namespace", ns)),
            self._k8s_step("head service account", _obj("ServiceAccount", self.sa["head"], ns)),
            self._k8s_step("worker service account", _obj("ServiceAccount", self.sa["worker"], ns)),
            self._k8s_step("head role", _obj("Role", HEAD_ROLE, ns, "rbac.authorization.k8s.io/v1", rules=HEAD_RULES)),
            self._k8s_step("head role binding", _obj(
                "RoleBinding", HEAD_ROLE_BINDING, ns, "rbac.authorization.k8s.io/v1",
                subjects=[{"kind": "ServiceAccount", "name": self.sa["head"], "namespace": ns}],
                roleRef={"kind": "Role", "name": HEAD_ROLE, "apiGroup": "rbac.authorization.k8s.io"})),
        ]
        if self.cloud is not None:
            out += self.cloud.steps(config)
        return out

    def info(self) -> Dict[str, Any]:
        info = {"namespace": self.namespace, "service_accounts": dict(self.sa)}
        if self.cloud is not None:
            info["cloud"] = self.cloud.info()
        return info

    # ------------------------------------------------------------------ service accounts
    def sa_annotated(self, role: str, key: str, value: Optional[str] = None) -> bool:
        sa = self.k.get("serviceaccount", self.sa[role], self.namespace) or {}
        v = (sa.get("metadata", {}).get("annotations") or {}).get(key)
        return v is not None and (value is None or v == value)

    def annotate_sa(self, role: str, annotations: Dict[str, Optional[str]]):
        self.k.annotate("serviceaccount", self.sa[role], self.namespace, annotations)

    def subject(self, role: str) -> str:
        return f"system:serviceaccount:{self.namespace}:{self.sa[role]}"


# =============================================================================== EKS
class EKSIntegration:
    ANNOTATION = "eks.amazonaws.com/role-arn"
    POLICIES = ("AmazonS3FullAccess",)
    # thumbprint of the root CA behind the regional EKS OIDC endpoints (IAM no longer checks it
    # for those issuers, but the API still requires one)
    DEFAULT_THUMBPRINT = "9e99a48a9960b14926bb7f3b02e22da2b0ab7280"

    def __init__(self, cp: Dict[str, Any], ws: KubernetesWorkspace, client_factory=None):
        self.cp, self.w = cp, ws
        if client_factory is None:
            import boto3
            client_factory = lambda svc: boto3.client(svc, region_name=cp["region"])  # noqa: E731
        self._factory = client_factory
        self.eks, self.iam = client_factory("eks"), client_factory("iam")
        self.cluster = cp["eks_cluster_name"]
        self.roles = {r: f"cloudtik-eks-{ws.ws}-{r}"[:64] for r in ("head", "worker")}
        self._issuer: Optional[str] = None

    def issuer(self) -> str:
        if self._issuer is None:
            self._issuer = self.eks.describe_cluster(name=self.cluster)["cluster"]["identity"]["oidc"]["issuer"]
        return self._issuer

    def _host(self) -> str:
        return self.issuer().replace("https://", "")

    def _provider_arn(self) -> Optional[str]:
        for p in self.iam.list_open_id_connect_providers()["OpenIDConnectProviderList"]:
            if p["Arn"].endswith(f"oidc-provider/{self._host()}"):
                return p["Arn"]
        return None

    def _create_provider(self):
        self.iam.create_open_id_connect_provider(
            Url=self.issuer(), ClientIDList=["sts.amazonaws.com"],
            ThumbprintList=[self.cp.get("oidc_thumbprint", self.DEFAULT_THUMBPRINT)],
            Tags=[{"Key": "cloudtik-workspace", "Value": self.w.ws}])

    def _role_exists(self, role: str) -> bool:
        try:
            self.iam.get_role(RoleName=self.roles[role])
            return True
        except Exception as e:  # noqa: BLE001 - botocore NoSuchEntity
            if "NoSuchEntity" in type(e).__name__ or "NoSuchEntity" in str(e):
                return False
            raise

    def _create_role(self, role: str):
        trust = {"Version": "2012-10-17", "Statement": [{
            "Effect": "Allow", "Principal": {"Federated": self._provider_arn()},
            "Action": "sts:AssumeRoleWithWebIdentity",
            "Condition": {"StringEquals": {f"{self._host()}:sub": self.w.subject(role),
                                           f"{self._host()}:aud": "sts.amazonaws.com"}}}]}
        self.iam.create_role(RoleName=self.roles[role], AssumeRolePolicyDocument=json.dumps(trust),
                             Tags=[{"Key": "cloudtik-workspace", "Value": self.w.ws}])
        for p in self.POLICIES:
            self.iam.attach_role_policy(RoleName=self.roles[role], PolicyArn=f"arn:aws:iam::aws:policy/{p}")

    def _delete_role(self, role: str):
        for p in self.POLICIES:
            self.iam.detach_role_policy(RoleName=self.roles[role], PolicyArn=f"arn:aws:iam::aws:policy/{p}")
        self.iam.delete_role(RoleName=self.roles[role])

    def _role_arn(self, role: str) -> str:
        return self.iam.get_role(RoleName=self.roles[role])["Role"]["Arn"]

    def steps(self, config) -> List[Step]:
        out = [Step("EKS OIDC identity provider", lambda: self._provider_arn() is not None, self._create_provider,
                    lambda: self.iam.delete_open_id_connect_provider(OpenIDConnectProviderArn=self._provider_arn()))]
        for role in ("head", "worker"):
            out.append(Step(f"{role} IAM role for service account", lambda r=role: self._role_exists(r),
                            lambda r=role: self._create_role(r), lambda r=role: self._delete_role(r)))
            out.append(Step(f"{role} service account role annotation",
                            lambda r=role: self.w.sa_annotated(r, self.ANNOTATION),
                            lambda r=role: self.w.annotate_sa(r, {self.ANNOTATION: self._role_arn(r)}),
                            lambda r=role: self.w.annotate_sa(r, {self.ANNOTATION: None})))
        if config.get("managed_cloud_storage"):
            from cloudtik_amd.providers.cloud.workspace import AWSWorkspace
            aws = AWSWorkspace(dict(self.cp), self.w.ws, self._factory)
            out += [s for s in aws.steps(config) if s.managed == "storage"]
        return out

    def info(self):
        return {"type": "aws", "eks_cluster": self.cluster, "roles": dict(self.roles)}


# =============================================================================== GKE
_IAM = "https://iam.googleapis.com/v1"


class GKEIntegration:
    ANNOTATION = "iam.gke.io/gcp-service-account"
    ROLES = ("roles/storage.admin",)

    def __init__(self, cp: Dict[str, Any], ws: KubernetesWorkspace, call=None):
        self.cp, self.w = cp, ws
        from cloudtik_amd.providers.cloud.workspace import GCPWorkspace
        if call is None:
            from cloudtik_amd.providers.cloud.rest_providers import GCPNodeProvider, requests_transport
            tok = GCPNodeProvider.__new__(GCPNodeProvider)
            tok.provider_config = cp
            call = requests_transport(tok._token)
        self.call = call
        self.project = cp["project_id"]
        self.gcp = GCPWorkspace(dict(cp, region=cp.get("region", "us-central1")), ws.ws, call)
        self.accounts = {r: f"cloudtik-gke-{ws.ws}-{r}"[:30].rstrip("-") for r in ("head", "worker")}

    def email(self, role: str) -> str:
        return f"{self.accounts[role]}@{self.project}.iam.gserviceaccount.com"

    def _sa_url(self, role: str) -> str:
        return f"{_IAM}/projects/{self.project}/serviceAccounts/{self.email(role)}"

    def _wi_member(self, role: str) -> str:
        return f"serviceAccount:{self.project}.svc.id.goog[{self.w.namespace}/{self.w.sa[role]}]"

    def _create_sa(self, role: str):
        self.call("POST", f"{_IAM}/projects/{self.project}/serviceAccounts", None,
                  {"accountId": self.accounts[role], "serviceAccount": {"displayName": f"CloudTik {self.w.ws} {role}"}})
        self.gcp._bind(f"serviceAccount:{self.email(role)}", self.ROLES, add=True)

    def _delete_sa(self, role: str):
        self.gcp._bind(f"serviceAccount:{self.email(role)}", self.ROLES, add=False)
        self.call("DELETE", self._sa_url(role), None, None)

    def _wi_bound(self, role: str) -> bool:
        pol = self.call("POST", self._sa_url(role) + ":getIamPolicy", None, {})
        return any(b["role"] == "roles/iam.workloadIdentityUser" and self._wi_member(role) in b["members"]
                   for b in pol.get("bindings", []))

    def _wi_bind(self, role: str, add: bool):
        pol = self.call("POST", self._sa_url(role) + ":getIamPolicy", None, {})
        bindings = pol.setdefault("bindings", [])
        b = next((x for x in bindings if x["role"] == "roles/iam.workloadIdentityUser"), None)
        member = self._wi_member(role)
        if add:
            if b is None:
                bindings.append({"role": "roles/iam.workloadIdentityUser", "members": [member]})
            elif member not in b["members"]:
                b["members"].append(member)
        elif b is not None and member in b["members"]:
            b["members"].remove(member)
        pol["bindings"] = [x for x in bindings if x["members"]]
        self.call("POST", self._sa_url(role) + ":setIamPolicy", None, {"policy": pol})

    def steps(self, config) -> List[Step]:
        out = []
        for role in ("head", "worker"):
            out += [
                Step(f"{role} Google service account",
                     lambda r=role: not _missing(lambda: self.call("GET", self._sa_url(r), None, None)),
                     lambda r=role: self._create_sa(r), lambda r=role: self._delete_sa(r)),
                Step(f"{role} workload identity binding", lambda r=role: self._wi_bound(r),
                     lambda r=role: self._wi_bind(r, True), lambda r=role: self._wi_bind(r, False)),
                Step(f"{role} service account identity annotation",
                     lambda r=role: self.w.sa_annotated(r, self.ANNOTATION, self.email(r)),
                     lambda r=role: self.w.annotate_sa(r, {self.ANNOTATION: self.email(r)}),
                     lambda r=role: self.w.annotate_sa(r, {self.ANNOTATION: None})),
            ]
        if config.get("managed_cloud_storage"):
            out += [s for s in self.gcp.steps(config) if s.managed == "storage"]
        return out

    def info(self):
        return {"type": "gcp", "service_accounts": {r: self.email(r) for r in self.accounts}}


# =============================================================================== AKS
class AKSIntegration:
    ANNOTATION = "azure.workload.identity/client-id"
    IDENTITY_API = "2023-01-31"

    def __init__(self, cp: Dict[str, Any], ws: KubernetesWorkspace, call=None):
        self.cp, self.w = cp, ws
        from cloudtik_amd.providers.cloud.workspace import ROLE_STORAGE_BLOB_OWNER, AzureWorkspace, _ARM
        if call is None:
            from cloudtik_amd.providers.cloud.rest_providers import AzureNodeProvider, requests_transport
            tok = AzureNodeProvider.__new__(AzureNodeProvider)
            tok.provider_config = cp
            call = requests_transport(tok._token)
        self.call, self.arm, self.blob_owner = call, _ARM, ROLE_STORAGE_BLOB_OWNER
        self.az = AzureWorkspace(cp, ws.ws, call)
        self.aks = cp["aks_cluster_name"]
        self.aks_rg = cp.get("aks_resource_group", self.az.rg)
        self.identities = {r: f"cloudtik-aks-{ws.ws}-{r}" for r in ("head", "worker")}

    def _id_url(self, role: str) -> str:
        return self.az._res("Microsoft.ManagedIdentity", f"userAssignedIdentities/{self.identities[role]}")

    def issuer(self) -> str:
        url = f"{self.arm}/subscriptions/{self.az.sub}/resourceGroups/{self.aks_rg}/providers/" \
              f"Microsoft.ContainerService/managedClusters/{self.aks}"
        props = self.call("GET", url, {"api-version": "2023-08-01"}, None)["properties"]
        issuer = (props.get("oidcIssuerProfile") or {}).get("issuerURL")
        if not issuer:
            raise RuntimeError(f"AKS cluster {self.aks} has no OIDC issuer: enable --enable-oidc-issuer "
                               "--enable-workload-identity")
        return issuer

    def _fic_url(self, role: str) -> str:
        return f"{self._id_url(role)}/federatedIdentityCredentials/cloudtik-{self.w.sa[role]}"

    def _create_identity(self, role: str):
        scope = f"/subscriptions/{self.az.sub}/resourceGroups/{self.az.rg}"
        self.az._put(self._id_url(role), "identity", {"location": self.az.location})
        self.az._assign(self._id_url(role), (self.blob_owner,), scope)

    def _client_id(self, role: str) -> str:
        return self.az._get(self._id_url(role), "identity")["properties"]["clientId"]

    def steps(self, config) -> List[Step]:
        out = []
        for role in ("head", "worker"):
            out += [
                Step(f"{role} managed identity",
                     lambda r=role: not _missing(lambda: self.az._get(self._id_url(r), "identity")),
                     lambda r=role: self._create_identity(r), lambda r=role: self.az._del(self._id_url(r), "identity")),
                Step(f"{role} federated identity credential",
                     lambda r=role: not _missing(lambda: self.call("GET", self._fic_url(r),
                                                                   {"api-version": self.IDENTITY_API}, None)),
                     lambda r=role: self.call("PUT", self._fic_url(r), {"api-version": self.IDENTITY_API}, {
                         "properties": {"issuer": self.issuer(), "subject": self.w.subject(r),
                                        "audiences": ["api://AzureADTokenExchange"]}}),
                     lambda r=role: self.call("DELETE", self._fic_url(r), {"api-version": self.IDENTITY_API}, None)),
                Step(f"{role} service account identity annotation",
                     lambda r=role: self.w.sa_annotated(r, self.ANNOTATION),
                     lambda r=role: self.w.annotate_sa(r, {self.ANNOTATION: self._client_id(r)}),
                     lambda r=role: self.w.annotate_sa(r, {self.ANNOTATION: None})),
            ]
        if config.get("managed_cloud_storage"):
            out += [s for s in self.az.steps(config) if s.managed == "storage"]
        return out

    def info(self):
        return {"type": "azure", "aks_cluster": self.aks, "identities": dict(self.identities)}


# =============================================================================== cluster services
def cluster_services(namespace: str, cluster_name: str, head_ports: Dict[str, Dict[str, Any]],
                     external: bool = False) -> List[Dict[str, Any]]:
    """Service manifests of one cluster: ``<cluster>-head`` (ClusterIP over the runtimes' head
    ports, selected by the head pod's labels), ``<cluster>-head-external`` (LoadBalancer, when
    ``external``) and the headless ``<cluster>-node`` service giving every pod a DNS name."""
    from cloudtik_amd.core import tags as T
    from cloudtik_amd.providers.kubernetes.node_provider import _label_value
    head_sel = {T.CLOUDTIK_TAG_CLUSTER_NAME: _label_value(cluster_name), T.CLOUDTIK_TAG_NODE_KIND: "head"}
    ports = [{"name": n[:15].lower().replace("_", "-"), "port": int(p["port"]), "targetPort": int(p["port"]),
              "protocol": "UDP" if str(p.get("protocol", "")).lower() == "udp" else "TCP"}
             for n, p in sorted(head_ports.items())]
    ports = ports or [{"name": "ssh", "port": 22, "targetPort": 22, "protocol": "TCP"}]
    out = [_obj("Service", f"{cluster_name}-head", namespace, spec={"type": "ClusterIP", "selector": head_sel,
                                                                     "ports": ports})]
    if external:
        out.append(_obj("Service", f"{cluster_name}-head-external", namespace,
                        spec={"type": "LoadBalancer", "selector": head_sel, "ports": ports}))
    out.append(_obj("Service", f"{cluster_name}-node", namespace, spec={
        "clusterIP": "None", "selector": {T.CLOUDTIK_TAG_CLUSTER_NAME: _label_value(cluster_name)},
        "ports": [{"name": "ssh", "port": 22, "targetPort": 22}]}))
    return out


__all__ = ["KubernetesWorkspace", "Kubectl", "KubectlError", "EKSIntegration", "GKEIntegration", "AKSIntegration",
           "cluster_services"]
