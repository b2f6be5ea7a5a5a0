"""Kubernetes workspaces (providers/kubernetes/workspace.py; reference
providers/_private/_kubernetes/config.py workspace functions and aws_eks / gcp_gke / azure_aks
config.py): namespace + service accounts + RBAC through kubectl, and the EKS (IRSA), GKE
(Workload Identity) and AKS (workload identity federation) pod identities -- against a fake
kubectl and the in-memory cloud fakes of test_cloud_workspace.py."""
import json

from test_cloud_workspace import FakeARM, FakeAWS, FakeGCP, NoSuchEntityException  # noqa: F401

from cloudtik_amd.core.workspace import Existence
from cloudtik_amd.providers.cloud.workspace import WorkspaceBuilder, cloud_workspace
from cloudtik_amd.providers.kubernetes.workspace import (AKSIntegration, EKSIntegration, GKEIntegration, Kubectl,
                                                         KubernetesWorkspace, cluster_services)


class FakeKubectl:
    """kubectl get / apply / delete / annotate over an in-memory object store."""

    def __init__(self):
        self.objs = {}
        self.cmds = []

    def __call__(self, cmd, stdin):
        self.cmds.append(cmd)
        args = cmd[1:]
        ns = None
        if args[:1] == ["-n"]:
            ns, args = args[1], args[2:]
        verb = args[0]
        if verb == "apply":
            o = json.loads(stdin)
            key = (o["kind"].lower(), o["metadata"].get("namespace"), o["metadata"]["name"])
            if key[1] and ("namespace", None, key[1]) not in self.objs:
                return 1, "", f'Error from server (NotFound): namespaces "{key[1]}" not found'
            self.objs[key] = o
            return 0, "applied", ""
        kind = {"sa": "serviceaccount"}.get(args[1].lower(), args[1].lower())
        key = (kind, ns if kind != "namespace" else None, args[2])
        if verb == "get":
            if key not in self.objs:
                return 1, "", f'Error from server (NotFound): {kind} "{args[2]}" not found'
            return 0, json.dumps(self.objs[key]), ""
        if verb == "delete":
            self.objs.pop(key, None)
            if kind == "namespace":       # the namespace takes its objects with it
                for k in [k for k in self.objs if k[1] == args[2]]:
                    del self.objs[k]
            return 0, "", ""
        if verb == "annotate":
            if key not in self.objs:
                return 1, "", "NotFound"
            ann = self.objs[key]["metadata"].setdefault("annotations", {})
            for a in args[4:]:
                if a.endswith("-") and "=" not in a:
                    ann.pop(a[:-1], None)
                else:
                    k, v = a.split("=", 1)
                    ann[k] = v
            return 0, "", ""
        raise AssertionError(cmd)


def _build(ws):
    return WorkspaceBuilder(ws.steps({}), log=lambda m: None)


def test_plain_kubernetes_workspace_lifecycle():
    kc = FakeKubectl()
    ws = KubernetesWorkspace({"type": "kubernetes"}, "w1", Kubectl(runner=kc))
    b = _build(ws)
    assert b.existence() == Existence.NOT_EXIST
    b.create()
    assert b.existence() == Existence.COMPLETED
    rb = kc.objs[("rolebinding", "cloudtik-w1", "cloudtik-head-role-binding")]
    assert rb["subjects"][0]["name"] == "cloudtik-head-service-account" and rb["roleRef"]["name"] == "cloudtik-head-role"
    assert "pods/exec" in kc.objs[("role", "cloudtik-w1", "cloudtik-head-role")]["rules"][0]["resources"]
    assert _build(ws).create() == []                                  # idempotent
    b.delete()
    assert not kc.objs and b.existence() == Existence.NOT_EXIST


class FakeAWSWithEKS(FakeAWS):
    def __init__(self):
        super().__init__()
        self.oidc = {}
        self.trust = {}

    def describe_cluster(self, name):
        assert name == "eks1"
        return {"cluster": {"identity": {"oidc": {"issuer": "https://oidc.eks.us-west-2.amazonaws.com/id/ABC"}}}}

    def list_open_id_connect_providers(self):
        return {"OpenIDConnectProviderList": [{"Arn": a} for a in self.oidc]}

    def create_open_id_connect_provider(self, Url, ClientIDList, ThumbprintList, Tags):
        self.oidc["arn:aws:iam::123:oidc-provider/" + Url.replace("https://", "")] = ClientIDList

    def delete_open_id_connect_provider(self, OpenIDConnectProviderArn):
        del self.oidc[OpenIDConnectProviderArn]

    def create_role(self, RoleName, AssumeRolePolicyDocument, Tags):
        super().create_role(RoleName, AssumeRolePolicyDocument, Tags)
        self.trust[RoleName] = json.loads(AssumeRolePolicyDocument)

    def get_role(self, RoleName):
        r = super().get_role(RoleName)
        r["Role"]["Arn"] = f"arn:aws:iam::123:role/{RoleName}"
        return r


def test_eks_irsa():
    kc, aws = FakeKubectl(), FakeAWSWithEKS()
    cfg = {"type": "kubernetes", "cloud_provider": {"type": "aws", "region": "us-west-2", "eks_cluster_name": "eks1"}}
    ws = KubernetesWorkspace(cfg, "w2", Kubectl(runner=kc), aws.client)
    assert isinstance(ws.cloud, EKSIntegration)
    b = WorkspaceBuilder(ws.steps({"managed_cloud_storage": True}), log=lambda m: None)
    b.create()
    assert b.existence() == Existence.COMPLETED and len(aws.buckets) == 1
    role = ws.cloud.roles["worker"]
    cond = aws.trust[role]["Statement"][0]["Condition"]["StringEquals"]
    assert cond["oidc.eks.us-west-2.amazonaws.com/id/ABC:sub"] == \
        "system:serviceaccount:cloudtik-w2:cloudtik-worker-service-account"
    assert aws.trust[role]["Statement"][0]["Principal"]["Federated"] in aws.oidc
    sa = kc.objs[("serviceaccount", "cloudtik-w2", "cloudtik-worker-service-account")]
    assert sa["metadata"]["annotations"]["eks.amazonaws.com/role-arn"] == f"arn:aws:iam::123:role/{role}"
    b.delete(delete_managed_storage=True)
    assert not aws.roles and not aws.oidc and not kc.objs and not aws.buckets


def test_gke_workload_identity():
    kc, gcp = FakeKubectl(), FakeGCP(project="proj")
    cfg = {"type": "kubernetes", "namespace": "ml", "cloud_provider": {"type": "gcp", "project_id": "proj"}}
    ws = KubernetesWorkspace(cfg, "w3", Kubectl(runner=kc), gcp)
    assert isinstance(ws.cloud, GKEIntegration)
    b = _build(ws)
    b.create()
    assert b.existence() == Existence.COMPLETED
    members = {m for bb in gcp.policy["bindings"] if bb["role"] == "roles/iam.workloadIdentityUser"
               for m in bb["members"]}
    assert "serviceAccount:proj.svc.id.goog[ml/cloudtik-head-service-account]" in members
    email = ws.cloud.email("head")
    sa = kc.objs[("serviceaccount", "ml", "cloudtik-head-service-account")]
    assert sa["metadata"]["annotations"]["iam.gke.io/gcp-service-account"] == email
    assert any(bb["role"] == "roles/storage.admin" and f"serviceAccount:{email}" in bb["members"]
               for bb in gcp.policy["bindings"])
    b.delete()
    assert b.existence() == Existence.NOT_EXIST and not gcp.policy["bindings"]


class FakeARMWithAKS(FakeARM):
    def __call__(self, method, url, params, body):
        out = super().__call__(method, url, params, body)
        if method == "PUT" and "userAssignedIdentities" in url and "federatedIdentityCredentials" not in url:
            out["properties"]["clientId"] = "client-" + out["properties"]["principalId"]
        return out


def test_aks_workload_identity():
    kc, arm = FakeKubectl(), FakeARMWithAKS()
    cp = {"type": "azure", "subscription_id": "sub", "resource_group": "rg", "aks_cluster_name": "aks1",
          "poll_interval_s": 0}
    arm.items["https://management.azure.com/subscriptions/sub/resourceGroups/rg/providers/"
              "Microsoft.ContainerService/managedClusters/aks1"] = {
        "properties": {"oidcIssuerProfile": {"issuerURL": "https://oidc.aks/issuer/"}}}
    ws = KubernetesWorkspace({"type": "kubernetes", "cloud_provider": cp}, "w4", Kubectl(runner=kc), arm)
    assert isinstance(ws.cloud, AKSIntegration)
    b = _build(ws)
    b.create()
    assert b.existence() == Existence.COMPLETED
    fic = next(v for k, v in arm.items.items() if "federatedIdentityCredentials" in k and "worker" in k)
    assert fic["properties"]["issuer"] == "https://oidc.aks/issuer/"
    assert fic["properties"]["subject"] == "system:serviceaccount:cloudtik-w4:cloudtik-worker-service-account"
    sa = kc.objs[("serviceaccount", "cloudtik-w4", "cloudtik-head-service-account")]
    assert sa["metadata"]["annotations"]["azure.workload.identity/client-id"].startswith("client-principal-")
    assert len([k for k in arm.items if "roleAssignments" in k]) == 2
    b.delete()
    assert not [k for k in arm.items if "userAssignedIdentities" in k] and not kc.objs


def test_cloud_workspace_factory_and_cluster_services():
    kc = FakeKubectl()
    plan = cloud_workspace({"type": "kubernetes", "_kubectl": Kubectl(runner=kc)}, "w5")
    assert isinstance(plan, KubernetesWorkspace) and plan.info()["namespace"] == "cloudtik-w5"
    svcs = cluster_services("ns", "c1", {"jupyter": {"port": 8888}, "mlflow": {"port": 5001}}, external=True)
    assert [s["metadata"]["name"] for s in svcs] == ["c1-head", "c1-head-external", "c1-node"]
    assert [p["port"] for p in svcs[0]["spec"]["ports"]] == [8888, 5001]
    assert svcs[1]["spec"]["type"] == "LoadBalancer" and svcs[2]["spec"]["clusterIP"] == "None"
    assert svcs[0]["spec"]["selector"]["cloudtik-node-kind"] == "head"
