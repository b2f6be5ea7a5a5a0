"""cloudtik-operator (reference providers/kubernetes/cloudtik_operator, SURVEY.md §2.9 / §4
k8s operator tests): reconcile CloudTikCluster objects held by a fake kubectl -- create on a
new generation, recover a lost head, report errors, tear down and release the finalizer on
deletion; the CRD and Helm values are valid YAML."""
import json
import os
import sys

import pytest
import yaml

from cloudtik_amd.providers.kubernetes.operator import (FINALIZER, CloudTikOperator, Kubectl, cr_to_config)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

FAKE = r'''#!/usr/bin/env python3
import json, os, sys
db = os.environ["FAKE_CRS"]
st = json.load(open(db))
a = sys.argv[1:]
if a[0] == "get":
    print(json.dumps({"items": list(st.values())}))
elif a[0] == "patch":
    name = a[2]; body = json.loads(a[a.index("-p") + 1])
    obj = st[name]
    for k, v in body.items():
        if isinstance(v, dict):
            obj.setdefault(k, {}).update(v)
        else:
            obj[k] = v
    json.dump(st, open(db, "w"))
    open(db + ".log", "a").write(" ".join(a) + "\n")
'''


def _cr(name, gen=1, **kw):
    cr = {"apiVersion": "cloudtik.io/v1", "kind": "CloudTikCluster",
          "metadata": {"name": name, "namespace": "ai", "generation": gen},
          "spec": {"max_workers": 2, "available_node_types": {"worker.mi355x": {"resources": {"GPU": 8}}}}}
    cr["metadata"].update(kw)
    return cr


@pytest.fixture
def fake(tmp_path, monkeypatch):
    k = tmp_path / "kubectl"
    k.write_text(FAKE)
    k.chmod(0o755)
    db = tmp_path / "crs.json"
    monkeypatch.setenv("FAKE_CRS", str(db))

    def put(*crs):
        db.write_text(json.dumps({c["metadata"]["name"]: c for c in crs}))

    def get(name):
        return json.loads(db.read_text())[name]
    return Kubectl([sys.executable, str(k)]), put, get


def test_cr_to_config_forces_kubernetes_provider():
    cfg = cr_to_config(_cr("c1"))
    assert cfg["cluster_name"] == "c1" and cfg["provider"] == {"type": "kubernetes", "namespace": "ai"}
    assert cfg["available_node_types"]["worker.mi355x"]["resources"] == {"GPU": 8}


def test_operator_lifecycle(fake):
    k, put, get = fake
    created, torn, alive = [], [], {"c1": True}
    op = CloudTikOperator(k, "ai", create_or_update=lambda c: created.append(c["cluster_name"]),
                          teardown=lambda c: torn.append(c["cluster_name"]),
                          head_alive=lambda c: alive[c["cluster_name"]])
    put(_cr("c1"))
    op.reconcile_all()
    cr = get("c1")
    assert created == ["c1"] and cr["status"]["phase"] == "Running" and cr["status"]["observedGeneration"] == 1
    assert FINALIZER in cr["metadata"]["finalizers"]
    op.reconcile_all()                               # steady state: nothing to do
    assert created == ["c1"]
    cr["metadata"]["generation"] = 2                 # spec edited
    put(cr)
    op.reconcile_all()
    assert created == ["c1", "c1"] and get("c1")["status"]["observedGeneration"] == 2
    alive["c1"] = False                              # head pod lost
    op.reconcile_all()
    assert created == ["c1"] * 3 and any("recovering" in e for e in op.events)
    cr = get("c1")
    cr["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
    put(cr)
    op.reconcile_all()
    assert torn == ["c1"] and FINALIZER not in get("c1")["metadata"]["finalizers"]


def test_operator_reports_errors(fake):
    k, put, get = fake

    def boom(cfg):
        raise RuntimeError("no amd.com/gpu capacity")
    op = CloudTikOperator(k, "ai", create_or_update=boom, teardown=lambda c: None, head_alive=lambda c: True)
    put(_cr("c2"))
    op.reconcile_all()
    st = get("c2")["status"]
    assert st["phase"] == "Error" and "amd.com/gpu" in st["message"] and "observedGeneration" not in st


def test_crd_and_chart_files():
    d = os.path.join(ROOT, "deploy", "helm", "cloudtik-operator")
    crd = yaml.safe_load(open(os.path.join(d, "crds", "cloudtikclusters.yaml")))
    assert crd["spec"]["group"] == "cloudtik.io" and crd["spec"]["names"]["kind"] == "CloudTikCluster"
    assert crd["spec"]["versions"][0]["subresources"] == {"status": {}}
    values = yaml.safe_load(open(os.path.join(d, "values.yaml")))
    assert values["exampleCluster"]["workerGPUs"] == 8
    assert yaml.safe_load(open(os.path.join(d, "Chart.yaml")))["name"] == "cloudtik-operator"
