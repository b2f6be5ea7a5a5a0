"""``cloudtik-operator``: Kubernetes operator for CloudTik clusters (reference
providers/kubernetes/cloudtik_operator/operator.py, a kopf operator).

Watches ``CloudTikCluster`` custom resources (``cloudtik.io/v1``, CRD and Helm chart in
``deploy/helm/cloudtik-operator``) and reconciles each one into a running cluster:

* a CR's ``spec`` is a CloudTik cluster config (``available_node_types``, ``head_node_type``,
  ``max_workers``, ``runtime``, ...); the operator forces ``cluster_name`` = the CR name and
  ``provider = {type: kubernetes, namespace: <CR namespace>}`` -- pods are nodes,
  ``amd.com/gpu`` requests give each worker pod its MI355X GPUs;
* new or changed spec (``metadata.generation`` > ``status.observedGeneration``): create or
  update the cluster (head pod + head setup, which starts the state service and the
  cluster controller / autoscaler on the head) -> ``status.phase = Running``;
* head pod gone while the CR exists: relaunch it (``Recovering`` -> ``Running``);
* CR being deleted (``deletionTimestamp``): tear the cluster down, then drop the
  operator's finalizer so Kubernetes can remove the object;
* failures set ``status.phase = Error`` with the message and are retried next pass.

The reference is event driven through kopf; kopf is not available here, so this is a
level-triggered poll loop over ``kubectl`` (``--interval``, default 5 s) -- equivalent for a
reconciler that always compares desired with observed state.

    cloudtik-operator --namespace cloudtik          # one namespace
    cloudtik-operator --all-namespaces
"""
from __future__ import annotations

import argparse
import copy
import json
import logging
import subprocess
import sys
import threading
import time
from typing import Any, Callable, Dict, List, Optional

logger = logging.getLogger(__name__)

GROUP, VERSION, PLURAL = "cloudtik.io", "v1", "cloudtikclusters"
RESOURCE = f"{PLURAL}.{GROUP}"
FINALIZER = "cloudtik.io/cluster-teardown"
PHASE_RUNNING, PHASE_UPDATING, PHASE_RECOVERING, PHASE_ERROR = "Running", "Updating", "Recovering", "Error"


def cr_to_config(cr: Dict[str, Any]) -> Dict[str, Any]:
    """CloudTikCluster object -> cluster config dict."""
    meta = cr["metadata"]
    cfg = copy.deepcopy(cr.get("spec") or {})
    cfg["cluster_name"] = meta["name"]
    prov = dict(cfg.get("provider") or {})
    prov.update(type="kubernetes", namespace=meta.get("namespace", "default"))
    cfg["provider"] = prov
    return cfg


class Kubectl:
    def __init__(self, kubectl: Optional[List[str]] = None):
        self.cmd = list(kubectl or ["kubectl"])

    def run(self, *args, input_obj=None, check=True) -> str:
        r = subprocess.run(self.cmd + list(args), input=json.dumps(input_obj) if input_obj is not None else None,
                           capture_output=True, text=True, timeout=120)
        if check and r.returncode != 0:
            raise RuntimeError(f"kubectl {' '.join(args)} failed: {r.stderr.strip()}")
        return r.stdout

    def list_clusters(self, namespace: Optional[str]) -> List[Dict[str, Any]]:
        scope = ["-n", namespace] if namespace else ["--all-namespaces"]
        return json.loads(self.run("get", RESOURCE, *scope, "-o", "json") or "{}").get("items", [])

    def patch(self, cr, patch: Dict[str, Any], subresource: Optional[str] = None):
        meta = cr["metadata"]
        args = ["patch", RESOURCE, meta["name"], "-n", meta.get("namespace", "default"), "--type", "merge",
                "-p", json.dumps(patch)]
        if subresource:
            args += ["--subresource", subresource]
        self.run(*args)


class CloudTikOperator:
    """Level-triggered reconciler.  ``create_or_update``, ``teardown`` and ``head_alive``
    are injectable (defaults call the cluster operator / kubernetes provider)."""

    def __init__(self, kubectl: Optional[Kubectl] = None, namespace: Optional[str] = None,
                 create_or_update: Optional[Callable[[Dict[str, Any]], None]] = None,
                 teardown: Optional[Callable[[Dict[str, Any]], None]] = None,
                 head_alive: Optional[Callable[[Dict[str, Any]], bool]] = None):
        self.k = kubectl or Kubectl()
        self.namespace = namespace
        self._create = create_or_update or _default_create_or_update
        self._teardown = teardown or _default_teardown
        self._head_alive = head_alive or _default_head_alive
        self.events: List[str] = []

    def _event(self, cr, msg):
        m = f"{cr['metadata'].get('namespace', 'default')}/{cr['metadata']['name']}: {msg}"
        self.events.append(m)
        logger.info(m)

    def _status(self, cr, **fields):
        try:
            self.k.patch(cr, {"status": fields}, subresource="status")
        except RuntimeError as e:            # older servers without the status subresource
            logger.debug("status subresource patch failed (%s); patching the object", e)
            self.k.patch(cr, {"status": fields})

    def reconcile(self, cr: Dict[str, Any]):
        meta = cr["metadata"]
        status = cr.get("status") or {}
        finalizers = list(meta.get("finalizers") or [])
        if meta.get("deletionTimestamp"):
            if FINALIZER in finalizers:
                self._event(cr, "deleting: tearing the cluster down")
                self._teardown(cr_to_config(cr))
                self.k.patch(cr, {"metadata": {"finalizers": [f for f in finalizers if f != FINALIZER]}})
            return
        if FINALIZER not in finalizers:
            self.k.patch(cr, {"metadata": {"finalizers": finalizers + [FINALIZER]}})
        gen = int(meta.get("generation", 1))
        observed = int(status.get("observedGeneration", 0))
        cfg = cr_to_config(cr)
        try:
            if gen > observed:
                self._status(cr, phase=PHASE_UPDATING, message="")
                self._event(cr, f"generation {gen}: creating / updating the cluster")
                self._create(cfg)
                self._status(cr, phase=PHASE_RUNNING, observedGeneration=gen, message="")
            elif not self._head_alive(cfg):
                self._status(cr, phase=PHASE_RECOVERING, message="head pod lost")
                self._event(cr, "head pod lost: recovering")
                self._create(cfg)
                self._status(cr, phase=PHASE_RUNNING, observedGeneration=gen, message="")
        except Exception as e:  # noqa: BLE001 - retried on the next pass
            self._event(cr, f"error: {e}")
            self._status(cr, phase=PHASE_ERROR, message=str(e)[:1000])

    def reconcile_all(self):
        for cr in self.k.list_clusters(self.namespace):
            self.reconcile(cr)

    def run(self, interval: float = 5.0, stop: Optional[threading.Event] = None):
        stop = stop or threading.Event()
        while not stop.is_set():
            try:
                self.reconcile_all()
            except Exception:  # noqa: BLE001
                logger.exception("reconcile pass failed")
            stop.wait(interval)


def _default_create_or_update(cfg):
    from cloudtik_amd.core.cluster_operator import create_or_update_cluster
    create_or_update_cluster(cfg, no_config_cache=True)


def _default_teardown(cfg):
    from cloudtik_amd.core.cluster_operator import teardown_cluster
    from cloudtik_amd.core.cluster_config import bootstrap_config
    teardown_cluster(bootstrap_config(cfg, no_config_cache=True))


def _default_head_alive(cfg) -> bool:
    from cloudtik_amd.core import tags as T
    from cloudtik_amd.core.provider_factory import get_node_provider
    p = get_node_provider(cfg["provider"], cfg["cluster_name"], use_cache=False)
    return bool(p.non_terminated_nodes({T.CLOUDTIK_TAG_NODE_KIND: T.NODE_KIND_HEAD}))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="cloudtik-operator", description=__doc__.split("\n")[0])
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--namespace", default="cloudtik")
    g.add_argument("--all-namespaces", action="store_true")
    ap.add_argument("--interval", type=float, default=5.0)
    ap.add_argument("--once", action="store_true", help="one reconcile pass, then exit")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(message)s")
    op = CloudTikOperator(namespace=None if a.all_namespaces else a.namespace)
    if a.once:
        op.reconcile_all()
        return 0
    import signal
    stop = threading.Event()
    for s in (signal.SIGTERM, signal.SIGINT):
        signal.signal(s, lambda *_: stop.set())
    op.run(a.interval, stop)
    return 0


if __name__ == "__main__":
    sys.exit(main())
