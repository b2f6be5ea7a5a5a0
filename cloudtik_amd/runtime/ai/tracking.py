"""Experiment tracking for AI-runtime jobs: MLflow-compatible runs, params, metrics and tags
(reference examples/runtime/ai/basics/*-mlflow.py log through ``mlflow`` to the cluster's
tracking server, runtime/ai/runtime.py starts it).

``start_run`` returns a ``Run`` that talks to

* the ``mlflow`` package when it is importable (``backend="mlflow"``);
* otherwise the tracking server's REST API directly (``/api/2.0/mlflow/...`` over
  ``requests``): jobs on a node without the mlflow client still log to the cluster's server;
* otherwise (no server reachable / configured) a local JSON-lines file, so examples and
  tests run anywhere.

The tracking URI defaults to ``MLFLOW_TRACKING_URI``, else the AI runtime's server on the
head (``http://$CLOUDTIK_HEAD_IP:$MLFLOW_PORT``).  Only rank 0 of a distributed job should
log (``Run.disabled`` when ``RANK`` is not 0).
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, Optional


def tracking_uri() -> Optional[str]:
    uri = os.environ.get("MLFLOW_TRACKING_URI")
    if uri:
        return uri
    head = os.environ.get("CLOUDTIK_HEAD_IP")
    if head:
        return f"http://{head}:{os.environ.get('MLFLOW_PORT', '5001')}"
    return None


class Run:
    def __init__(self, backend: str, run_id: str, experiment: str, sink=None, base: Optional[str] = None,
                 disabled: bool = False):
        self.backend, self.run_id, self.experiment = backend, run_id, experiment
        self._sink, self._base, self.disabled = sink, base, disabled
        self._step = 0

    # ------------------------------------------------------------------ logging
    def _rest(self, path: str, body: Dict[str, Any]):
        import requests
        r = requests.post(f"{self._base}/api/2.0/mlflow/{path}", json=body, timeout=10)
        r.raise_for_status()
        return r.json()

    def _write(self, rec: Dict[str, Any]):
        self._sink.write(json.dumps(dict(rec, run_id=self.run_id, time=time.time())) + "\n")
        self._sink.flush()

    def log_param(self, key: str, value: Any):
        if self.disabled:
            return
        if self.backend == "mlflow":
            import mlflow
            mlflow.log_param(key, value)
        elif self.backend == "rest":
            self._rest("runs/log-parameter", {"run_id": self.run_id, "key": key, "value": str(value)})
        else:
            self._write({"param": key, "value": value})

    def log_params(self, params: Dict[str, Any]):
        for k, v in params.items():
            self.log_param(k, v)

    def log_metric(self, key: str, value: float, step: Optional[int] = None):
        if self.disabled:
            return
        step = self._step if step is None else step
        if self.backend == "mlflow":
            import mlflow
            mlflow.log_metric(key, float(value), step=step)
        elif self.backend == "rest":
            self._rest("runs/log-metric", {"run_id": self.run_id, "key": key, "value": float(value),
                                           "timestamp": int(time.time() * 1000), "step": int(step)})
        else:
            self._write({"metric": key, "value": float(value), "step": int(step)})

    def log_metrics(self, metrics: Dict[str, float], step: Optional[int] = None):
        for k, v in metrics.items():
            self.log_metric(k, v, step)

    def set_tag(self, key: str, value: Any):
        if self.disabled:
            return
        if self.backend == "mlflow":
            import mlflow
            mlflow.set_tag(key, value)
        elif self.backend == "rest":
            self._rest("runs/set-tag", {"run_id": self.run_id, "key": key, "value": str(value)})
        else:
            self._write({"tag": key, "value": value})

    def end(self, status: str = "FINISHED"):
        if self.disabled:
            return
        if self.backend == "mlflow":
            import mlflow
            mlflow.end_run(status=status)
        elif self.backend == "rest":
            self._rest("runs/update", {"run_id": self.run_id, "status": status,
                                       "end_time": int(time.time() * 1000)})
        elif self._sink is not None:
            self._write({"status": status})
            self._sink.close()

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        self.end("FAILED" if exc_type else "FINISHED")


def _rest_experiment(base: str, name: str) -> str:
    import requests
    r = requests.get(f"{base}/api/2.0/mlflow/experiments/get-by-name", params={"experiment_name": name}, timeout=10)
    if r.status_code == 200:
        return r.json()["experiment"]["experiment_id"]
    r = requests.post(f"{base}/api/2.0/mlflow/experiments/create", json={"name": name}, timeout=10)
    r.raise_for_status()
    return r.json()["experiment_id"]


def start_run(experiment: str = "cloudtik", run_name: Optional[str] = None, uri: Optional[str] = None,
              local_dir: Optional[str] = None, backend: Optional[str] = None) -> Run:
    """A run on the best available backend (see module doc)."""
    disabled = int(os.environ.get("RANK", "0") or 0) != 0
    uri = uri or tracking_uri()
    if backend in (None, "mlflow"):
        try:
            import mlflow
            if uri:
                mlflow.set_tracking_uri(uri)
            mlflow.set_experiment(experiment)
            r = mlflow.start_run(run_name=run_name) if not disabled else None
            return Run("mlflow", r.info.run_id if r else "", experiment, disabled=disabled)
        except ImportError:
            if backend == "mlflow":
                raise
    if backend in (None, "rest") and uri and uri.startswith("http"):
        try:
            if disabled:
                return Run("rest", "", experiment, base=uri, disabled=True)
            import requests
            eid = _rest_experiment(uri, experiment)
            body = {"experiment_id": eid, "start_time": int(time.time() * 1000)}
            if run_name:
                body["run_name"] = run_name
            r = requests.post(f"{uri}/api/2.0/mlflow/runs/create", json=body, timeout=10)
            r.raise_for_status()
            return Run("rest", r.json()["run"]["info"]["run_id"], experiment, base=uri)
        except Exception as e:   # noqa: BLE001 - server unreachable: fall back to local
            if backend == "rest":
                raise
            print(f"[tracking] {uri} not usable ({e}); logging locally", flush=True)
    d = local_dir or os.environ.get("CLOUDTIK_TRACKING_DIR", os.path.expanduser("~/.cloudtik/tracking"))
    os.makedirs(d, exist_ok=True)
    rid = f"{int(time.time() * 1000)}-{os.getpid()}"
    sink = None if disabled else open(os.path.join(d, f"{experiment}.jsonl"), "a")
    run = Run("local", rid, experiment, sink=sink, disabled=disabled)
    if not disabled and run_name:
        run.set_tag("run_name", run_name)
    return run
