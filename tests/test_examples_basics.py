"""The AI basics examples (examples/ai/basics; reference examples/runtime/ai/basics) run end to
end on CPU: concurrent tracked hyperparameter trials, Horovod-API data parallelism over 2
gloo ranks, scikit-learn model selection and the tabular embedding model -- and the tracking
client logs to an MLflow-REST server (an in-process stand-in) or to local files."""
import json
import os
import socket
import subprocess
import sys
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASICS = os.path.join(ROOT, "examples", "ai", "basics")


def _run(args, env_extra, timeout=600):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", **env_extra)
    env.pop("MLFLOW_TRACKING_URI", None)
    env.pop("CLOUDTIK_HEAD_IP", None)
    env.update(env_extra)
    r = subprocess.run([sys.executable] + args, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def _records(d, name):
    with open(os.path.join(d, f"{name}.jsonl")) as f:
        return [json.loads(l) for l in f]


def test_digits_hyperopt_tracked_trials(tmp_path):
    out = _run([os.path.join(BASICS, "digits_hyperopt_tracking.py"), "--trials", "4", "--concurrent", "2",
                "--epochs", "6"], {"CLOUDTIK_TRACKING_DIR": str(tmp_path)})
    assert out["trials"] == 4 and out["failed"] == 0 and out["best"]["accuracy"] > 0.8
    recs = _records(tmp_path, "digits-hyperopt")
    runs = {r["run_id"] for r in recs}
    assert len(runs) == 4
    assert sum(1 for r in recs if r.get("metric") == "val_accuracy") == 4 * 6
    assert sum(1 for r in recs if r.get("status") == "FINISHED") == 4


def test_digits_horovod_two_ranks(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = _run(["-m", "cloudtik_amd.runner.launch", "--num-proc", "2", "--master-port", str(port),
                os.path.join(BASICS, "digits_horovod.py"), "--epochs", "6"],
               {"CLOUDTIK_TRACKING_DIR": str(tmp_path), "CLOUDTIK_DEVICE": "cpu"})
    assert out["world"] == 2 and out["val_accuracy"] > 0.85
    recs = _records(tmp_path, "digits-horovod")
    assert len({r["run_id"] for r in recs}) == 1          # only rank 0 logs


def test_iris_and_rossmann(tmp_path):
    out = _run([os.path.join(BASICS, "iris_sklearn_tune.py"), "--trials", "6", "--concurrent", "3"],
               {"CLOUDTIK_TRACKING_DIR": str(tmp_path)})
    assert out["best_accuracy"] > 0.9 and out["trials"] == 6
    out = _run([os.path.join(BASICS, "rossmann_tabular.py"), "--epochs", "4"],
               {"CLOUDTIK_TRACKING_DIR": str(tmp_path)})
    assert out["val_rmspe"] < 0.2


class _FakeMLflow(BaseHTTPRequestHandler):
    calls = []

    def log_message(self, *a):
        pass

    def _send(self, obj, code=200):
        body = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_GET(self):
        self.calls.append(("GET", self.path, None))
        if "experiments/get-by-name" in self.path:
            return self._send({"error_code": "RESOURCE_DOES_NOT_EXIST"}, 404)
        self._send({})

    def do_POST(self):
        body = json.loads(self.rfile.read(int(self.headers["Content-Length"])) or b"{}")
        self.calls.append(("POST", self.path, body))
        if self.path.endswith("experiments/create"):
            return self._send({"experiment_id": "7"})
        if self.path.endswith("runs/create"):
            return self._send({"run": {"info": {"run_id": "r1", "experiment_id": body["experiment_id"]}}})
        self._send({})


def test_tracking_client_speaks_mlflow_rest(tmp_path, monkeypatch):
    pytest.importorskip("requests")
    srv = HTTPServer(("127.0.0.1", 0), _FakeMLflow)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        import cloudtik_amd.runtime.ai.tracking as tr
        monkeypatch.setenv("MLFLOW_TRACKING_URI", f"http://127.0.0.1:{srv.server_port}")
        monkeypatch.setenv("RANK", "0")
        with tr.start_run("exp1", run_name="n1", backend="rest") as run:
            assert run.backend == "rest" and run.run_id == "r1"
            run.log_param("lr", 0.1)
            run.log_metric("loss", 0.5, step=3)
            run.set_tag("k", "v")
        paths = [p for m, p, b in _FakeMLflow.calls if m == "POST"]
        assert [p.rsplit("/", 2)[-2] + "/" + p.rsplit("/", 1)[-1] for p in paths] == [
            "experiments/create", "runs/create", "runs/log-parameter", "runs/log-metric", "runs/set-tag",
            "runs/update"]
        metric = next(b for m, p, b in _FakeMLflow.calls if p.endswith("log-metric"))
        assert metric["key"] == "loss" and metric["step"] == 3 and metric["run_id"] == "r1"
        assert next(b for m, p, b in _FakeMLflow.calls if p.endswith("runs/update"))["status"] == "FINISHED"
        # non-zero ranks never log
        monkeypatch.setenv("RANK", "1")
        n = len(_FakeMLflow.calls)
        with tr.start_run("exp1", backend="rest") as run:
            run.log_metric("loss", 1.0)
        assert len(_FakeMLflow.calls) == n
    finally:
        srv.shutdown()
