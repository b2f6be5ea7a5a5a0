"""End-to-end cluster lifecycle on the virtual provider (several nodes on this host):
``cloudtik start`` -> head setup (state service, node agent, controller) -> the controller
launches and sets up min_workers -> scale up on a GPU request -> exec / submit / health /
metrics -> ``cloudtik stop``.  Reference test strategy: the mock-provider scaler tests of
tests/unit -- here the real CLI, daemons and controller run."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "bin", "cloudtik")

CONFIG = """
cluster_name: {name}
provider:
    type: virtual
available_node_types:
    head.default:
        node_config: {{instance_type: virtual.head}}
        resources: {{CPU: 2}}
    worker.default:
        node_config: {{instance_type: virtual.worker}}
        resources: {{CPU: 2, GPU: 1}}
        min_workers: 2
        max_workers: 4
head_node_type: head.default
runtime:
    types: [ai]
    ai: {{with_gpu: false}}
"""


def _run(env, *args, timeout=240, check=True):
    r = subprocess.run([CLI, *args], env=env, capture_output=True, text=True, timeout=timeout)
    if check and r.returncode != 0:
        raise AssertionError(f"cloudtik {' '.join(args)} failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    return r.stdout


@pytest.fixture
def cluster(tmp_path):
    name = f"t{os.getpid() % 10000}"
    cfg = tmp_path / "cluster.yaml"
    cfg.write_text(CONFIG.format(name=name))
    env = dict(os.environ, CLOUDTIK_LOCAL_STATE_DIR=str(tmp_path / "state"), CLOUDTIK_UPDATE_INTERVAL_S="1",
               CLOUDTIK_METRIC_PORT="0", CLOUDTIK_CONFIG_CACHE=str(tmp_path / "cache"),
               CLOUDTIK_PYTHON=sys.executable)
    yield env, str(cfg), name
    _run(env, "stop", str(cfg), "-y", "--hard", check=False)


def test_virtual_cluster_lifecycle(cluster, tmp_path):
    env, cfg, name = cluster
    out = _run(env, "start", cfg, "-y")
    assert "is up" in out
    assert "2 worker(s) ready" in _run(env, "wait-for-ready", cfg, "--timeout", "120")
    info = json.loads(_run(env, "info", cfg, "--json"))
    assert info["status"] == "RUNNING" and info["total_workers_ready"] == 2
    assert info["resources"]["GPU"] == 2

    # a GPU request beyond capacity launches a third worker
    _run(env, "scale", cfg, "--gpus", "3")
    deadline = time.time() + 120
    while time.time() < deadline:
        info = json.loads(_run(env, "info", cfg, "--json"))
        if info["total_workers_ready"] >= 3:
            break
        time.sleep(2)
    assert info["total_workers_ready"] == 3

    out = _run(env, "exec", cfg, "--all-nodes", "echo node=$CLOUDTIK_NODE_IP head=$CLOUDTIK_HEAD_IP")
    assert out.count("head=" + info["head_ip"]) == 4

    job = tmp_path / "job.py"
    job.write_text("import sys\nprint('JOB-ARGS', sys.argv[1:])\n")
    assert "JOB-ARGS ['x', 'y']" in _run(env, "submit", cfg, str(job), "x", "y")
    # north-star config #1: AI runtime MNIST MLP on CPU through `cloudtik submit` -> cloudtik-run
    out = _run(env, "submit", cfg, os.path.join(ROOT, "examples", "ai", "mnist_mlp.py"), "--epochs", "2",
               "--train-size", "3000")
    res = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert res["final"]["eval_accuracy"] > 0.8

    assert "healthy" in _run(env, "health-check", cfg)
    ps = _run(env, "process-status", cfg)
    assert "cloudtik_cluster_controller" in ps and ps.count("cloudtik_node_monitor") == 4
    assert info["head_ip"] in _run(env, "resource-metrics", cfg)
    dump = _run(env, "cluster-dump", cfg, "-o", str(tmp_path / "dump.tar.gz"))
    assert os.path.exists(dump.strip())

    _run(env, "stop", cfg, "-y")
    assert "RUNNING" not in _run(env, "info", cfg, "--json")


def test_on_demand_workflow_example(tmp_path):
    """examples/workflows/on_demand_ai_job.py: start -> wait -> submit (pid job waiter) -> stop."""
    name = f"w{os.getpid() % 10000}"
    cfg = tmp_path / "cluster.yaml"
    cfg.write_text(CONFIG.format(name=name).replace("min_workers: 2", "min_workers: 1"))
    marker = tmp_path / "done.txt"
    job = tmp_path / "job.py"
    job.write_text(f"open({str(marker)!r}, 'w').write('ok')\n")
    env = dict(os.environ, CLOUDTIK_LOCAL_STATE_DIR=str(tmp_path / "state"), CLOUDTIK_UPDATE_INTERVAL_S="1",
               CLOUDTIK_METRIC_PORT="0", CLOUDTIK_CONFIG_CACHE=str(tmp_path / "cache"),
               CLOUDTIK_PYTHON=sys.executable, PYTHONPATH=ROOT)
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "workflows", "on_demand_ai_job.py"),
                            str(cfg), str(job), "--min-workers", "1"], env=env, capture_output=True, text=True,
                           timeout=400)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        assert "job finished" in r.stdout and "cluster stopped" in r.stdout
        assert marker.read_text() == "ok"
    finally:
        _run(env, "stop", str(cfg), "-y", "--hard", check=False)
