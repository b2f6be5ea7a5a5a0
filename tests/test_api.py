"""Python API (Cluster / AICluster / events / job waiters) against a virtual cluster."""
import os
import sys
import time

import pytest

CONFIG = {
    "cluster_name": "apitest{}".format(os.getpid() % 10000),
    "provider": {"type": "virtual"},
    "available_node_types": {
        "head.default": {"node_config": {"instance_type": "virtual.head"}, "resources": {"CPU": 2}},
        "worker.default": {"node_config": {"instance_type": "virtual.worker"}, "resources": {"CPU": 2},
                           "min_workers": 1, "max_workers": 2},
    },
    "head_node_type": "head.default",
    "runtime": {"types": ["ai"], "ai": {"with_gpu": False}},
}


@pytest.fixture
def env(tmp_path, monkeypatch):
    monkeypatch.setenv("CLOUDTIK_LOCAL_STATE_DIR", str(tmp_path / "state"))
    monkeypatch.setenv("CLOUDTIK_UPDATE_INTERVAL_S", "1")
    monkeypatch.setenv("CLOUDTIK_METRIC_PORT", "0")
    monkeypatch.setenv("CLOUDTIK_PYTHON", sys.executable)
    return tmp_path


def test_cluster_api_lifecycle(env):
    import copy
    from cloudtik_amd.core.api import Cluster
    from cloudtik_amd.core.event_system import CreateClusterEvent
    from cloudtik_amd.runtime.ai.api import AICluster
    c = AICluster(copy.deepcopy(CONFIG))
    seen = []
    for ev in (CreateClusterEvent.up_started, CreateClusterEvent.head_node_acquired,
               CreateClusterEvent.run_setup_cmd, CreateClusterEvent.start_cloudtik_runtime,
               CreateClusterEvent.cluster_booting_completed):
        c.register_callback(ev, lambda d, ev=ev: seen.append(ev))
    try:
        c.start()
        assert seen == [CreateClusterEvent.up_started, CreateClusterEvent.head_node_acquired,
                        CreateClusterEvent.run_setup_cmd, CreateClusterEvent.start_cloudtik_runtime,
                        CreateClusterEvent.cluster_booting_completed]
        assert c.wait_for_ready(min_workers=1, timeout=120) >= 1
        info = c.get_info()
        assert info["status"] == "RUNNING" and info["total_workers_ready"] >= 1
        assert c.get_mlflow_uri().endswith(":5001")
        assert c.get_head_node_ip() == info["head_ip"]
        out = c.exec("echo hello-$CLOUDTIK_NODE_IP", with_output=True)
        assert b"hello-" + info["head_ip"].encode() in out
        # a detached job followed by the pid job waiter
        job = env / "job.py"
        job.write_text("import time, pathlib; time.sleep(2); pathlib.Path('done.txt').write_text('ok')\n")
        t0 = time.time()
        c.submit(str(job), job_waiter="pid")
        assert time.time() - t0 >= 1.5
        assert b"ok" in c.exec("cat ~/user/jobs/done.txt", with_output=True)
        assert c.health_check()["healthy"]
    finally:
        c.stop()
    assert Cluster(copy.deepcopy(CONFIG)).get_info()["status"] == "STOPPED"
