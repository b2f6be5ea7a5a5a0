"""Service daemon / pull jobs (reference core/_private/util/service/*)."""
import logging
import os
import subprocess
import sys
import threading
import time

from cloudtik_amd.core.service_daemon import PullJob, ScriptPullJob, cmd_args_to_call_args

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Flaky(PullJob):
    def __init__(self, fail_times=3, interval=0.01):
        super().__init__(interval)
        self.fail_times = fail_times
        self.calls = 0

    def pull(self):
        self.calls += 1
        if self.calls <= self.fail_times:
            raise RuntimeError("backend down")


def test_cmd_args_to_call_args():
    args, kw = cmd_args_to_call_args(["a", "3", "k=1", 'j={"x": [1, 2]}', "s=text"])
    assert args == ["a", 3] and kw == {"k": 1, "j": {"x": [1, 2]}, "s": "text"}


def test_pull_job_survives_and_deduplicates_errors(caplog):
    job = Flaky(fail_times=3)
    state = {"last": None, "count": 0}
    with caplog.at_level(logging.INFO):
        for _ in range(5):
            job.run_once(state)
    assert job.errors == 3 and job.pulls == 2
    assert sum("pull failed: backend down" in r.getMessage() for r in caplog.records) == 1
    assert state["last"] is None


def test_pull_job_stops_on_event():
    job = Flaky(fail_times=0, interval=0.01)
    job.stop_event = threading.Event()
    t = threading.Thread(target=job.run)
    t.start()
    time.sleep(0.1)
    job.stop_event.set()
    t.join(2)
    assert not t.is_alive() and job.pulls >= 2


def test_script_pull_job_runs_script(tmp_path):
    out = tmp_path / "count.txt"
    script = tmp_path / "pull.py"
    script.write_text("import sys\nopen(sys.argv[1], 'a').write('x')\n")
    job = ScriptPullJob(0.01, str(script), [str(out)])
    job.pull()
    job.pull()
    assert out.read_text() == "xx"


def test_service_daemon_start_stop_cli(tmp_path):
    out = tmp_path / "ticks.txt"
    script = tmp_path / "tick.sh"
    script.write_text(f"echo tick >> {out}\n")
    env = dict(os.environ, CLOUDTIK_SESSION_DIR=str(tmp_path / "session"),
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    cli = [os.path.join(ROOT, "bin", "cloudtik"), "node", "service-daemon"]
    r = subprocess.run(cli + ["start", "ticker", "--pull-script", str(script), "--interval", "0.1"],
                       capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == 0, r.stderr
    deadline = time.time() + 20
    while time.time() < deadline and (not out.exists() or len(out.read_text().split()) < 3):
        time.sleep(0.1)
    assert len(out.read_text().split()) >= 3
    r = subprocess.run(cli + ["stop", "ticker"], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == 0 and "stopped" in r.stdout
    n = len(out.read_text().split())
    time.sleep(0.5)
    assert len(out.read_text().split()) == n
