"""Failure detection / elastic recovery / fault injection and profiling hooks
(SURVEY.md §5.1, §5.3, §5.4): cloudtik-run --max-restarts with checkpoint auto-resume under
an injected rank failure, async checkpoints, step-phase timers, rocprof wrapping."""
import json
import os
import socket
import subprocess

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = os.path.join(ROOT, "bin", "cloudtik-run")

JOB = r"""
import json, os, sys, torch
sys.path.insert(0, %(root)r)
from cloudtik_amd.models.mlp import MLP
from cloudtik_amd.train.trainer import Trainer
torch.manual_seed(0)
x = torch.randn(16 * 8, 1, 28, 28, generator=torch.Generator().manual_seed(1))
y = torch.randint(0, 10, (16 * 8,), generator=torch.Generator().manual_seed(2))
batches = [(x[i:i + 16], y[i:i + 16]) for i in range(0, len(x), 16)]
t = Trainer(MLP(), "sgd", lr=0.05, train_loader=batches, epochs=2, log_every=0,
            checkpoint_dir=%(ckpt)r, checkpoint_every=2, async_checkpoint=%(async_)r)
resumed_at = t.global_step
t.fit()
t.close()
out = {"rank": t.rank, "restart": int(os.environ.get("CLOUDTIK_RESTART_COUNT", "0")),
       "resumed_at": resumed_at, "final_step": t.global_step,
       "w": float(sum(p.double().sum() for p in t.model.parameters()))}
open(os.path.join(%(out)r, "rank%%d.json" %% t.rank), "w").write(json.dumps(out))
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_job(tmp_path, name, env_extra, async_=False, restarts=1):
    ckpt = tmp_path / f"ckpt_{name}"
    out = tmp_path / f"out_{name}"
    out.mkdir()
    job = tmp_path / f"job_{name}.py"
    job.write_text(JOB % {"root": ROOT, "ckpt": str(ckpt), "out": str(out), "async_": async_})
    env = dict(os.environ, **env_extra)
    r = subprocess.run([RUN, "--nproc-per-node", "2", "--master-port", str(_port()), "--max-restarts", str(restarts),
                        str(job)], capture_output=True, text=True, timeout=300, env=env)
    res = {int(f[4:-5]): json.loads((out / f).read_text()) for f in os.listdir(out)}
    return r, res


def test_injected_rank_failure_restarts_and_resumes(tmp_path):
    # clean reference run
    r0, ref = _run_job(tmp_path, "ref", {}, restarts=0)
    assert r0.returncode == 0, r0.stderr[-2000:]
    # rank 1 dies at step 5 of the first attempt; the job restarts from the step-4 checkpoint
    r, res = _run_job(tmp_path, "fail", {"CLOUDTIK_INJECT_FAIL_RANK": "1", "CLOUDTIK_INJECT_FAIL_STEP": "5"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "injected fault: rank 1 step 5" in r.stderr
    assert "restarting the job" in r.stderr
    assert sorted(res) == [0, 1]
    for v in res.values():
        assert v["restart"] == 1 and v["resumed_at"] == 4 and v["final_step"] == 16
        # resumed training reproduces the uninterrupted run (same data order, restored state)
        assert abs(v["w"] - ref[v["rank"]]["w"]) < 1e-6 * max(1.0, abs(ref[v["rank"]]["w"]))


def test_injected_failure_without_restart_fails_job(tmp_path):
    r, _ = _run_job(tmp_path, "norestart", {"CLOUDTIK_INJECT_FAIL_RANK": "0", "CLOUDTIK_INJECT_FAIL_STEP": "3",
                                             "CLOUDTIK_INJECT_FAIL_CODE": "23"}, restarts=0)
    assert r.returncode == 23


def test_async_checkpoint_job_restart(tmp_path):
    r, res = _run_job(tmp_path, "async", {"CLOUDTIK_INJECT_FAIL_RANK": "*", "CLOUDTIK_INJECT_FAIL_STEP": "7"},
                      async_=True)
    assert r.returncode == 0, r.stderr[-3000:]
    # the step-6 save is still in flight when every rank dies at step 7 if the host is
    # loaded: the job then resumes from the last COMMITTED checkpoint (step 4), never from a
    # partial one, and all ranks agree on it
    assert len({v["resumed_at"] for v in res.values()}) == 1
    for v in res.values():
        assert v["restart"] == 1 and v["resumed_at"] in (4, 6) and v["final_step"] == 16


def test_async_checkpoint_roundtrip(tmp_path):
    from cloudtik_amd.models.mlp import MLP
    from cloudtik_amd.train.checkpoint import Checkpointer
    from cloudtik_amd.train.optim import build_optimizer
    torch.manual_seed(0)
    m = MLP()
    opt = build_optimizer("adamw", m, 1e-3, 0.0, None)
    m(torch.randn(4, 1, 28, 28)).sum().backward()
    opt.step()
    ck = Checkpointer(str(tmp_path), keep=2)
    h = ck.save_async(3, m, opt, extra={"k": 1})
    assert h.wait() == os.path.join(str(tmp_path), "step-3")
    ck.save_async(5, m, opt).wait()
    ck.save_async(7, m, opt).wait()
    assert ck.steps() == [5, 7]
    saved = {k: v.clone() for k, v in m.state_dict().items()}
    torch.manual_seed(9)
    m2 = MLP()
    opt2 = build_optimizer("adamw", m2, 1e-3, 0.0, None)
    meta = ck.load_latest(m2, opt2)
    assert meta["step"] == 7
    for k, v in m2.state_dict().items():
        assert torch.equal(v, saved[k])
    assert torch.equal(opt2.exp_avg, opt.exp_avg)


def test_step_timer_and_log_timer():
    from cloudtik_amd.utils.profiling import LogTimer, StepTimer, range as roctx_range
    t = StepTimer(device="cpu")
    for _ in range(3):
        with t.phase("forward"):
            sum(range(1000)) if False else None
        with t.phase("backward"), roctx_range("inner"):
            pass
        t.step_done()
    s = t.summary()
    assert set(s) == {"forward", "backward", "step"} and all(v >= 0 for v in s.values())
    logs = []
    with LogTimer("phase", log=lambda fmt, *a: logs.append(fmt % a)):
        pass
    assert logs and logs[0].startswith("phase: ")


def test_rocprof_command_puts_program_after_dashes():
    from cloudtik_amd.utils.profiling import rocprof_command
    cmd = rocprof_command(["/usr/bin/python3", "train.py", "--x"], "/tmp/p/rank0")
    i = cmd.index("--")
    assert cmd[i + 1:] == ["/usr/bin/python3", "train.py", "--x"]
    assert "--kernel-trace" in cmd and "--stats" in cmd and "-d" in cmd
    pmc = rocprof_command(["./b"], "/tmp/p", pmc=["SQ_WAVES", "GRBM_COUNT"])
    assert "--pmc" in pmc and "--stats" not in pmc and "--marker-trace" not in pmc


def test_cloudtik_run_profile_flag_wraps_ranks(tmp_path, monkeypatch):
    """--profile puts every rank under rocprofv3 (a stub records its argv here)."""
    stub = tmp_path / "rocprofv3"
    stub.write_text("#!/bin/bash\necho \"$@\" > \"$(dirname $0)/argv_$RANK\"\n")
    stub.chmod(0o755)
    env = dict(os.environ, PATH=f"{tmp_path}:{os.environ['PATH']}")
    r = subprocess.run([RUN, "-np", "2", "--profile", str(tmp_path / "prof"), "--no-python", "true"],
                       capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0, r.stderr
    for rank in (0, 1):
        argv = (tmp_path / f"argv_{rank}").read_text().split()
        assert argv[argv.index("-d") + 1].endswith(f"prof/rank{rank}")
        assert argv[argv.index("--") + 1:] == ["true"]


def test_daemon_debug_wrappers(tmp_path, monkeypatch):
    """CLOUDTIK_<PROC>_VALGRIND / _GDB / _PERFTOOLS_PROFILER / jemalloc wrap a daemon's argv
    (reference services.py:246-339); a requested tool that is missing fails loudly."""
    from cloudtik_amd.core import services
    monkeypatch.setenv("CLOUDTIK_SESSION_DIR", str(tmp_path / "session"))
    for tool in ("valgrind", "gdb", "tmux"):
        f = tmp_path / tool
        f.write_text("#!/bin/sh\n")
        f.chmod(0o755)
    monkeypatch.setenv("PATH", f"{tmp_path}:{os.environ['PATH']}")
    env = {"CLOUDTIK_STATE_SERVER_VALGRIND": "1"}
    argv = services.wrap_command("state_server", ["/bin/server", "--port", "1"], env)
    assert argv[0].endswith("valgrind") and argv[-3:] == ["/bin/server", "--port", "1"]
    env = {"CLOUDTIK_CONTROLLER_GDB": "1"}
    argv = services.wrap_command("controller", ["python", "-m", "x"], env)
    assert argv[0].endswith("tmux") and "gdb" in argv[-1] and "cloudtik_controller" in argv
    env = {"CLOUDTIK_NODE_MONITOR_PERFTOOLS_PROFILER": "1", "PERFTOOLS_PATH": "/lib/libprofiler.so",
           "CLOUDTIK_JEMALLOC_PATH": "/lib/libjemalloc.so", "CLOUDTIK_JEMALLOC_PROFILE": "node_monitor"}
    argv = services.wrap_command("node_monitor", ["python"], env)
    assert argv == ["python"] and env["LD_PRELOAD"].split() == ["/lib/libprofiler.so", "/lib/libjemalloc.so"]
    assert env["CPUPROFILE"].endswith("node_monitor.prof") and "prof:true" in env["MALLOC_CONF"]
    monkeypatch.setenv("PATH", "/nonexistent")
    import pytest
    with pytest.raises(RuntimeError, match="valgrind"):
        services.wrap_command("x", ["y"], {"CLOUDTIK_X_VALGRIND": "1"})
