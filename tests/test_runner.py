"""cloudtik-run tests (reference runtime/ai/runner: distributor host parsing, local and
distributed launchers, function-call API)."""
import os
import re
import socket
import subprocess
import sys

import pytest

from cloudtik_amd.runner.affinity import parse_cpulist, rank_cpu_sets
from cloudtik_amd.runner.distributor import Distributor, parse_host, parse_hostfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN = os.path.join(ROOT, "bin", "cloudtik-run")

JOB = """
import os, torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(dist.get_rank())])
dist.all_reduce(t)
line = f"RESULT {dist.get_rank()} {dist.get_world_size()} {os.environ['LOCAL_RANK']} {os.environ['NODE_RANK']} {t.item()}"
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"result_{dist.get_rank()}.txt"), "w").write(line)
dist.destroy_process_group()
"""


def _results(d):
    # gloo prints to stdout from every rank (lines interleave), so ranks write files
    return [open(os.path.join(d, f)).read().split() for f in sorted(os.listdir(d)) if f.startswith("result_")]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_parse_hosts_and_hostfile(tmp_path):
    assert parse_host("10.0.0.1:8").slots == 8
    assert parse_host("node-a slots=4").slots == 4
    assert parse_host("node-b").slots is None
    hf = tmp_path / "hosts"
    hf.write_text("# comment\n10.0.0.1 slots=8\n10.0.0.2:8\n")
    hs = parse_hostfile(str(hf))
    assert [h.host for h in hs] == ["10.0.0.1", "10.0.0.2"] and all(h.slots == 8 for h in hs)


def test_distributor_resolution():
    d = Distributor(hosts="a:8,b:8")
    assert (d.nnodes, d.nproc_per_node, d.num_proc) == (2, 8, 16)
    assert d.host_ranks() == [("a", 0, 8, 0), ("b", 1, 8, 8)]
    d = Distributor(num_proc=12, hosts="a:8,b:8")
    assert d.host_ranks()[1] == ("b", 1, 4, 8)
    d = Distributor(num_proc=4, nproc_per_node=2)
    assert (d.nnodes, d.num_proc, d.nproc_per_node) == (2, 4, 2)
    with pytest.raises(ValueError):
        Distributor(num_proc=20, hosts="a:8,b:8")


def test_affinity_splits_numa_cores():
    assert parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    # 8 GPUs, 4 per socket; 2 sockets x 8 cores
    sets = rank_cpu_sets(8, gpu_numa=[0, 0, 0, 0, 1, 1, 1, 1],
                         cpus_of_node=lambda n: list(range(8 * n, 8 * n + 8)))
    assert sets[0] == [0, 1] and sets[3] == [6, 7] and sets[4] == [8, 9]
    assert len({c for s in sets.values() for c in s}) == 16


def test_local_launcher_allreduce(tmp_path):
    job = tmp_path / "job.py"
    job.write_text(JOB)
    r = subprocess.run([RUN, "--nproc-per-node", "3", "--master-port", str(_port()), str(job)],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    lines = _results(tmp_path)
    assert sorted(int(l[1]) for l in lines) == [0, 1, 2]
    assert all(l[2] == "3" and float(l[5]) == 3.0 for l in lines)


def test_failure_stops_job():
    r = subprocess.run([RUN, "-np", "3", "--no-python", "bash", "-c", "if [ $RANK = 1 ]; then exit 7; fi; sleep 30"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 7


def test_distributed_launcher_two_nodes(tmp_path):
    """Two 'hosts' through a fake remote shell that runs the command locally."""
    job = tmp_path / "job.py"
    job.write_text(JOB)
    rsh = tmp_path / "fake_rsh"
    rsh.write_text('#!/bin/bash\nshift\nexport PATH="%s:$PATH"\nexec bash -c "$1"\n' % os.path.join(ROOT, "bin"))
    rsh.chmod(0o755)
    logs = tmp_path / "logs"
    r = subprocess.run([RUN, "--hosts", "10.255.0.1:2,10.255.0.2:2", "--rsh", str(rsh), "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), "--log-dir", str(logs), str(job)],
                       capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout + r.stderr
    assert len(os.listdir(logs)) == 4            # one log file per rank
    res = _results(tmp_path)
    assert sorted(int(l[1]) for l in res) == [0, 1, 2, 3]
    assert {l[4] for l in res} == {"0", "1"}          # node ranks
    assert all(float(l[5]) == 6.0 for l in res)


def test_run_function_api():
    from cloudtik_amd.runner import run
    out = run(lambda x: (int(os.environ["RANK"]), x * 2), args=(21,), num_proc=2, master_port=_port())
    assert out == [(0, 42), (1, 42)]


def test_cloudtik_rsh_agent_routes_through_head_exec(tmp_path):
    """--rsh cloudtik starts remote node launchers with `cloudtik head exec CMD --node-ip IP`
    (reference runtime/ai/scripts/cloudtik-rsh.sh); a fake cloudtik runs them locally."""
    job = tmp_path / "job.py"
    job.write_text(JOB)
    fake = tmp_path / "fake_cloudtik"
    calls = tmp_path / "calls.txt"
    fake.write_text('#!/bin/bash\n# args: head exec "<cmd>" --node-ip=<ip>\necho "$4" >> %s\n'
                    'export PATH="%s:$PATH"\nexec bash -c "$3"\n' % (calls, os.path.join(ROOT, "bin")))
    fake.chmod(0o755)
    r = subprocess.run([RUN, "--hosts", "10.255.0.3:1,10.255.0.4:1", "--rsh", "cloudtik", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), str(job)], capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, PYTHONPATH=ROOT, CLOUDTIK_BIN=str(fake)))
    assert r.returncode == 0, r.stdout + r.stderr
    assert sorted(calls.read_text().split()) == ["--node-ip=10.255.0.3", "--node-ip=10.255.0.4"]
    assert sorted(int(l[1]) for l in _results(tmp_path)) == [0, 1]


def test_distributed_launcher_terminates_all_hosts_on_failure(tmp_path):
    """A rank failing on one host ends the job on every host (reference rsh_exec.py:196-263):
    the healthy host's ranks (sleeping 120 s) are signalled through the remote shell and the
    launcher returns the failing exit code long before they would have finished."""
    import time
    rsh = tmp_path / "fake_rsh"
    rsh.write_text('#!/bin/bash\nshift\nexport PATH="%s:$PATH"\nexec bash -c "$1"\n' % os.path.join(ROOT, "bin"))
    rsh.chmod(0o755)
    marker = tmp_path / "alive"
    prog = (f"if [ $NODE_RANK = 1 ]; then sleep 2; exit 5; fi; "
            f"trap 'echo terminated > {marker}_$RANK; exit 143' TERM; sleep 120 & wait")
    t0 = time.time()
    r = subprocess.run([RUN, "--hosts", "10.255.0.5:2,10.255.0.6:1", "--rsh", str(rsh), "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), "--no-python", "bash", "-c", prog],
                       capture_output=True, text=True, timeout=100, env=dict(os.environ, PYTHONPATH=ROOT))
    took = time.time() - t0
    assert r.returncode == 5, r.stdout + r.stderr
    assert took < 60, took
    assert "terminating the job on every host" in r.stderr
    time.sleep(1)
    assert sorted(p.name for p in tmp_path.glob("alive_*")) == ["alive_0", "alive_1"]
