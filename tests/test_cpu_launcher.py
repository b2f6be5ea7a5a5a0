"""CPU launching (runner/cpu.py + launchers.CpuLauncher): topology parsing, the core-pool
scheduler's placement modes, allocator / OpenMP-runtime environments and an end-to-end
`cloudtik-run --launcher cpu` job (reference runtime/ai/runner/cpu/cpu_pool.py,
cpu_launcher.py, local_launcher.py)."""
import json
import os
import subprocess
import sys
import types

import pytest

from cloudtik_amd.runner import cpu as C

# 2 sockets = 2 NUMA nodes, 4 cores each, 2 hardware threads per core (siblings = cpu + 8)
LSCPU = "# CPU,Core,Socket,Node\n" + "\n".join(
    f"{cpu},{cpu % 8},{(cpu % 8) // 4},{(cpu % 8) // 4}" for cpu in range(16))


def _ids(sched):
    return [[c.cpu for c in p] for p in sched]


def test_topology_and_default_schedule():
    s = C.CpuPoolScheduler(lscpu_text=LSCPU)
    assert len(s.pool) == 16 and s.num_sockets() == 2 and s.num_nodes() == 2
    assert [c.cpu for c in s.physical_cores()] == list(range(8))
    assert _ids(s.schedule()) == [[0, 1, 2, 3], [4, 5, 6, 7]]           # one process per node


def test_schedule_modes():
    s = C.CpuPoolScheduler(lscpu_text=LSCPU)
    assert _ids(s.schedule(num_proc=4)) == [[0, 1], [2, 3], [4, 5], [6, 7]]
    assert _ids(s.schedule(ncores_per_proc=3)) == [[0, 1, 2], [3, 4, 5]]                     # crosses nodes
    assert _ids(s.schedule(ncores_per_proc=3, skip_cross_node_cores=True)) == [[0, 1, 2], [4, 5, 6]]
    logical = s.schedule(num_proc=2, use_logical_cores=True)
    assert _ids(logical) == [[0, 1, 2, 3, 8, 9, 10, 11], [4, 5, 6, 7, 12, 13, 14, 15]]
    assert _ids(s.schedule(nodes_list=[1])) == [[4, 5, 6, 7]]
    assert _ids(s.schedule(num_proc=2, cores_list=[0, 8, 1, 9])) == [[0, 1], [8, 9]]
    with pytest.raises(ValueError):
        s.schedule(num_proc=3, ncores_per_proc=4)
    with pytest.raises(ValueError):
        s.schedule(nodes_list=[7])
    # latency / throughput modes override the explicit counts
    a = types.SimpleNamespace(latency_mode=True, throughput_mode=False, num_proc=3, ncores_per_proc=1,
                              use_logical_cores=True, nodes_list="0")
    C.apply_mode(a, s)
    assert (a.num_proc, a.ncores_per_proc, a.use_logical_cores, a.nodes_list) == (0, 4, False, "")
    a = types.SimpleNamespace(latency_mode=False, throughput_mode=True, num_proc=0, ncores_per_proc=2,
                              use_logical_cores=False, nodes_list="")
    C.apply_mode(a, s)
    assert (a.num_proc, a.ncores_per_proc) == (2, 0)
    with pytest.raises(ValueError):
        C.apply_mode(types.SimpleNamespace(latency_mode=True, throughput_mode=True), s)


def test_ranges():
    assert C.ranges([3, 0, 1, 2, 8, 9, 11]) == "0-3,8-9,11"
    assert C.ranges([5]) == "5"


def test_allocator_and_omp_environments(tmp_path):
    libdir = tmp_path / "lib"
    libdir.mkdir()
    (libdir / "libjemalloc.so.2").write_bytes(b"")
    (libdir / "libiomp5.so").write_bytes(b"")
    pre, env, kind = C.allocator_env("auto", benchmark=False, dirs=[str(libdir)])
    assert kind == "jemalloc" and pre == [str(libdir / "libjemalloc.so.2")]
    assert "background_thread:true" in env["MALLOC_CONF"] and "decay" not in env["MALLOC_CONF"]
    assert "dirty_decay_ms:-1" in C.allocator_env("jemalloc", True, [str(libdir)])[1]["MALLOC_CONF"]
    assert C.allocator_env("tcmalloc", dirs=[str(libdir)])[2] == "default"       # not installed
    assert C.allocator_env("default", dirs=[str(libdir)]) == ([], {}, "default")
    pre, env, rt = C.omp_env("auto", [4, 5, 6], dirs=[str(libdir)])
    assert rt == "intel" and pre == [str(libdir / "libiomp5.so")]
    assert env["OMP_NUM_THREADS"] == "3" and env["KMP_AFFINITY"].startswith("granularity=fine")
    pre, env, rt = C.omp_env("default", [4, 5, 6], dirs=[str(libdir)])
    assert rt == "default" and not pre and env["GOMP_CPU_AFFINITY"] == "4 5 6"
    assert "GOMP_CPU_AFFINITY" not in C.omp_env("default", [1, 2], set_affinity=False, dirs=[])[1]


def test_task_prefix(monkeypatch):
    s = C.CpuPoolScheduler(lscpu_text=LSCPU)
    node1 = s.schedule(nodes_list=[1])[0]
    monkeypatch.setattr(C.shutil, "which", lambda name: f"/usr/bin/{name}")
    assert C.task_prefix("auto", node1) == (["numactl", "-C", "4-7", "-m", "1"], "numactl")
    cross = s.schedule(ncores_per_proc=6)[0]
    assert C.task_prefix("numactl", cross)[0] == ["numactl", "-C", "0-5"]          # no membind
    assert C.task_prefix("taskset", node1) == (["taskset", "-c", "4-7"], "taskset")
    assert C.task_prefix("none", node1) == ([], "none")
    monkeypatch.setattr(C.shutil, "which", lambda name: None)
    assert C.task_prefix("auto", node1) == ([], "none")


def test_cpu_flags_forwarded_to_remote_nodes():
    from cloudtik_amd.runner.launch import build_parser
    a = build_parser().parse_args(["--cpu", "--hosts", "h1,h2", "--ncores-per-proc", "8", "--throughput-mode",
                                   "--memory-allocator", "jemalloc", "prog.py", "--x", "1"])
    argv = C.cpu_flags_argv(a)
    assert argv == ["--ncores-per-proc", "8", "--task-manager", "auto", "--throughput-mode",
                    "--memory-allocator", "jemalloc", "--omp-runtime", "auto"]
    from cloudtik_amd.runner.distributor import Distributor
    from cloudtik_amd.runner.launchers import DistributedLauncher
    a.master_addr, a.launcher = "h1", "distributed"
    cmd = DistributedLauncher(a, Distributor(0, 0, 2, "h1,h2", None)).remote_command("h2", 1, 2, 2)
    assert "--launcher cpu" in cmd and "--throughput-mode" in cmd and "--ncores-per-proc 8" in cmd


def test_cloudtik_run_cpu_launcher_end_to_end(tmp_path):
    prog = tmp_path / "probe.py"
    prog.write_text(
        "import json, os, sys\n"
        "out = {'rank': int(os.environ['RANK']), 'world': int(os.environ['WORLD_SIZE']),\n"
        "       'omp': os.environ.get('OMP_NUM_THREADS'), 'cpus': sorted(os.sched_getaffinity(0))}\n"
        "open(sys.argv[1] + '/r%d.json' % out['rank'], 'w').write(json.dumps(out))\n")
    ncpu = len(os.sched_getaffinity(0))
    if ncpu < 4:
        pytest.skip("needs 4 CPUs")
    env = dict(os.environ, PYTHONPATH=os.getcwd())
    env.pop("OMP_NUM_THREADS", None)
    r = subprocess.run([sys.executable, "-m", "cloudtik_amd.runner.launch", "--launcher", "cpu",
                        "--num-proc", "2", "--ncores-per-proc", "2", "--task-manager", "taskset",
                        "--memory-allocator", "default", "--omp-runtime", "default", str(prog), str(tmp_path)],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    res = [json.loads((tmp_path / f"r{i}.json").read_text()) for i in range(2)]
    assert [x["world"] for x in res] == [2, 2] and [x["omp"] for x in res] == ["2", "2"]
    assert all(len(x["cpus"]) == 2 for x in res)
    assert not set(res[0]["cpus"]) & set(res[1]["cpus"])                      # disjoint placements
