"""cluster-dump depth (core/cluster_dump.py; reference core/_private/cluster/cluster_dump.py
:42-77,227-360,546-758): a node archive holds logs, debug state, pip packages, the process
table and AMD GPU state; the cluster dump selects nodes (--hosts / --head-only), collects them
in parallel, isolates a failing node, and from the CLI host runs the collection on the head."""
import json
import os
import shutil
import tarfile

import pytest

from cloudtik_amd.core import cluster_dump as cd
from cloudtik_amd.core import tags as T


@pytest.fixture
def session(tmp_path, monkeypatch):
    d = tmp_path / "session"
    (d / "logs").mkdir(parents=True)
    (d / "logs" / "cloudtik_cluster_controller.err").write_text("controller log line\n")
    (d / "logs" / cd.DEBUG_STATE_FILE).write_text('{"workers": 2}')
    monkeypatch.setenv("CLOUDTIK_SESSION_DIR", str(d))
    return d


def _fake_sysfs(root):
    node = root / "class" / "kfd" / "kfd" / "topology" / "nodes"
    (node / "0").mkdir(parents=True)
    (node / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    (node / "1").mkdir()
    (node / "1" / "properties").write_text("simd_count 1024\ngfx_target_version 90500\nlocation_id 256\n")
    ras = root / "class" / "drm" / "card1" / "device" / "ras"
    ras.mkdir(parents=True)
    (ras / "umc_err_count").write_text("ue: 0\nce: 3\n")
    return root


def _names(path):
    with tarfile.open(path) as t:
        return set(t.getnames())


def test_node_archive_contents(session, tmp_path):
    sysfs = _fake_sysfs(tmp_path / "sys")
    out = cd.collect_local(cd.DumpParameters(runtimes=["spark"]), str(tmp_path / "n.tar.gz"), sysfs=str(sysfs))
    names = _names(out)
    assert "logs/cloudtik_cluster_controller.err" in names and cd.DEBUG_STATE_FILE in names
    assert "pip_packages.txt" in names and "meta/process_info.txt" in names
    assert "gpu/kfd_topology.json" in names and "gpu/ras_errors.json" in names
    with tarfile.open(out) as t:
        pip = t.extractfile("pip_packages.txt").read().decode()
        topo = json.loads(t.extractfile("gpu/kfd_topology.json").read())
        ras = json.loads(t.extractfile("gpu/ras_errors.json").read())
    assert any(ln.lower().startswith("torch==") for ln in pip.splitlines())
    assert [r["gfx_target_version"] for r in topo] == ["90500"]            # CPU node filtered out
    assert ras["card1"]["umc_err_count"].startswith("ue: 0")
    # switches off
    out2 = cd.collect_local(cd.DumpParameters(logs=False, pip=False, processes=False, gpu=False, debug_state=False),
                            str(tmp_path / "n2.tar.gz"), sysfs=str(sysfs))
    assert _names(out2) == set()


class FakeExecutor:
    """What `cloudtik node dump` on a remote node leaves behind, without ssh."""

    def __init__(self, ip, store, fail=False):
        self.ip, self.store, self.fail, self.cmds = ip, store, fail, []

    def run(self, cmd, timeout=120, **kw):
        self.cmds.append(cmd)
        if self.fail and cmd.startswith("cloudtik node dump --silent"):
            raise OSError("ssh: connect to host timed out")
        if cmd.startswith("cloudtik node dump"):
            remote = cmd.split("--output ")[1].split()[0]
            params = cd.DumpParameters(pip="--no-pip" not in cmd, gpu=False, processes=False)
            self.store[remote] = cd.collect_local(params, remote + f".{self.ip}")

    def run_rsync_down(self, source, target, options=None):
        shutil.copy(self.store[source], target)


def _mock_cluster(name):
    from cloudtik_amd.core.provider_factory import get_node_provider
    from cloudtik_amd.providers.mock.node_provider import MockProvider
    MockProvider.reset(name)
    p = get_node_provider({"type": "mock"}, name, use_cache=False)
    head = next(iter(p.create_node({}, {T.CLOUDTIK_TAG_CLUSTER_NAME: name, T.CLOUDTIK_TAG_NODE_KIND: "head"}, 1)))
    ws = list(p.create_node({}, {T.CLOUDTIK_TAG_CLUSTER_NAME: name, T.CLOUDTIK_TAG_NODE_KIND: "worker"}, 3))
    cfg = {"cluster_name": name, "provider": {"type": "mock"}, "runtime": {"types": ["ai"]},
           "available_node_types": {}, "head_node_type": "head"}
    return cfg, p, head, ws


def test_cluster_dump_selection_parallel_and_failure_isolation(session, tmp_path, monkeypatch):
    cfg, p, head, ws = _mock_cluster("dump-c1")
    monkeypatch.setattr("cloudtik_amd.core.cluster_operator.get_cluster_info", lambda c: {"cluster": c["cluster_name"]})
    store, exs = {}, {}

    def executor_fn(config, provider, node_id):
        ip = provider.internal_ip(node_id)
        exs[ip] = FakeExecutor(ip, store, fail=(node_id == ws[1]))
        return exs[ip]

    out = cd.dump_cluster(cfg, p, cd.DumpParameters(pip=False), str(tmp_path / "all.tar.gz"), executor_fn=executor_fn)
    names = _names(out)
    hip, wips = p.internal_ip(head), [p.internal_ip(w) for w in ws]
    assert f"all/head_{hip}/logs/cloudtik_cluster_controller.err" in names
    assert f"all/worker_{wips[0]}/{cd.DEBUG_STATE_FILE}" in names and f"all/worker_{wips[2]}/logs" in names
    assert not any(n.startswith(f"all/worker_{wips[1]}/") for n in names)         # its dump failed ...
    with tarfile.open(out) as t:
        fails = t.extractfile("all/dump_failures.txt").read().decode()
    assert wips[1] in fails and "timed out" in fails                               # ... and is reported
    assert all("--no-pip" in exs[ip].cmds[0] and "--runtimes=ai" in exs[ip].cmds[0] for ip in wips)
    assert any(c.startswith("rm -f /tmp/cloudtik_dump_worker_") for c in exs[wips[0]].cmds)
    # node selection
    exs.clear()
    cd.dump_cluster(cfg, p, cd.DumpParameters(), str(tmp_path / "h.tar.gz"), head_only=True, executor_fn=executor_fn)
    assert list(exs) == [hip]
    exs.clear()
    cd.dump_cluster(cfg, p, cd.DumpParameters(), str(tmp_path / "s.tar.gz"), hosts=f"{wips[2]},{ws[0]}",
                    executor_fn=executor_fn)
    assert sorted(exs) == sorted([wips[2], wips[0]])


def test_cli_host_runs_the_collection_on_the_head(tmp_path, monkeypatch):
    from cloudtik_amd.core import cluster_operator as op
    cfg, p, head, ws = _mock_cluster("dump-c2")
    cfg["auth"] = {}
    monkeypatch.setattr(op, "_provider", lambda c: p)
    out = op.cluster_dump(cfg, str(tmp_path / "c.tar.gz"), hosts="10.0.0.9", head_only=False,
                          params=cd.DumpParameters(gpu=False))
    cmds = p.runner.commands_for(head)
    run = [c for c in cmds if "cloudtik head cluster-dump" in c]
    assert run and "--no-gpu" in run[0] and "--hosts 10.0.0.9" in run[0] and "--pip" in run[0]
    assert any(c.startswith("rsync-down /tmp/cloudtik_cluster_dump_dump-c2_") and c.endswith(out) for c in cmds)
    assert not any("cloudtik node dump" in c for w in ws for c in p.runner.commands_for(w))


def test_cli_options_reach_the_parameters(monkeypatch, tmp_path):
    from click.testing import CliRunner
    from cloudtik_amd.cli.main import cli
    seen = {}

    def fake(config_file, output=None, include_logs=True, override_cluster_name=None, hosts=None, head_only=False,
             params=None, on_head=False):
        seen.update(hosts=hosts, head_only=head_only, params=params)
        return "x.tar.gz"
    monkeypatch.setattr("cloudtik_amd.core.cluster_operator.cluster_dump", fake)
    r = CliRunner().invoke(cli, ["cluster-dump", "c.yaml", "--hosts", "a,b", "--head-only", "--no-pip",
                                 "--no-processes-verbose", "--runtimes", "spark,hdfs"])
    assert r.exit_code == 0, r.output
    pr = seen["params"]
    assert seen["hosts"] == "a,b" and seen["head_only"] and not pr.pip and pr.logs and pr.gpu
    assert not pr.processes_verbose and pr.runtimes == ["spark", "hdfs"]
