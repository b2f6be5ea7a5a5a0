"""Role-aware health checks (runtime/common/health_check.py; reference
runtime/common/health_check.py + xinetd health-check services): role probes for MySQL /
Postgres / Redis / HDFS from canned CLI output, the xinetd HTTP responder, and the xinetd
runtime rendering one service per runtime with a health_check_port."""
import io
import os

from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.runtime.common.health_check import check, respond


def _render(name, rc, env, head=False, monkeypatch=None, tmp_path=None):
    """Render one runtime's files on a node with ``env`` (same helper as
    tests/test_configured_runtimes.py, kept local: no test module imports another)."""
    rt = rf.get_runtime(name, rc)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("RUNTIME_PATH", str(tmp_path))
    if rt.spec.home_env:
        monkeypatch.setenv(rt.spec.home_env, str(tmp_path / name))
    out = rt.render(head)
    return {os.path.relpath(p, tmp_path): open(p).read() for p in out}


def runner(outputs):
    def run(cmd):
        for key, (rc, out) in outputs.items():
            if key in cmd:
                return rc, out
        return 1, ""
    return run


def test_roles():
    assert check("mysql", "/primary", run=runner({"mysql": (0, "0\n")}))[0] == 200
    assert check("mysql", "/primary", run=runner({"mysql": (0, "1\n")}))[0] == 503
    assert check("mysql", "/secondary", run=runner({"mysql": (0, "1\n")}))[0] == 200
    assert check("postgres", "/", run=runner({"psql": (0, "t\n")})) == (200, "postgres secondary\n")
    assert check("redis", "/master", run=runner({"redis-cli": (0, "master\n0\n")}))[0] == 200
    assert check("redis", "/master", run=runner({"redis-cli": (0, "slave\n10.0.0.1\n")}))[0] == 503
    assert check("hdfs", "/active", {"namenode_id": "nn1"}, run=runner({"haadmin": (0, "standby\n")}))[0] == 503
    assert check("mysql", "/", run=runner({}))[0] == 503                     # server down


def test_xinetd_responder_and_runtime(tmp_path, monkeypatch):
    out = io.StringIO()
    respond("mysql", io.StringIO("GET /primary HTTP/1.1\r\n"), out, run=runner({"mysql": (0, "0\n")}))
    assert out.getvalue().startswith("HTTP/1.1 200 OK\r\n") and out.getvalue().endswith("mysql primary\n")
    cfg = {"runtime": {"types": ["mysql", "xinetd"], "mysql": {"health_check_port": 9201, "port": 3307},
                       "redis": {}}}
    env = rf.get_runtime("xinetd", {}).with_environment_variables(cfg, None, None)
    files = _render("xinetd", {}, env, monkeypatch=monkeypatch, tmp_path=tmp_path)
    svc = files["xinetd/mysql-health-check"]
    assert "port = 9201" in svc and "server_args = -m cloudtik_amd.runtime.common.health_check mysql --port 3307" in svc
    assert list(files) == ["xinetd/mysql-health-check"]


def test_haproxy_probes_the_role_health_check(tmp_path, monkeypatch):
    cfg = {"backend": {"servers": ["10.0.0.12:3306", "10.0.0.13:3306"], "health_check_port": 9201,
                       "health_check_path": "/primary"}, "protocol": "tcp", "port": 3306}
    text = _render("haproxy", cfg, {}, head=True, monkeypatch=monkeypatch, tmp_path=tmp_path)["haproxy/haproxy.cfg"]
    assert "option httpchk GET /primary" in text and "server s1 10.0.0.13:3306 check port 9201" in text
