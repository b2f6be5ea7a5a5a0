"""PgBouncer / pgpool-II backends from service discovery (runtime/pooler_discovery.py;
reference runtime/pgbouncer/discovery.py:12-52, pgbouncer/utils.py:119-205,
pgbouncer/scripting.py:311-344, runtime/pgpool/discovery.py:12-64, pgpool/scripting.py:108-160).
A fake discovery source and a recording reload runner."""
import json
import os

import pytest

from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.runtime import pooler_discovery as PD


class Source:
    def __init__(self, rows):
        self.rows = rows

    def __call__(self):
        return list(self.rows)


def _pg(name, host, port=5432, cluster="c2"):
    return {"name": name, "host": host, "port": port, "meta": {"cloudtik-cluster": cluster,
                                                                 "cloudtik-runtime": "postgres"}}


class R:
    def __init__(self, rc=0):
        self.returncode = rc


def test_config_mode_resolution():
    assert PD.resolve_config_mode({"databases": {"a": {}}}, ["consul"]) == "static"
    assert PD.resolve_config_mode({}, ["postgres", "pgbouncer"]) == "local"
    assert PD.resolve_config_mode({}, ["consul", "pgbouncer"]) == "dynamic"
    assert PD.resolve_config_mode({"config_mode": "dynamic"}, ["consul"]) == "dynamic"
    with pytest.raises(ValueError):
        PD.resolve_config_mode({"config_mode": "dynamic"}, ["pgbouncer"])       # nothing to discover with
    with pytest.raises(ValueError):
        PD.resolve_config_mode({"config_mode": "automatic"}, [])


def test_pgbouncer_databases_follow_postgres_services(tmp_path):
    conf = tmp_path / "pgbouncer.ini"
    conf.write_text(PD.pgbouncer_ini({"fixed": "host=10.9.9.9 port=5432"},
                                     {"listen_port": 6432, "pool_mode": "transaction"}))
    src = Source([_pg("orders-db", "10.0.0.2"), _pg("orders-db", "10.0.0.3"), _pg("users", "10.0.1.2", 5433)])
    ran = []
    job = PD.DiscoverPgBouncerBackends(conf_path=str(conf), query=src, runner=lambda c: ran.append(c) or R(),
                                       reload_cmd="RELOAD", database={"user": "app", "dbname": "prod"})
    job.static = {"fixed": "host=10.9.9.9 port=5432"}
    job.pull()
    text = conf.read_text()
    assert "orders_db = host=10.0.0.2,10.0.0.3 port=5432 dbname=prod user=app" in text
    assert "users = host=10.0.1.2 port=5433 dbname=prod user=app" in text
    assert "fixed = host=10.9.9.9 port=5432" in text                       # static entries kept
    assert "[pgbouncer]\nlisten_port = 6432\npool_mode = transaction" in text   # settings untouched
    assert ran == ["RELOAD"]
    job.pull()
    assert ran == ["RELOAD"]                                               # unchanged: no reload
    src.rows = src.rows[:1] + src.rows[2:]                                 # a server goes away
    job.pull()
    assert "orders_db = host=10.0.0.2 port=5432" in conf.read_text() and len(ran) == 2
    src.rows = src.rows[:1]                                                # a service goes away
    job.pull()
    assert "users =" not in conf.read_text() and len(ran) == 3


def test_pgbouncer_failed_reload_is_retried(tmp_path):
    conf = tmp_path / "pgbouncer.ini"
    conf.write_text(PD.pgbouncer_ini({}, {"listen_port": 6432}))
    rcs = [1, 0]
    ran = []
    job = PD.DiscoverPgBouncerBackends(conf_path=str(conf), query=Source([_pg("db", "10.0.0.2")]),
                                       runner=lambda c: ran.append(c) or R(rcs.pop(0)), reload_cmd="RELOAD")
    with pytest.raises(RuntimeError):
        job.pull()
    # the file was written but the reload failed: the next pull reloads although the file is
    # already current (the set is unchanged since), then the job is idle
    job.pull()
    assert len(ran) == 2 and job.reloads == 1
    job.pull()
    assert len(ran) == 2


def test_pgpool_appends_new_backends(tmp_path):
    conf = tmp_path / "pgpool.conf"
    conf.write_text("port = 6432\n" + "\n".join(PD.pgpool_backend_lines(0, "10.0.0.2", 5432)) + "\n")
    src = Source([_pg("pg", "10.0.0.2"), _pg("pg", "10.0.0.3")])
    ran = []
    job = PD.DiscoverPgpoolBackends(conf_path=str(conf), query=src, runner=lambda c: ran.append(c) or R(),
                                    reload_cmd="pgpool reload")
    job.pull()
    assert PD.pgpool_backends(conf.read_text()) == [("10.0.0.2", 5432), ("10.0.0.3", 5432)]
    assert "backend_flag1 = 'ALLOW_TO_FAILOVER'" in conf.read_text() and ran == ["pgpool reload"]
    src.rows = [_pg("pg", "10.0.0.3"), _pg("pg", "10.0.0.4", 5433)]       # 10.0.0.2 gone, .4 new
    job.pull()
    # numbering kept (pgpool addresses backends by index); only the new server appended
    assert PD.pgpool_backends(conf.read_text()) == [("10.0.0.2", 5432), ("10.0.0.3", 5432), ("10.0.0.4", 5433)]
    assert len(ran) == 2
    job.pull()
    assert len(ran) == 2


def _render(name, cfg, monkeypatch, tmp_path, runtimes):
    for k, v in {"RUNTIME_PATH": str(tmp_path), "CLOUDTIK_NODE_IP": "10.0.0.1", "CLOUDTIK_HEAD_IP": "10.0.0.1",
                 "CLOUDTIK_CLUSTER": "c1", "CLOUDTIK_RUNTIMES": runtimes}.items():
        monkeypatch.setenv(k, v)
    rt = rf.get_runtime(name, cfg)
    return rt, {os.path.relpath(p, tmp_path): t for p, t in rt.render(True).items()}


def test_pooler_runtimes_config_modes(tmp_path, monkeypatch):
    rt, f = _render("pgbouncer", {}, monkeypatch, tmp_path / "a", "postgres,pgbouncer")
    assert "* = host=10.0.0.1 port=5432" in f["pgbouncer/pgbouncer.ini"] and "pgbouncer/discovery.json" not in f
    assert not any("service-daemon" in s for s in rt.start_steps(True))
    rt, f = _render("pgbouncer", {"backend": {"databases": {"app": {"host": "10.5.0.1", "dbname": "a"}}}},
                    monkeypatch, tmp_path / "b", "consul,pgbouncer")
    assert "app = host=10.5.0.1 port=5432 dbname=a" in f["pgbouncer/pgbouncer.ini"]
    rt, f = _render("pgbouncer", {"backend": {"service_selector": {"clusters": ["c2"]},
                                              "database": {"user": "app"}}}, monkeypatch, tmp_path / "c",
                    "consul,pgbouncer")
    d = json.loads(f["pgbouncer/discovery.json"])
    assert d["service_selector"] == {"clusters": ["c2"]} and d["database"] == {"user": "app"}
    assert d["conf_path"].endswith("pgbouncer/pgbouncer.ini") and "kill -HUP" in d["reload_cmd"]
    assert any("service-daemon start pgbouncer-discovery" in s and "DiscoverPgBouncerBackends" in s
               for s in rt.start_steps(True))
    assert any("service-daemon stop pgbouncer-discovery" in s for s in rt.stop_steps(True))

    rt, f = _render("pgpool", {"backend": {"servers": ["10.6.0.1:5432", "10.6.0.2"]}}, monkeypatch,
                    tmp_path / "d", "pgpool")
    assert PD.pgpool_backends(f["pgpool/pgpool.conf"]) == [("10.6.0.1", 5432), ("10.6.0.2", 5432)]
    assert "backend_flag0 = 'ALWAYS_PRIMARY'" in f["pgpool/pgpool.conf"]
    rt, f = _render("pgpool", {"backend": {"config_mode": "dynamic"}}, monkeypatch, tmp_path / "e", "consul,pgpool")
    assert PD.pgpool_backends(f["pgpool/pgpool.conf"]) == []
    assert "pgpool reload" in json.loads(f["pgpool/discovery.json"])["reload_cmd"]
    assert any("DiscoverPgpoolBackends" in s for s in rt.start_steps(True))
