"""Database runtimes that actually replicate (runtime/replication.py, runtime/redis_cluster.py;
reference runtime/mysql/scripts/mysql.sh:340-402 + mysql-init.sh, postgres/scripts/postgres.sh:
515-533 + repmgr*.sh, mongodb/scripts/mongodb.sh:600-680 + mongodb-sharding.sh,
redis/scripting.py:94-243 + scripts/redis-sentinel.sh).

The reference tests its control plane with a mock process runner that records every shell
command (tests/unit/test_cloudtik.py:91-205); these tests do the same for the node-side start
of each database runtime: ``node_services("start", head)`` runs with ``subprocess.run``
replaced by a recorder, per node role, and the recorded commands are checked.  The Redis
Cluster protocol (bootstrap, meet, role, re-shard with key migration) runs against an
in-process fake cluster that implements the commands it uses."""
import os
import re
import shlex
import subprocess
import time
import zlib

import pytest
import yaml

from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.runtime import redis_cluster as RC
from cloudtik_amd.runtime.replication import mongo_shard_layout, mysql_group_name

HEAD, W = "10.0.0.1", ["10.0.0.12", "10.0.0.13", "10.0.0.14"]
MEMBERS = ",".join(f"{i + 2}@{ip}" for i, ip in enumerate(W))


def _start(name, rc, head, ip, monkeypatch, tmp_path, seq=None, members_env=None):
    """(recorded start commands, rendered files) of one node."""
    rt = rf.get_runtime(name, rc)
    env = {"RUNTIME_PATH": str(tmp_path), "CLOUDTIK_NODE_IP": ip, "CLOUDTIK_HEAD_IP": HEAD,
           "CLOUDTIK_NODE_SEQ_ID": str(seq or 1), "CLOUDTIK_CLUSTER": "c1"}
    if members_env:
        env[members_env] = MEMBERS
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    files = {os.path.relpath(p, tmp_path): open(p).read() for p in rt.render(head)}
    ran = []

    class R:
        returncode = 0

    import cloudtik_amd.runtime.common.runtime_base as RB
    monkeypatch.setattr(RB.subprocess, "run", lambda cmd, env=None, **kw: ran.append(cmd[-1]) or R())
    rt.node_services("start", head)
    RAW[:] = ran
    return [_decode(c) for c in ran], files


_REAL_RUN = subprocess.run    # _start patches subprocess.run (the module attribute) while it records
RAW = []          # the undecoded commands of the last _start (for the bash checks)
_FEED = re.compile(r"printf '%s\\n' ('(?:[^']|'\"'\"')*') \| ")


def _decode(cmd):
    """The SQL fed on stdin (``printf '%s\\n' <quoted> | mysql ...``) shown unquoted, so the
    assertions below read the statements the server receives."""
    return _FEED.sub(lambda m: shlex.split(m.group(1))[0] + "\n| ", cmd)


# ------------------------------------------------------------------------------- MySQL
def test_mysql_source_replica(tmp_path, monkeypatch):
    rc = {"cluster_mode": "replication", "replication_password": "s3cret"}
    head, hf = _start("mysql", rc, True, HEAD, monkeypatch, tmp_path / "h", members_env="MYSQL_MEMBERS")
    assert head[0] == "sudo service mysql start"
    h = "\n".join(head)
    assert "CREATE USER IF NOT EXISTS 'repl_user'@'%' IDENTIFIED BY 's3cret'" in h
    assert "SET SESSION sql_log_bin = 0;" in h and "CHANGE REPLICATION SOURCE" not in h
    assert ".replication-initialized" in h                    # once per node
    work, wf = _start("mysql", rc, False, W[0], monkeypatch, tmp_path / "w", seq=2, members_env="MYSQL_MEMBERS")
    w = "\n".join(work)
    assert work[0] == "sudo service mysql start"
    assert "CHANGE REPLICATION SOURCE TO SOURCE_HOST = '10.0.0.1', SOURCE_PORT = 3306" in w
    assert "SOURCE_AUTO_POSITION = 1" in w and "START REPLICA;" in w
    # the replica waits for the source to accept the replication user before pointing at it
    assert w.index("mysqladmin -h 10.0.0.1") < w.index("CHANGE REPLICATION SOURCE")
    cnf = wf["mysql/conf.d/cloudtik.cnf"]
    assert "server-id = 2" in cnf and "read_only = ON" in cnf and "gtid_mode = ON" in cnf
    assert "read_only" not in hf["mysql/conf.d/cloudtik.cnf"]
    # a standalone server runs on the head only
    assert _start("mysql", {}, False, W[0], monkeypatch, tmp_path / "n", seq=2)[0] == []


def test_mysql_group_replication(tmp_path, monkeypatch):
    rc = {"cluster_mode": "group_replication"}
    head, hf = _start("mysql", rc, True, HEAD, monkeypatch, tmp_path / "h", members_env="MYSQL_MEMBERS")
    work, wf = _start("mysql", rc, False, W[1], monkeypatch, tmp_path / "w", seq=3, members_env="MYSQL_MEMBERS")
    for files in (hf, wf):
        cnf = files["mysql/conf.d/cloudtik.cnf"]
        assert f"group_replication_group_name = {mysql_group_name('c1')}" in cnf
        assert "group_replication_group_seeds = 10.0.0.1:33061,10.0.0.12:33061,10.0.0.13:33061,10.0.0.14:33061" in cnf
        assert "plugin_load_add = group_replication.so" in cnf
    assert "group_replication_local_address = 10.0.0.13:33061" in wf["mysql/conf.d/cloudtik.cnf"]
    h, w = "\n".join(head), "\n".join(work)
    assert "SET GLOBAL group_replication_bootstrap_group = ON;\nSTART GROUP_REPLICATION;" in h
    assert "bootstrap_group = ON" not in w and "START GROUP_REPLICATION;" in w
    for t in (h, w):
        assert "FOR CHANNEL 'group_replication_recovery'" in t and "GROUP_REPLICATION_STREAM" in t


# ------------------------------------------------------------------------------- PostgreSQL
def test_postgres_standby_is_cloned_before_it_starts(tmp_path, monkeypatch):
    rc = {"cluster_mode": "replication", "replication_password": "pw"}
    head, _ = _start("postgres", rc, True, HEAD, monkeypatch, tmp_path / "h")
    h = "\n".join(head)
    assert head[0] == "sudo service postgresql start"
    assert "CREATE ROLE repl_user WITH REPLICATION LOGIN PASSWORD 'pw'" in h and "pg_basebackup" not in h
    work, wf = _start("postgres", rc, False, W[0], monkeypatch, tmp_path / "w", seq=2)
    i_clone = next(i for i, c in enumerate(work) if "pg_basebackup" in c)
    i_start = work.index("sudo service postgresql start")
    assert i_clone < i_start                                    # a standby, never a second primary
    clone = work[i_clone]
    assert "-h 10.0.0.1 -p 5432 -U repl_user" in clone and "-X stream -R" in clone
    assert '[ -f "$D/standby.signal" ] ||' in clone            # skipped once it is a standby
    assert "pg_isready -h 10.0.0.1" in clone                    # waits for the primary
    assert "CREATE ROLE" not in "\n".join(work)
    assert "hot_standby = on" in wf["postgres/conf.d/cloudtik.conf"]


def test_postgres_repmgr_failover(tmp_path, monkeypatch):
    rc = {"cluster_mode": "replication", "repmgr": {"enabled": True}}
    head, hf = _start("postgres", rc, True, HEAD, monkeypatch, tmp_path / "h")
    h = "\n".join(head)
    assert "CREATE ROLE repmgr WITH SUPERUSER" in h and "primary register --force" in h
    assert "repmgrd -f" in h
    conf = hf["postgres/repmgr.conf"]
    assert "node_id=1" in conf and "failover='automatic'" in conf and "promote_command='repmgr standby promote" in conf
    assert "shared_preload_libraries = 'repmgr'" in hf["postgres/conf.d/cloudtik.conf"]
    work, wf = _start("postgres", rc, False, W[2], monkeypatch, tmp_path / "w", seq=4)
    w = "\n".join(work)
    assert "standby clone --force" in w and "pg_basebackup" not in w
    assert w.index("standby clone") < w.index("sudo service postgresql start") < w.index("standby register")
    assert "node_id=5" in wf["postgres/repmgr.conf"] and "host=10.0.0.14" in wf["postgres/repmgr.conf"]


# ------------------------------------------------------------------------------- MongoDB
def test_mongodb_replica_set(tmp_path, monkeypatch):
    rc = {"cluster_mode": "replication"}
    head, hf = _start("mongodb", rc, True, HEAD, monkeypatch, tmp_path / "h", members_env="MONGODB_MEMBERS")
    h = "\n".join(head)
    assert 'rs.initiate({_id: "c1-rs", members: [{_id: 0, host: "10.0.0.1:27017", priority: 5}]})' in h
    assert "AlreadyInitialized" in h
    work, _ = _start("mongodb", rc, False, W[0], monkeypatch, tmp_path / "w", seq=2, members_env="MONGODB_MEMBERS")
    w = "\n".join(work)
    assert "--host 10.0.0.1 --port 27017" in w and 'rs.add({host: "10.0.0.12:27017"})' in w
    assert "rs.initiate" not in w
    assert yaml.safe_load(hf["mongodb/mongod.conf"])["replication"]["replSetName"] == "c1-rs"


def test_mongodb_sharded_cluster(tmp_path, monkeypatch):
    rc = {"cluster_mode": "sharding", "shard_size": 2}
    members = [(2, W[0]), (3, W[1]), (4, W[2])]
    assert mongo_shard_layout(members, 2, "c1") == [{"name": "c1-shard0", "members": [W[0], W[1]]},
                                                   {"name": "c1-shard1", "members": [W[2]]}]
    head, hf = _start("mongodb", rc, True, HEAD, monkeypatch, tmp_path / "h", members_env="MONGODB_MEMBERS")
    h = "\n".join(head)
    assert head[0].startswith("mongod --fork --config") and "mongod-cfg.conf" in head[0]
    assert "configsvr: true" in h and "mongos --config" in h
    mongos = yaml.safe_load(hf["mongodb/mongos.conf"])
    assert mongos["sharding"]["configDB"] == "c1-cfg/10.0.0.1:27019" and mongos["net"]["port"] == 27017
    # first member of shard 0: initiates its set and registers it with mongos on the head
    p, pf = _start("mongodb", rc, False, W[0], monkeypatch, tmp_path / "p", seq=2, members_env="MONGODB_MEMBERS")
    t = "\n".join(p)
    assert 'rs.initiate({_id: "c1-shard0"' in t and 'sh.addShard("c1-shard0/10.0.0.12:27018")' in t
    assert "--host 10.0.0.1 --port 27017" in t
    conf = yaml.safe_load(pf["mongodb/mongod.conf"])
    assert conf["sharding"]["clusterRole"] == "shardsvr" and conf["replication"]["replSetName"] == "c1-shard0"
    # second member: joins its shard's set through the first member
    s, _ = _start("mongodb", rc, False, W[1], monkeypatch, tmp_path / "s", seq=3, members_env="MONGODB_MEMBERS")
    t = "\n".join(s)
    assert "--host 10.0.0.12 --port 27018" in t and 'rs.add({host: "10.0.0.13:27018"})' in t
    assert "addShard" not in t and "rs.initiate" not in t


# ------------------------------------------------------------------------------- Redis
def test_redis_sentinel_and_cluster_start(tmp_path, monkeypatch):
    rc = {"cluster_mode": "replication", "password": "pw", "sentinel": {"enabled": True}}
    work, wf = _start("redis", rc, False, W[0], monkeypatch, tmp_path / "w", seq=2, members_env="REDIS_MEMBERS")
    sc = wf["redis/sentinel.conf"]
    assert "sentinel monitor c1-master 10.0.0.1 6379 3" in sc          # majority of 4 nodes
    assert "sentinel auth-pass c1-master pw" in sc
    assert any(c.startswith("redis-sentinel ") for c in work)
    rc = {"cluster_mode": "sharding", "sharding": {"replicas_per_master": 1}}
    head, hf = _start("redis", rc, True, HEAD, monkeypatch, tmp_path / "h", members_env="REDIS_MEMBERS")
    join = [c for c in head if "redis_cluster join" in c]
    assert join and "--head" in join[0] and "--replicas-per-master 1" in join[0]
    assert "--seeds 10.0.0.1,10.0.0.12,10.0.0.13,10.0.0.14" in join[0]
    assert "cluster-enabled yes" in hf["redis/redis.conf"]


# ---- an in-process Redis Cluster that implements the commands redis_cluster.py sends
def _slot(key) -> int:
    return zlib.crc32(key if isinstance(key, bytes) else key.encode()) % RC.SLOTS


class FakeCluster:
    def __init__(self):
        self.nodes = {}                  # ip -> FakeNode

    def connect(self, host, port):
        return self.nodes[host]


class FakeNode:
    def __init__(self, cluster, ip, port=6379):
        self.cluster, self.ip, self.port = cluster, ip, port
        self.id = f"{abs(hash(ip)) % (16 ** 12):040x}"
        self.slots, self.master, self.data = set(), None, {}
        self.importing, self.migrating = {}, {}
        self.known = {self.id}
        cluster.nodes[ip] = self

    def _view(self):
        return [n for n in self.cluster.nodes.values() if n.id in self.known]

    def execute(self, *args):
        a = [x.decode() if isinstance(x, bytes) else str(x) for x in args]
        cmd = a[0].upper()
        if cmd == "MIGRATE":
            dst = self.cluster.nodes[a[1]]
            for k in a[a.index("KEYS") + 1:]:
                dst.data[k] = self.data.pop(k)
            return "OK"
        sub = a[1].upper()
        if sub == "MYID":
            return self.id.encode()
        if sub == "NODES":
            lines = []
            for n in self._view():
                flags = ("myself," if n is self else "") + ("slave" if n.master else "master")
                rng = []
                for s in sorted(n.slots):
                    if rng and rng[-1][1] == s - 1:
                        rng[-1][1] = s
                    else:
                        rng.append([s, s])
                toks = [f"{lo}-{hi}" if lo != hi else str(lo) for lo, hi in rng]
                lines.append(f"{n.id} {n.ip}:{n.port}@16379 {flags} {n.master or '-'} 0 0 1 connected {' '.join(toks)}")
            return ("\n".join(lines) + "\n").encode()
        if sub == "MEET":
            other = self.cluster.nodes[a[2]]
            group = self.known | other.known
            for n in self.cluster.nodes.values():      # gossip converges at once
                if n.id in group:
                    n.known = set(group)
            return "OK"
        if sub == "ADDSLOTSRANGE":
            lo, hi = int(a[2]), int(a[3])
            assert not any(lo <= s <= hi for n in self._view() for s in n.slots)
            self.slots |= set(range(lo, hi + 1))
            return "OK"
        if sub == "REPLICATE":
            assert not self.slots
            self.master = a[2]
            return "OK"
        if sub == "GETKEYSINSLOT":
            return [k.encode() for k in self.data if _slot(k) == int(a[2])][: int(a[3])]
        if sub == "SETSLOT":
            s, what = int(a[2]), a[3].upper()
            if what == "IMPORTING":
                self.importing[s] = a[4]
            elif what == "MIGRATING":
                assert s in self.slots
                self.migrating[s] = a[4]
            elif what == "NODE":
                owner = next(n for n in self.cluster.nodes.values() if n.id == a[4])
                for n in self.cluster.nodes.values():
                    n.slots.discard(s)
                owner.slots.add(s)
                self.importing.pop(s, None)
                self.migrating.pop(s, None)
            return "OK"
        raise AssertionError(f"unexpected command {a}")


@pytest.mark.parametrize("replicas,masters", [(0, 4), (1, 2)])
def test_redis_cluster_bootstrap_join_and_reshard(replicas, masters):
    fc = FakeCluster()
    ips = [HEAD] + W
    nodes = [FakeNode(fc, ip) for ip in ips]
    for i in range(500):                          # data written while the head owns everything
        nodes[0].data[f"k{i}"] = i
    roles = []
    for i, ip in enumerate(ips):
        mgr = RC.RedisClusterManager(fc.connect, replicas_per_master=replicas, wait=1, poll=0.01)
        roles.append(mgr.join(ip, ips, head=(i == 0)))
    assert roles[0] == "bootstrap"
    owners = [n for n in nodes if n.slots]
    assert len(owners) == masters and sum(r == "replica" for r in roles) == len(ips) - masters
    covered = sorted(s for n in owners for s in n.slots)
    assert covered == list(range(RC.SLOTS))       # every slot exactly once
    sizes = sorted(len(n.slots) for n in owners)
    assert sizes[-1] - sizes[0] <= masters        # an even share each
    for n in owners:                              # every key moved with its slot
        for k in n.data:
            assert _slot(k) in n.slots
    assert sum(len(n.data) for n in nodes) == 500
    for n in nodes:
        if n.master:
            assert any(m.id == n.master for m in owners)
    # a restarted node does nothing (marker file) -- and the nodes view parses back
    view = RC.parse_nodes(nodes[0].execute("CLUSTER", "NODES"))
    assert sum(len(v.slots) for v in view) == RC.SLOTS


# ------------------------------------------------------------------------------- the steps in bash
_CASES = [
    ("mysql", {"cluster_mode": "replication", "replication_password": "it's"}, "MYSQL_MEMBERS"),
    ("mysql", {"cluster_mode": "group_replication"}, "MYSQL_MEMBERS"),
    ("postgres", {"cluster_mode": "replication", "replication_password": "p'w"}, "POSTGRES_MEMBERS"),
    ("postgres", {"cluster_mode": "replication", "repmgr": {"enabled": True}}, "POSTGRES_MEMBERS"),
    ("mongodb", {"cluster_mode": "replication"}, "MONGODB_MEMBERS"),
]


@pytest.mark.parametrize("name,rc,menv", _CASES)
def test_every_step_parses_in_bash(name, rc, menv, tmp_path, monkeypatch):
    """Every generated start step is a complete bash program (``bash -n``): a step whose SQL
    body or quoting runs past its own end would swallow the rest of the line."""
    for head, ip, seq in ((True, HEAD, 1), (False, W[0], 2)):
        _start(name, rc, head, ip, monkeypatch, tmp_path / f"{head}", seq=seq, members_env=menv)
        assert RAW
        for cmd in RAW:
            r = _REAL_RUN(["bash", "-n", "-c", cmd], capture_output=True, text=True)
            assert r.returncode == 0, (cmd, r.stderr)


_STUBS = {
    "sudo": 'if [ "$1" = -u ]; then shift 2; fi; exec "$@"',
    "mysql": 'cat >> "$LOG"; echo "-- end" >> "$LOG"',
    "psql": 'cat >> "$LOG"; echo "-- end" >> "$LOG"',
    "mysqladmin": "exit 0", "pg_isready": "exit 0", "service": "exit 0", "pgrep": "exit 1",
    "repmgr": 'echo "repmgr $*" >> "$LOG"', "repmgrd": 'echo "repmgrd $*" >> "$LOG"',
    "createdb": "exit 0", "tee": "cat > /dev/null",
}


def _run_stubbed(cmds, tmp_path):
    bind = tmp_path / "bin"
    bind.mkdir()
    for n, body in _STUBS.items():
        (bind / n).write_text("#!/bin/bash\n" + body + "\n")
        (bind / n).chmod(0o755)
    log = tmp_path / "server.log"
    env = dict(os.environ, PATH=f"{bind}:{os.environ['PATH']}", LOG=str(log))
    for cmd in cmds:
        r = _REAL_RUN(["bash", "-c", cmd], capture_output=True, text=True, env=env, timeout=60)
        assert r.returncode == 0, (cmd, r.stderr)
    return log.read_text() if log.exists() else ""


def test_mysql_replica_steps_run(tmp_path, monkeypatch):
    """The replica's steps executed by bash against stub binaries: the server receives the
    user statements and then the CHANGE REPLICATION SOURCE, with a quote in the password kept
    intact; a second run is a no-op (the marker)."""
    rc = {"cluster_mode": "replication", "replication_password": "it's"}
    _start("mysql", rc, False, W[0], monkeypatch, tmp_path / "w", seq=2, members_env="MYSQL_MEMBERS")
    cmds = [c for c in RAW if not c.startswith("sudo service")]
    got = _run_stubbed(cmds, tmp_path)
    assert "IDENTIFIED BY 'it''s';" in got                      # SQL-escaped, shell-intact
    assert got.index("CREATE USER IF NOT EXISTS") < got.index("CHANGE REPLICATION SOURCE TO")
    assert got.rstrip().endswith("START REPLICA;\n-- end".rstrip())
    marker = tmp_path / "w" / "mysql" / ".replication-initialized"
    assert marker.exists()
    (tmp_path / "server.log").unlink()
    import shutil
    shutil.rmtree(tmp_path / "bin")
    assert _run_stubbed(cmds, tmp_path) == ""                  # re-run: nothing sent again


def test_postgres_primary_steps_run(tmp_path, monkeypatch):
    rc = {"cluster_mode": "replication", "repmgr": {"enabled": True}, "replication_password": "p'w"}
    _start("postgres", rc, True, HEAD, monkeypatch, tmp_path / "h", members_env="POSTGRES_MEMBERS")
    cmds = [c for c in RAW if not c.startswith("sudo service")]
    got = _run_stubbed(cmds, tmp_path)
    assert "CREATE ROLE repl_user WITH REPLICATION LOGIN PASSWORD 'p''w';" in got
    assert "repmgr -f" in got and "primary register --force" in got and "repmgrd -f" in got


# ------------------------------------------------------------------------------- Redis with a password
def test_redis_sharding_join_passes_password(tmp_path, monkeypatch):
    rc = {"cluster_mode": "sharding", "password": "pa ss"}
    head, hf = _start("redis", rc, True, HEAD, monkeypatch, tmp_path / "h", members_env="REDIS_MEMBERS")
    join = [c for c in head if "redis_cluster join" in c]
    assert join and join[0].startswith("REDIS_PASSWORD='pa ss' ")        # env, not argv
    assert "requirepass pa ss" in hf["redis/redis.conf"]


def test_redis_reshard_migrate_authenticates():
    """With a password the key migration carries ``AUTH <pw>`` (the target needs it)."""
    fc = FakeCluster()
    ips = [HEAD, W[0]]
    nodes = [FakeNode(fc, ip) for ip in ips]
    for i in range(50):
        nodes[0].data[f"k{i}"] = i
    sent = []
    orig = FakeNode.execute

    def spy(self, *args):
        a = [str(x) for x in args]
        if a[0] == "MIGRATE":
            sent.append(a)
            assert a[a.index("KEYS") - 2:a.index("KEYS")] == ["AUTH", "pw"]
        return orig(self, *args)

    FakeNode.execute = spy
    try:
        for i, ip in enumerate(ips):
            RC.RedisClusterManager(fc.connect, wait=1, poll=0.01, password="pw").join(ip, ips, head=(i == 0))
    finally:
        FakeNode.execute = orig
    assert sent and sum(len(n.data) for n in nodes) == 50


def _state_server(tmp_path, password):
    import socket
    from cloudtik_amd.core.state.state_client import StateServer
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return StateServer(port=port, data_dir=str(tmp_path), password=password).start()


def test_redis_cluster_against_native_resp_server(tmp_path, monkeypatch):
    """Where redis_cluster.py and the in-tree RESP server (native/state_server) overlap:
    (1) the join's connection authenticates with the password -- without it every probe is
    refused (NOAUTH), which ``_alive`` must read as "not a live member" and not crash on;
    (2) the cluster-wide role lock (``_state_lock``) is a real DistributedLock on the head's
    state server: two concurrent role assignments never overlap."""
    import threading
    from cloudtik_amd.core import constants as C
    from cloudtik_amd.core.state.resp import RespConnection, RespError
    srv = _state_server(tmp_path, "s3cret")
    try:
        def conn(pw):
            return lambda host, port: RespConnection(host, port, pw, timeout=5).connect()

        # authenticated: the server answers (and refuses CLUSTER, which it does not implement)
        ok = RC.RedisClusterManager(conn("s3cret"), port=srv.port)
        with pytest.raises(RespError) as e:
            ok.nodes("127.0.0.1")
        assert "NOAUTH" not in str(e.value)
        bad = RC.RedisClusterManager(conn(None), port=srv.port)
        with pytest.raises(RespError) as e:
            bad.nodes("127.0.0.1")
        assert "NOAUTH" in str(e.value).upper()
        assert not bad._alive("127.0.0.1")
        with pytest.raises(RuntimeError, match="no live redis cluster member"):
            bad.join("10.9.9.9", ["127.0.0.1"], head=False)

        monkeypatch.setenv("CLOUDTIK_HEAD_IP", "127.0.0.1")
        monkeypatch.setenv("CLOUDTIK_STATE_PASSWORD", "s3cret")
        monkeypatch.setattr(C, "CLOUDTIK_DEFAULT_PORT", srv.port)
        spans = []

        def role(i):
            with RC._state_lock("c1.redis.role")():
                t0 = time.monotonic()
                time.sleep(0.2)
                spans.append((t0, time.monotonic()))

        th = [threading.Thread(target=role, args=(i,)) for i in range(3)]
        for t in th:
            t.start()
        for t in th:
            t.join(30)
        spans.sort()
        assert len(spans) == 3
        assert all(spans[i][1] <= spans[i + 1][0] for i in range(2))     # mutually exclusive
        from cloudtik_amd.core.state.lock import LOCK_NAMESPACE
        chk = RespConnection("127.0.0.1", srv.port, "s3cret").connect()
        assert chk.get(f"@namespace_{LOCK_NAMESPACE}:c1.redis.role") is None      # released
    finally:
        srv.stop()
