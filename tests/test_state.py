"""Native state server + client tests (reference: core/_private/state/* used via redis)."""
import json
import socket
import threading
import time

import pytest

from cloudtik_amd.core.state.resp import RespConnection, RespError, encode_command
from cloudtik_amd.core.state.state_client import (ControlState, ScalingStateClient, StateClient,
                                                  StateNodeManager, StateServer, StateTableStore)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def server(tmp_path):
    srv = StateServer(port=_free_port(), data_dir=str(tmp_path), password="secret").start()
    yield srv
    srv.stop()


def test_encode_command():
    assert encode_command("SET", "k", b"v") == b"*3\r\n$3\r\nSET\r\n$1\r\nk\r\n$1\r\nv\r\n"


def test_auth_required(server):
    c = RespConnection("127.0.0.1", server.port, password=None).connect()
    with pytest.raises(RespError):
        c.execute("GET", "x")
    assert c.ping()
    assert c.execute("AUTH", "secret") == "OK"
    assert c.get("x") is None


def test_kv_namespaces_and_overwrite(server):
    c = StateClient.create(server.address, "secret")
    assert c.kv_put("k", "v1") == 0
    assert c.kv_put("k", "v2", overwrite=False) == 1
    assert c.kv_get("k") == b"v1"
    assert c.kv_put("k", "v3") == 1
    c.kv_put("k", "other", namespace="ns")
    assert c.kv_get("k") == b"v3" and c.kv_get("k", "ns") == b"other"
    c.kv_put("job:1", "a", namespace="ns")
    c.kv_put("job:2", "b", namespace="ns")
    assert sorted(c.kv_keys("job:", "ns")) == [b"job:1", b"job:2"]
    assert c.kv_del("job:", "ns", del_by_prefix=True) == 2
    assert not c.kv_exists("job:1", "ns")
    assert c.kv_multi_get(["k", "missing"]) == {b"k": b"v3", b"missing": None}
    with pytest.raises(ValueError):
        c.kv_put(b"@namespace_x:y", "z")


def test_binary_values_and_large_payload(server):
    c = StateClient.create(server.address, "secret")
    blob = bytes(range(256)) * 4096 + b"\r\n$-1\r\n"
    c.kv_put("blob", blob)
    assert c.kv_get("blob") == blob


def test_data_types(server):
    c = StateClient.create(server.address, "secret").conn
    assert c.rpush("l", "a", "b", "c") == 3
    assert c.lrange("l", 0, -1) == [b"a", b"b", b"c"]
    assert c.lrange("l", -2, -1) == [b"b", b"c"]
    c.ltrim("l", 1, -1)
    assert c.execute("LLEN", "l") == 2
    assert c.execute("LPOP", "l") == b"b"
    assert c.hset("h", "f", "1") == 1
    assert c.execute("HINCRBY", "h", "f", 4) == 5
    assert c.hgetall("h") == {b"f": b"5"}
    assert c.incr("n", 3) == 3 and c.incr("n") == 4
    with pytest.raises(RespError):
        c.execute("LPUSH", "n", "x")  # WRONGTYPE
    c.set("t", "1", ex=100)
    assert 0 < c.execute("TTL", "t") <= 100
    c.execute("SET", "p", "1", "PX", "50")
    time.sleep(0.12)
    assert c.get("p") is None
    assert c.execute("TYPE", "h") == "hash"
    assert c.execute("DBSIZE") >= 3
    assert c.config_get("port")["port"] == str(server.port)
    assert b"id=" in c.execute("CLIENT", "LIST")


def test_pipeline(server):
    c = StateClient.create(server.address, "secret").conn
    out = c.pipeline([("SET", f"k{i}", i) for i in range(100)] + [("GET", "k42"), ("BOGUS",)])
    assert out[100] == b"42" and isinstance(out[101], RespError)


def test_pubsub_and_patterns(server):
    c = StateClient.create(server.address, "secret")
    ps = c.conn.pubsub()
    ps.subscribe("logs")
    ps2 = c.conn.pubsub()
    ps2.psubscribe("ev:*")
    assert c.publish("logs", "line1") == 1
    assert c.publish("ev:node", {"a": 1}) == 1
    assert ps.get_message(2.0) == (b"logs", b"line1")
    ch, data = ps2.get_message(2.0)
    assert ch == b"ev:node" and json.loads(data) == {"a": 1}
    assert ps.get_message(0.05) is None
    ps.close()
    ps2.close()


def test_many_concurrent_clients(server):
    errs = []

    def worker(i):
        try:
            c = StateClient.create(server.address, "secret")
            for j in range(50):
                c.conn.incr("counter")
                c.table_put("t", f"{i}-{j}", {"i": i})
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(16)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs
    c = StateClient.create(server.address, "secret")
    assert int(c.conn.get("counter")) == 800
    assert len(c.table_get_all("t")) == 800


def test_snapshot_persistence(tmp_path):
    port = _free_port()
    with StateServer(port=port, data_dir=str(tmp_path)) as s:
        c = StateClient.create(s.address)
        c.kv_put("persist", "yes")
        c.table_put("node_table", "n1", {"ip": "10.0.0.1"})
        c.conn.rpush("q", "1", "2")
        c.save()
    with StateServer(port=port, data_dir=str(tmp_path)) as s:
        c = StateClient.create(s.address)
        assert c.kv_get("persist") == b"yes"
        assert c.table_get("node_table", "n1") == {"ip": "10.0.0.1"}
        assert c.conn.lrange("q") == [b"1", b"2"]


def test_control_state_tables_and_scaling(server):
    cs = ControlState(server.address, "secret")
    nm = StateNodeManager(cs.tables)
    nm.register_node("n1", {"node_ip": "10.0.0.1", "node_type": "worker"})
    nm.heartbeat("n1", {"resources": {"GPU": 8}})
    assert cs.get_node_table().get("n1")["resources"] == {"GPU": 8}
    cs.get_node_metrics_table().put("n1", {"cpu": 0.5})
    sc = ScalingStateClient.create_from(cs)
    hb = sc.get_cluster_heartbeat_state()
    assert hb["n1"]["node_ip"] == "10.0.0.1" and hb["n1"]["last_heartbeat_time"] > 0
    assert sc.get_node_resource_states() == {"n1": {"cpu": 0.5}}
    assert sc.get_scaling_state() is None
    sc.update_scaling_state({"autoscaling_instructions": {"resource_demands": [{"GPU": 8}]}})
    assert sc.get_scaling_state()["autoscaling_instructions"]["resource_demands"] == [{"GPU": 8}]
    nm.drain_node("n1")
    assert nm.get_node_table() == {}
    assert isinstance(StateTableStore(cs.client).get_user_state_table("x").get_all(), dict)


def test_protocol_error_closes_connection(server):
    s = socket.create_connection(("127.0.0.1", server.port))
    s.sendall(b"*1\r\n+bad\r\n")
    data = s.recv(1024)
    assert data.startswith(b"-ERR")
    s.close()
    # server still healthy
    assert StateClient.create(server.address, "secret").ping()


def test_distributed_lock_and_leader_election(server):
    from cloudtik_amd.core.state.lock import DistributedLock, LeaderElection
    c1 = StateClient.create(server.address, "secret")
    c2 = StateClient.create(server.address, "secret")
    a = DistributedLock(c1, "job", ttl_ms=300)
    b = DistributedLock(c2, "job", ttl_ms=300)
    assert a.acquire(blocking=False) and not b.acquire(blocking=False)
    assert not b.release()                 # cannot release someone else's lease
    assert a.renew() and a.owner() == a.token
    time.sleep(0.45)                        # lease expires without renewal
    assert b.acquire(blocking=False) and not a.renew()
    assert b.release() and a.acquire(timeout=1)
    a.release()
    events = []
    e1 = LeaderElection(c1, "ctl", "node-1", ttl_ms=300, on_elected=lambda: events.append("1+"),
                        on_demoted=lambda: events.append("1-"))
    e2 = LeaderElection(c2, "ctl", "node-2", ttl_ms=300, on_elected=lambda: events.append("2+"))
    e1.step()
    e2.step()
    assert e1.is_leader() and not e2.is_leader() and e2.leader() == "node-1"
    e1.resign()                              # hand over
    e2.step()
    assert e2.is_leader() and events == ["1+", "1-", "2+"]


def test_state_server_under_asan_ubsan(tmp_path):
    """The state server built with -fsanitize=address,undefined serves a
    concurrent KV / table / list / pub-sub / snapshot workload and exits without a report."""
    import os
    log = tmp_path / "asan.log"
    os.environ.setdefault("ASAN_OPTIONS", "detect_leaks=1:abort_on_error=0")
    srv = StateServer(port=_free_port(), data_dir=str(tmp_path), password="pw", log_file=str(log),
                      sanitize=True).start(wait=60)
    try:
        errs = []

        def worker(i):
            try:
                c = StateClient.create(srv.address, "pw")
                for j in range(30):
                    c.conn.incr("n")
                    c.table_put("t", f"{i}-{j}", {"v": "x" * (j * 97)})
                    c.conn.rpush("l", str(j))
                c.table_get_all("t")
            except Exception as e:  # pragma: no cover
                errs.append(e)
        sub = StateClient.create(srv.address, "pw")
        ps = sub.conn
        ps.execute("SUBSCRIBE", "ch")
        ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        pub = StateClient.create(srv.address, "pw")
        pub.conn.execute("PUBLISH", "ch", "hello")
        pub.save()
        assert not errs
        assert int(pub.conn.get("n")) == 240
    finally:
        srv.stop()
    text = log.read_text(errors="replace") if log.exists() else ""
    assert "AddressSanitizer" not in text and "runtime error" not in text, text[-3000:]
