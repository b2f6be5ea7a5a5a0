"""Spark runtime API helpers, Consul client (against a fake agent) and the event summarizer."""
import base64
import http.server
import json
import threading

from cloudtik_amd.core.head.event_summarizer import EventSummarizer
from cloudtik_amd.runtime.common.consul import ConsulClient, service_dns_name


def test_event_summarizer():
    s = EventSummarizer()
    s.add("Adding {} node(s) of type gpu", quantity=1)
    s.add("Adding {} node(s) of type gpu", quantity=2)
    s.add("Removing {} idle node(s)", quantity=1)
    s.add_once_per_interval("warn A", "a", 60, now=0)
    s.add_once_per_interval("warn A", "a", 60, now=10)      # throttled
    assert s.summary() == ["Adding 3 node(s) of type gpu", "Removing 1 idle node(s)", "warn A"]
    s.clear()
    s.add_once_per_interval("warn A", "a", 60, now=61)
    assert s.summary() == ["warn A"]


def test_consul_client_against_fake_agent():
    state = {"kv": {}, "services": {}}

    class H(http.server.BaseHTTPRequestHandler):
        def _send(self, obj, code=200):
            body = b"" if obj is None else json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self):
            p = self.path
            if p.startswith("/v1/catalog/services"):
                return self._send({k: v["Tags"] for k, v in state["services"].items()})
            if p.startswith("/v1/catalog/service/"):
                name = p.split("/")[4].split("?")[0]
                svc = state["services"].get(name)
                return self._send([{"Address": "10.0.0.5", "ServiceAddress": svc.get("Address", ""),
                                    "ServicePort": svc["Port"]}] if svc else [])
            if p.startswith("/v1/kv/"):
                k = p[len("/v1/kv/"):]
                if k not in state["kv"]:
                    return self._send(None, 404)
                return self._send([{"Key": k, "Value": base64.b64encode(state["kv"][k]).decode()}])
            self._send(None, 404)

        def do_PUT(self):
            n = int(self.headers.get("Content-Length") or 0)
            body = self.rfile.read(n)
            if self.path == "/v1/agent/service/register":
                d = json.loads(body)
                state["services"][d["Name"]] = d
                return self._send(None)
            if self.path.startswith("/v1/kv/"):
                state["kv"][self.path[len("/v1/kv/"):]] = body
                return self._send(True)
            self._send(None, 404)

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        c = ConsulClient(f"127.0.0.1:{srv.server_address[1]}")
        c.register_service("hdfs-rpc", 8020, address="10.0.0.7", tags=["storage"])
        assert c.services() == {"hdfs-rpc": ["storage"]}
        assert c.service_addresses("hdfs-rpc") == [("10.0.0.7", 8020)]
        assert c.kv_get("missing") is None
        assert c.kv_put("cfg/a", b"1") and c.kv_get("cfg/a") == b"1"
    finally:
        srv.shutdown()
    assert service_dns_name("hdfs-rpc", "storage") == "storage.hdfs-rpc.service.consul"


def test_spark_api_default_storage_from_workspace(monkeypatch):
    from cloudtik_amd.core import service_discovery as sd
    from cloudtik_amd.runtime.common import discovery
    from cloudtik_amd.runtime.spark import api
    svc = sd.define_runtime_service("hdfs", "hdfs-rpc", 8020)
    gv = {sd.service_global_key("storage", "storage-hdfs-rpc"): sd.encode_service_address(svc, "10.9.0.1")}
    monkeypatch.setattr(discovery, "_workspace_global_variables", lambda config: gv)
    monkeypatch.setattr("cloudtik_amd.core.cluster_operator.get_head_node_ip", lambda *a, **k: "10.0.0.1")
    cfg = {"cluster_name": "spark1", "provider": {"type": "local"}, "runtime": {"types": ["spark"]}}
    assert api.get_runtime_default_storage(cfg) == {"default_storage_uri": "hdfs://10.9.0.1:8020"}
