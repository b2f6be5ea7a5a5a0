"""Script registry, data API and head REST requests (CPU)."""
import http.server
import importlib.util
import json
import threading

import pytest

from cloudtik_amd.core import cluster_tunnel_request as ctr
from cloudtik_amd.core.script_registry import get_registered_script, registry
from cloudtik_amd.runtime.ai.data import DataAPIType, get_data_api


def test_script_registry_aliases_resolve_to_modules():
    reg = registry()
    assert reg["ai.launch"] == "cloudtik_amd.runner.launch"
    for alias, module in reg.items():
        assert importlib.util.find_spec(module) is not None, alias
    assert get_registered_script("no.such.alias") is None


def test_data_api():
    api = get_data_api()
    assert api.native and api.pandas().DataFrame({"a": [1]}).shape == (1, 1)
    assert get_data_api("spark").api_type is DataAPIType.SPARK
    assert not get_data_api("modin").native
    with pytest.raises(ValueError):
        get_data_api("dask")


def test_rest_direct_and_tunnel_command():
    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            body = json.dumps({"path": self.path}).encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    try:
        out = ctr.request_rest_direct("127.0.0.1", srv.server_address[1], "/api/v1/status")
        assert json.loads(out) == {"path": "/api/v1/status"}
    finally:
        srv.shutdown()
    cmd = ctr.ssh_tunnel_command({"ssh_user": "ops", "ssh_port": 2222, "ssh_private_key": "/k",
                                  "ssh_proxy_command": "nc -X 5 -x proxy:1080 %h %p"},
                                 "1.2.3.4", 5555, "10.0.0.1", 8265)
    assert cmd[-1] == "ops@1.2.3.4" and "127.0.0.1:5555:10.0.0.1:8265" in cmd
    assert "ProxyCommand=nc -X 5 -x proxy:1080 1.2.3.4 2222" in cmd and ["-i", "/k"] == cmd[cmd.index("-i"):][:2]
