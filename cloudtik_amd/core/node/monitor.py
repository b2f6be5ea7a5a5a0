"""Per-node agent (reference core/_private/node/node_monitor.py:NodeMonitor and
core/_private/log_monitor.py:LogMonitor, merged into one lightweight process).

Every ``CLOUDTIK_HEARTBEAT_PERIOD_SECONDS`` it writes the node's heartbeat (ip, kind,
static resources -- CPU / memory / GPU count / ``accelerator_type:MI355X``) into the node
table; every ``--metrics-period`` seconds the sampled load (CPU, memory, per-GPU busy %,
VRAM, temperature, power) into the node-metrics table and the node's daemon list into the
node-processes table.  New lines of the session logs are published on the log channel so
``cloudtik monitor`` can follow them from anywhere.

    python -m cloudtik_amd.core.node.monitor --address HEAD:6789 --node-ip IP [--head]
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import time
from typing import Dict, Optional

from cloudtik_amd.core import constants as C
from cloudtik_amd.core.node.metrics import NodeMetricsCollector
from cloudtik_amd.core.state.state_client import (LOG_CHANNEL, NODE_METRICS_TABLE, NODE_PROCESSES_TABLE,
                                                  NODE_TABLE, StateClient)

logger = logging.getLogger(__name__)


class LogTailer:
    """Follows every file in a directory, returning new complete lines."""

    def __init__(self, directory: str, max_lines: int = C.LOG_MONITOR_NUM_LINES_TO_READ):
        self.dir = directory
        self.max_lines = max_lines
        self.pos: Dict[str, int] = {}

    def poll(self):
        out = []
        try:
            names = sorted(os.listdir(self.dir))
        except OSError:
            return out
        for fn in names[:C.LOG_MONITOR_MAX_OPEN_FILES]:
            path = os.path.join(self.dir, fn)
            if not os.path.isfile(path):
                continue
            size = os.path.getsize(path)
            start = self.pos.get(path)
            if start is None:
                start = max(0, size - 4096)     # do not replay old history on (re)start
            if size < start:
                start = 0                       # rotated / truncated
            if size == start:
                self.pos[path] = start
                continue
            with open(path, "rb") as f:
                f.seek(start)
                data = f.read(1 << 20)
            cut = data.rfind(b"\n")
            if cut < 0:
                self.pos[path] = start
                continue
            self.pos[path] = start + cut + 1
            for line in data[:cut].split(b"\n")[-self.max_lines:]:
                out.append((fn, line.decode(errors="replace")))
        return out


class NodeMonitor:
    def __init__(self, address: str, node_ip: str, head: bool = False, node_id: Optional[str] = None,
                 resources: Optional[Dict] = None, logs_dir: Optional[str] = None,
                 password: Optional[str] = None, metrics_period: float = 5.0):
        self.address = address
        self.node_ip = node_ip
        self.node_id = node_id or os.environ.get(C.CLOUDTIK_RUNTIME_ENV_NODE_ID) or node_ip
        self.head = head
        if resources is None:
            from cloudtik_amd.core.resources import detect_resources
            resources = detect_resources()
        self.resources = resources
        self.client = StateClient.create(address, password, client_name=f"node-monitor-{self.node_id}")
        self.collector = NodeMetricsCollector()
        self.tailer = LogTailer(logs_dir) if logs_dir else None
        self.metrics_period = metrics_period
        self._stop = False
        self._last_metrics = 0.0
        self.started = time.time()

    def stop(self, *_):
        self._stop = True

    def heartbeat(self):
        self.client.table_put(NODE_TABLE, self.node_id, {
            "node_id": self.node_id, "node_ip": self.node_ip,
            "node_kind": "head" if self.head else "worker",
            "node_type": os.environ.get(C.CLOUDTIK_RUNTIME_ENV_NODE_TYPE, ""),
            "resources": self.resources, "last_heartbeat_time": time.time(),
            "start_time": self.started, "state": "RUNNING"})

    def report_metrics(self):
        from cloudtik_amd.core import services
        m = self.collector.collect()
        m["node_ip"] = self.node_ip
        m["resources"] = self.resources
        self.client.table_put(NODE_METRICS_TABLE, self.node_id, m)
        procs = {n: {"pid": i["pid"], "alive": i["alive"]} for n, i in services.list_processes().items()}
        self.client.table_put(NODE_PROCESSES_TABLE, self.node_id,
                              {"node_ip": self.node_ip, "processes": procs, "time": time.time()})

    def publish_logs(self):
        if self.tailer is None:
            return
        lines = self.tailer.poll()
        if lines:
            self.client.publish(LOG_CHANNEL, json.dumps({"ip": self.node_ip, "lines": lines}))

    def run(self, max_iterations: Optional[int] = None):
        i = 0
        while not self._stop:
            try:
                self.heartbeat()
                if time.time() - self._last_metrics >= self.metrics_period:
                    self.report_metrics()
                    self._last_metrics = time.time()
                self.publish_logs()
            except (ConnectionError, OSError) as e:
                logger.warning("state service unreachable: %s", e)
            i += 1
            if max_iterations is not None and i >= max_iterations:
                break
            time.sleep(C.CLOUDTIK_HEARTBEAT_PERIOD_SECONDS)
        try:
            self.client.table_delete(NODE_TABLE, self.node_id)
        except (ConnectionError, OSError):
            pass


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--node-ip", required=True)
    ap.add_argument("--head", action="store_true")
    ap.add_argument("--resources", default=None, help="JSON resource dict (default: detected)")
    ap.add_argument("--logs-dir", default=None)
    ap.add_argument("--metrics-period", type=float, default=5.0)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format=C.LOGGER_FORMAT)
    mon = NodeMonitor(a.address, a.node_ip, a.head,
                      resources=json.loads(a.resources) if a.resources else None,
                      logs_dir=a.logs_dir, password=os.environ.get("CLOUDTIK_STATE_PASSWORD") or None,
                      metrics_period=a.metrics_period)
    signal.signal(signal.SIGTERM, mon.stop)
    signal.signal(signal.SIGINT, mon.stop)
    mon.run()


if __name__ == "__main__":
    main()
