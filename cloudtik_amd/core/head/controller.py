"""Cluster controller daemon on the head (reference core/_private/cluster/cluster_controller.py
+ cluster_metrics.py + prometheus_metrics.py).

Loads the bootstrapped cluster config, connects to the state service and runs
:class:`ClusterScaler.update` every ``CLOUDTIK_UPDATE_INTERVAL_S`` seconds.  Controller
metrics are exported in Prometheus text format on ``CLOUDTIK_METRIC_PORT`` (nodes by
status / type, pending launches, update duration, failures).

    python -m cloudtik_amd.core.head.controller --address IP:6789 --config ~/cloudtik_bootstrap_config.yaml
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import time
from typing import Optional

import yaml

from cloudtik_amd.core import constants as C
from cloudtik_amd.core.head.scaler import ClusterScaler
from cloudtik_amd.core.provider_factory import get_node_provider
from cloudtik_amd.core.state.state_client import StateClient

logger = logging.getLogger(__name__)


class ControllerMetrics:
    def __init__(self, port: Optional[int] = None):
        try:
            import prometheus_client as pc
        except ImportError:  # pragma: no cover
            self.enabled = False
            return
        self.enabled = True
        self.registry = pc.CollectorRegistry()
        self.workers = pc.Gauge("cloudtik_cluster_workers", "worker nodes by status", ["status"], registry=self.registry)
        self.types = pc.Gauge("cloudtik_cluster_nodes_by_type", "worker nodes by node type", ["node_type"], registry=self.registry)
        self.pending = pc.Gauge("cloudtik_cluster_pending_launches", "pending launches", ["node_type"], registry=self.registry)
        self.update_time = pc.Histogram("cloudtik_cluster_update_seconds", "scaler update duration", registry=self.registry)
        self.failures = pc.Counter("cloudtik_cluster_update_failures", "scaler update failures", registry=self.registry)
        self.demands = pc.Gauge("cloudtik_cluster_resource_demands", "pending resource demand bundles", registry=self.registry)
        if port:
            try:
                pc.start_http_server(port, registry=self.registry)
            except OSError as e:
                logger.warning("metrics port %s unavailable: %s", port, e)

    def observe(self, summary, seconds: float):
        if not self.enabled:
            return
        self.update_time.observe(seconds)
        self.workers.clear()
        for st, nodes in summary["nodes_by_status"].items():
            self.workers.labels(st).set(len(nodes))
        self.types.clear()
        for t, n in summary["nodes_by_type"].items():
            self.types.labels(t).set(n)
        self.pending.clear()
        for t, n in summary["launching"].items():
            self.pending.labels(t).set(n)
        self.demands.set(len(summary["resource_demands"]))


class ClusterController:
    def __init__(self, address: str, config_file: str, password: Optional[str] = None,
                 metrics_port: Optional[int] = C.CLOUDTIK_METRIC_PORT):
        self.config_file = os.path.expanduser(config_file)
        self._mtime = None
        config = self._read_config()
        self.state = StateClient.create(address, password, client_name="cluster-controller")
        self.provider = get_node_provider(config["provider"], config["cluster_name"], use_cache=False)
        self.scaler = ClusterScaler(config, self.provider, self.state, config_reader=self._reload)
        self.metrics = ControllerMetrics(metrics_port)
        self._stop = False

    def _read_config(self):
        self._mtime = os.path.getmtime(self.config_file)
        with open(self.config_file) as f:
            return yaml.safe_load(f)

    def _reload(self):
        try:
            if os.path.getmtime(self.config_file) != self._mtime:
                return self._read_config()
        except OSError:
            pass
        return None

    def stop(self, *_):
        self._stop = True

    def run(self, max_rounds: Optional[int] = None):
        rounds = 0
        while not self._stop:
            t0 = time.time()
            try:
                self.scaler.update()
            except Exception:  # noqa: BLE001
                if self.metrics.enabled:
                    self.metrics.failures.inc()
                logger.exception("controller giving up after repeated failures")
                raise
            dt = time.time() - t0
            try:
                summary = self.scaler.summary()
                self.metrics.observe(summary, dt)
                # the last round's scaler state for `cloudtik cluster-dump` (debug_state.txt)
                from cloudtik_amd.core.cluster_dump import write_debug_state
                write_debug_state(dict(summary, update_seconds=round(dt, 3),
                                       quorum=getattr(self.scaler.quorum, "notifications", [])[-10:]))
            except Exception:  # noqa: BLE001
                pass
            rounds += 1
            if max_rounds is not None and rounds >= max_rounds:
                return
            end = time.time() + C.CLOUDTIK_UPDATE_INTERVAL_S
            while not self._stop and time.time() < end:
                time.sleep(0.2)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--metrics-port", type=int, default=C.CLOUDTIK_METRIC_PORT)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format=C.LOGGER_FORMAT)
    ctl = ClusterController(a.address, a.config, os.environ.get("CLOUDTIK_STATE_PASSWORD") or None,
                            a.metrics_port or None)
    signal.signal(signal.SIGTERM, ctl.stop)
    signal.signal(signal.SIGINT, ctl.stop)
    ctl.run()


if __name__ == "__main__":
    main()
