#!/usr/bin/env python3
"""On-demand AI job workflow (reference examples/workflows/example-on-demand-ai-job.py):
start a cluster from a config, wait for its workers, submit a training script with a job
waiter, collect the result, and tear the cluster down -- all through the Python API.

    python examples/workflows/on_demand_ai_job.py cluster.yaml examples/ai/mnist_mlp.py --epochs 1

With the ``virtual`` provider the "cluster" is several node sessions on this host, which
makes the workflow runnable anywhere; with ``onpremise`` / ``local`` it drives real
MI355X nodes and the script runs under ``cloudtik-run`` on every GPU.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cluster_config")
    ap.add_argument("script")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    ap.add_argument("--min-workers", type=int, default=None)
    ap.add_argument("--keep", action="store_true", help="leave the cluster running")
    a = ap.parse_args()

    from cloudtik_amd.core.api import Cluster
    from cloudtik_amd.core.event_system import CreateClusterEvent

    cluster = Cluster(a.cluster_config)
    cluster.register_callback(CreateClusterEvent.cluster_booting_completed,
                              lambda ev: print(f"[workflow] head ready: {ev.get('head_node_ip', '')}", flush=True))
    t0 = time.time()
    cluster.start()
    try:
        n = cluster.wait_for_ready(min_workers=a.min_workers, timeout=600)
        print(f"[workflow] {n} worker(s) ready after {time.time() - t0:.1f}s", flush=True)
        print(f"[workflow] nodes: {[x.get('node_ip') for x in cluster.get_nodes()]}", flush=True)
        cluster.submit(a.script, a.script_args, job_waiter="pid")
        print(f"[workflow] job finished after {time.time() - t0:.1f}s", flush=True)
    finally:
        if not a.keep:
            cluster.stop()
            print("[workflow] cluster stopped", flush=True)


if __name__ == "__main__":
    main()
