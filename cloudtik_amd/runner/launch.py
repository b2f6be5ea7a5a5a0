"""``cloudtik-run``: launch a (distributed) training program, one process per MI355X GPU
(reference runtime/ai/runner/launch.py:1-330).

    cloudtik-run train.py --epochs 3                       # all local GPUs, 1 rank each
    cloudtik-run --nproc-per-node 4 train.py               # 4 ranks
    cloudtik-run --hosts 10.0.0.1,10.0.0.2 train.py        # 2 nodes x all GPUs
    cloudtik-run --hostfile hosts --launcher mpi train.py
    cloudtik-run -m package.module args                    # python -m
    cloudtik-run --no-python ./binary args
    cloudtik-run --launcher cpu --throughput-mode infer.py # CPU job: one process per socket
    cloudtik-run --cpu --hosts h1,h2 --ncores-per-proc 8 prep.py   # CPU job on 2 nodes
"""
from __future__ import annotations

import argparse
import os
import sys

from cloudtik_amd.runner.distributor import Distributor
from cloudtik_amd.runner.launchers import create_launcher


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="cloudtik-run", description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--num-proc", "--num_proc", "-np", type=int, default=0, help="Total number of processes.")
    p.add_argument("--nnodes", type=int, default=0, help="Number of nodes.")
    p.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=0,
                   help="Processes per node (default: number of visible GPUs).")
    p.add_argument("--hosts", default="", help="Comma separated hosts, optionally host:slots.")
    p.add_argument("--hostfile", default="", help="File with one 'host [slots=N]' per line.")
    p.add_argument("--master-addr", "--master_addr", default="",
                   help="Rendezvous address (default: the first host, or 127.0.0.1 on one node).")
    p.add_argument("--master-port", "--master_port", type=int, default=29500)
    p.add_argument("--launcher", default="", choices=["", "local", "cpu", "distributed", "rsh", "mpi", "horovod",
                                                      "horovod-local"])
    p.add_argument("--cpu", action="store_true",
                   help="CPU processes placed by the core-pool scheduler (with --hosts: on every node)")
    p.add_argument("--rsh", default=None, help="Remote shell for the rsh/distributed launcher.")
    p.add_argument("--node-rank", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--first-rank", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--local-world", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("-m", "--module", action="store_true", help="Run the program as 'python -m'.")
    p.add_argument("--no-python", "--no_python", action="store_true", help="Execute the program directly.")
    p.add_argument("--log-dir", "--log_dir", default="", help="Write each rank's output to a file here.")
    p.add_argument("--log-file-prefix", "--log_file_prefix", default="run")
    p.add_argument("--no-bind-cpus", dest="bind_cpus", action="store_false",
                   help="Do not pin ranks to their GPU's NUMA-node cores.")
    p.add_argument("--max-restarts", "--max_restarts", type=int, default=0,
                   help="Restart the whole job up to N times after a rank fails; ranks see "
                        "CLOUDTIK_RESTART_COUNT / CLOUDTIK_RESUME=1 and resume from their checkpoint.")
    p.add_argument("--resume", action="store_true",
                   help="Ask the program to resume from its latest checkpoint (CLOUDTIK_RESUME=1).")
    p.add_argument("--profile", default="",
                   help="Run every rank under 'rocprofv3 --kernel-trace --stats'; output in DIR/rank<R>.")
    p.add_argument("--verbose", action="store_true")
    from cloudtik_amd.runner.cpu import add_cpu_args
    add_cpu_args(p)
    p.add_argument("program")
    p.add_argument("program_args", nargs=argparse.REMAINDER)
    return p


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    if args.launcher == "cpu":
        args.cpu = True
    d = Distributor(args.num_proc, args.nnodes, args.nproc_per_node, args.hosts or None, args.hostfile or None)
    launcher = args.launcher or ("distributed" if d.distributed_with_hosts and d.nnodes > 1 else
                                 ("cpu" if args.cpu else "local"))
    args.launcher = launcher
    if args.resume:
        os.environ["CLOUDTIK_RESUME"] = "1"
    base_port = args.master_port
    rc = 0
    for attempt in range(max(0, args.max_restarts) + 1):
        os.environ["CLOUDTIK_RESTART_COUNT"] = str(attempt)
        if attempt:
            os.environ["CLOUDTIK_RESUME"] = "1"
            # a fresh rendezvous port: the previous attempt's store may still be in TIME_WAIT
            args.master_port = base_port + attempt
            print(f"[cloudtik-run] restarting the job (attempt {attempt + 1} of {args.max_restarts + 1}) "
                  f"after exit code {rc}", file=sys.stderr)
        rc = create_launcher(launcher, args, d).run()
        if rc == 0 or args.node_rank or args.first_rank:
            # remote node launchers do not restart on their own: the driver restarts the job
            break
    return rc


if __name__ == "__main__":
    sys.exit(main())
