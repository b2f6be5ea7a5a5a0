"""Collection switches shared by ``cloudtik cluster-dump``, ``cloudtik head cluster-dump`` and
``cloudtik node dump`` (reference scripts.py cluster-dump options; ``--gpu`` is the AMD GPU
state of core/cluster_dump.py)."""
import functools

import click


def dump_options(f):
    @click.option("--logs/--no-logs", default=True, help="Session logs (and the runtimes' logs).")
    @click.option("--debug-state/--no-debug-state", default=True, help="The controller's last scaler state.")
    @click.option("--pip/--no-pip", default=True, help="Installed Python packages.")
    @click.option("--processes/--no-processes", default=True, help="CloudTik and runtime processes.")
    @click.option("--processes-verbose/--no-processes-verbose", default=True, help="Full command lines.")
    @click.option("--gpu/--no-gpu", default=True, help="AMD GPU state: amd-smi, KFD topology, RAS counters.")
    @click.option("--runtimes", default=None, help="Runtimes whose logs / processes to include (comma list).")
    @functools.wraps(f)
    def wrapper(*args, logs, debug_state, pip, processes, processes_verbose, gpu, runtimes, **kw):
        from cloudtik_amd.core.cluster_dump import DumpParameters
        kw["params"] = DumpParameters(logs=logs, debug_state=debug_state, pip=pip, processes=processes,
                                      processes_verbose=processes_verbose, gpu=gpu,
                                      runtimes=[r for r in (runtimes or "").split(",") if r])
        return f(*args, **kw)
    return wrapper
