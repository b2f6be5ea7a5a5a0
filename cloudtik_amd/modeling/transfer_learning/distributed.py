"""Distributed fine-tuning launched FROM the model API (reference
modeling/transfer_learning/common/pytorch/model.py:217-237 ``fit_distributed`` and
image_classification_model.py:250 ``train(..., distributed=True, nnodes, nproc_per_node,
hosts, hostfile)``).

``model.train(dataset, ..., distributed=True, nnodes=2, nproc_per_node=8, hosts="a,b")``:

1. the driver saves the job into ``shared_dir`` (a directory every node can read: NFS /
   the ``mount`` runtime's HDFS fuse mount, or local for one node): the model's current
   weights (safetensors, via the model's own ``export``), which parameters are frozen, the
   training arguments (JSON) and the datasets (cloudpickle -- a dataset is arbitrary Python;
   only this job's own file is ever deserialized);
2. ``runner.run_command`` starts ``python -m cloudtik_amd.modeling.transfer_learning.distributed
   <dir>`` on every rank (the ``cloudtik-run`` launchers: local ranks, or one per node over
   ssh / ``cloudtik head exec``);
3. each rank joins the process group (RCCL on GPUs, gloo on CPU), rebuilds the model from the
   saved weights, and runs the model's normal ``train`` -- the Trainer shards the data with a
   DistributedSampler and all-reduces gradient buckets;
4. rank 0 exports the trained model and the history; the driver loads both back into the
   calling model object, so the API returns exactly what a local ``train`` would.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time
from typing import Any, Dict, Optional

SPEC = "job.json"


_LOCAL_HOSTS = {"localhost", "127.0.0.1", "::1"}


def _host_names(hosts: Optional[str], hostfile: Optional[str]):
    names = []
    for item in (hosts or "").split(","):
        h = item.strip().split(":")[0]
        if h:
            names.append(h)
    if hostfile:
        with open(hostfile) as f:
            for line in f:
                line = line.split("#", 1)[0].strip()
                if line:
                    names.append(line.split()[0].split(":")[0])
    return names


def spans_hosts(nnodes: int, hosts: Optional[str], hostfile: Optional[str]) -> bool:
    """Whether a launch would put ranks on more than this host."""
    import socket
    if nnodes > 1:
        return True
    local = _LOCAL_HOSTS | {socket.gethostname(), socket.getfqdn()}
    names = set(_host_names(hosts, hostfile))
    return bool(names - local) or len(names) > 1


def fit_distributed(model, dataset, train_kwargs: Dict[str, Any], nnodes: int = 1, nproc_per_node: int = 1,
                    hosts: Optional[str] = None, hostfile: Optional[str] = None, shared_dir: Optional[str] = None,
                    launcher: Optional[str] = None, master_port: int = 29500, env: Optional[dict] = None):
    """Train ``model`` on ``dataset`` over ranks started by ``run_command``.  The job directory
    (model export, ``datasets.pkl``, the trained model and history written by rank 0) must be
    readable by every rank: a job that spans hosts needs ``shared_dir`` on a filesystem all of
    them mount.  ``datasets.pkl`` is a cloudpickle that every rank LOADS (executes): keep
    ``shared_dir`` writable only by trusted users."""
    import cloudpickle
    from cloudtik_amd.runner import run_command
    if shared_dir is None and spans_hosts(nnodes, hosts, hostfile):
        raise ValueError("a distributed job that spans hosts needs shared_dir= (a directory every host mounts): "
                         "the ranks on other hosts read the job files from it and rank 0 writes the trained "
                         "model there")
    root = shared_dir or tempfile.mkdtemp(prefix="cloudtik-tl-")
    job = os.path.join(root, f"tl_job_{time.strftime('%Y%m%d-%H%M%S')}_{os.getpid()}")
    os.makedirs(job)
    model.export(os.path.join(job, "model"))
    kw = dict(train_kwargs)
    eval_dataset = kw.pop("eval_dataset", None)
    with open(os.path.join(job, "datasets.pkl"), "wb") as f:
        cloudpickle.dump({"train": dataset, "eval": eval_dataset}, f)
    frozen = [n for n, p in model.model.named_parameters() if not p.requires_grad]
    with open(os.path.join(job, SPEC), "w") as f:
        json.dump({"train_kwargs": kw, "frozen": frozen}, f)
    rc = run_command([sys.executable, "-m", "cloudtik_amd.modeling.transfer_learning.distributed", job],
                     nnodes=nnodes, nproc_per_node=nproc_per_node, hosts=hosts, hostfile=hostfile,
                     launcher=launcher, master_port=master_port, no_python=True, env=env)
    if rc != 0:
        raise RuntimeError(f"distributed training failed with exit code {rc} (job files in {job})")
    from cloudtik_amd.modeling.transfer_learning.model_factory import load_model
    trained = load_model(os.path.join(job, "trained"), device=getattr(model, "device", None))
    model.model.load_state_dict(trained.model.state_dict())
    with open(os.path.join(job, "history.json")) as f:
        model.history = json.load(f)
    return model.history


def main(argv=None) -> int:
    import cloudpickle
    from cloudtik_amd.modeling.transfer_learning.model_factory import load_model
    from cloudtik_amd.train.trainer import setup_distributed
    job = (argv or sys.argv[1:])[0]
    rank, world, device = setup_distributed()
    with open(os.path.join(job, SPEC)) as f:
        spec = json.load(f)
    model = load_model(os.path.join(job, "model"), device=device)
    frozen = set(spec.get("frozen") or [])
    for n, p in model.model.named_parameters():
        p.requires_grad_(n not in frozen)
    if hasattr(model, "freeze_backbone"):
        model.freeze_backbone = bool(frozen)
    with open(os.path.join(job, "datasets.pkl"), "rb") as f:
        ds = cloudpickle.load(f)               # written by the driver of this very job
    history = model.train(ds["train"], eval_dataset=ds["eval"], **spec["train_kwargs"])
    if rank == 0:
        model.export(os.path.join(job, "trained"))
        with open(os.path.join(job, "history.json"), "w") as f:
            json.dump(history, f)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    print(f"[transfer-learning] rank {rank}/{world} done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
