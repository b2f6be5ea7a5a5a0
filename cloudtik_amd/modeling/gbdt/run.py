"""``ai.modeling.xgboost`` workflow: process raw data -> train -> predict (reference
xgboost/modeling/run.py:98-330 with the same options and YAML configs).

Single process by default; for data-parallel training launch it with ``cloudtik-run -np N``
(one rank per GPU, torch.distributed env:// rendezvous): each rank takes an equal row shard
of the training split and histograms are all-reduced per tree level.  ``--num-actors N``
without a launcher runs the fault-tolerant driver (elastic.py): N actor processes, a model
checkpoint every ``--checkpoint-frequency`` rounds, ``--max-actor-restarts`` restarts per
actor and, with ``--elastic-training``, up to ``--max-failed-actors`` actors dropped
(reference RayParams, xgboost/modeling/run.py:90-106).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import Any, Dict

import numpy as np
import yaml


def _load_yaml(path):
    if not path:
        return {}
    with open(path) as f:
        return yaml.safe_load(f) or {}


def _rank_world():
    import torch.distributed as dist
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        if not dist.is_initialized():
            import torch
            backend = "nccl" if torch.cuda.is_available() else "gloo"
            if torch.cuda.is_available():
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
            dist.init_process_group(backend)
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def parse_args(argv=None):
    ap = argparse.ArgumentParser("ai.modeling.xgboost", description=__doc__)
    a = ap.add_argument
    a("--single-node", "--single_node", action="store_true", help="accepted for compatibility")
    a("--no-process-data", "--no_process_data", action="store_true")
    a("--no-train", "--no_train", action="store_true")
    a("--no-predict", "--no_predict", action="store_true")
    a("--in-memory", "--in_memory", action="store_true", help="keep processed data in memory only")
    a("--raw-data-path", "--raw_data_path")
    a("--data-processing-config", "--data_processing_config")
    a("--training-config", "--training_config")
    a("--dataset-config", "--dataset_config")
    a("--no-save", "--no_save", action="store_true")
    a("--processed-data-path", "--processed_data_path")
    a("--temp-dir", "--temp_dir", default="/tmp")
    a("--output-dir", "--output_dir", default="./output")
    a("--model-file", "--model_file")
    a("--predict-output", "--predict_output")
    a("--target-col", "--target_col")
    a("--data-api", "--data_api", default="pandas")
    a("--num-actors", "--num_actors", type=int, default=1,
      help="> 1: fault-tolerant actor processes from this driver (or launch with cloudtik-run -np N)")
    a("--cpus-per-actor", "--cpus_per_actor", type=int, default=0)
    a("--gpus-per-actor", "--gpus_per_actor", type=int, default=0)
    a("--device", default=None)
    a("--elastic-training", "--elastic_training", action="store_true")
    a("--max-failed-actors", "--max_failed_actors", type=int, default=0)
    a("--max-actor-restarts", "--max_actor_restarts", type=int, default=0)
    a("--checkpoint-frequency", "--checkpoint_frequency", type=int, default=5)
    return ap.parse_args(argv)


def _parquet_shard(path, target, ignore, actor_id, num_actors):
    """Elastic actor shard: rows actor_id::num_actors of the processed training split."""
    import pandas as pd
    from cloudtik_amd.modeling.gbdt import DMatrix
    from cloudtik_amd.modeling.gbdt.data import feature_frame
    X, y = feature_frame(pd.read_parquet(path), target, ignore)
    return DMatrix(X.iloc[actor_id::num_actors], y.iloc[actor_id::num_actors])


def run(args) -> Dict[str, Any]:
    import torch
    from cloudtik_amd.modeling.gbdt import Booster, DMatrix
    from cloudtik_amd.modeling.gbdt.data import feature_frame, process_data, read_table

    rank, world = _rank_world()
    os.makedirs(args.output_dir, exist_ok=True)
    dp_cfg = _load_yaml(args.data_processing_config)
    tr_cfg = _load_yaml(args.training_config)
    ds_cfg = _load_yaml(args.dataset_config)
    target = args.target_col or ds_cfg.get("target_col")
    ignore = ds_cfg.get("ignore_cols", [])
    processed = args.processed_data_path or os.path.join(args.output_dir, "processed")
    result: Dict[str, Any] = {}
    splits = None
    if not args.no_process_data:
        t0 = time.time()
        df = read_table(args.raw_data_path, args.data_api)
        splits = process_data(df, dp_cfg)
        result["process_seconds"] = time.time() - t0
        if not args.in_memory and not args.no_save and rank == 0:
            os.makedirs(processed, exist_ok=True)
            for name, d in splits.items():
                d.to_parquet(os.path.join(processed, f"{name}.parquet"))
    if splits is None:
        import pandas as pd
        splits = {os.path.splitext(f)[0]: pd.read_parquet(os.path.join(processed, f))
                  for f in sorted(os.listdir(processed)) if f.endswith(".parquet")}
    if not target:
        raise SystemExit("--target-col (or target_col in --dataset-config) is required")
    spec = tr_cfg.get("model_spec", {})
    params = dict(spec.get("model_params", {}))
    tparams = spec.get("training_params", {})
    device = args.device or ("cuda" if torch.cuda.is_available() else "cpu")
    model_file = args.model_file or os.path.join(args.output_dir, "model.json")
    booster = None
    if not args.no_train:
        Xtr, ytr = feature_frame(splits["train"], target, ignore)
        if world > 1:
            Xtr, ytr = Xtr.iloc[rank::world], ytr.iloc[rank::world]
        evals = []
        for name in ("valid", "test"):
            if name in splits and len(splits[name]):
                Xe, ye = feature_frame(splits[name], target, ignore)
                evals.append((DMatrix(Xe, ye), name))
        t0 = time.time()
        rounds = int(tparams.get("num_boost_round", 100))
        if args.num_actors > 1 and world == 1:
            # fault-tolerant multi-actor training from this driver process
            import functools
            from cloudtik_amd.modeling.gbdt.elastic import ElasticParams, train_elastic
            train_path = os.path.join(processed, "train.parquet")
            if not os.path.exists(train_path):
                os.makedirs(processed, exist_ok=True)
                splits["train"].to_parquet(train_path)
            ep = ElasticParams(num_actors=args.num_actors, elastic_training=args.elastic_training,
                               max_failed_actors=args.max_failed_actors,
                               max_actor_restarts=args.max_actor_restarts,
                               checkpoint_frequency=args.checkpoint_frequency,
                               checkpoint_dir=os.path.join(args.output_dir, "checkpoints"),
                               device="cuda" if device.startswith("cuda") else "cpu")
            booster, report = train_elastic(params, functools.partial(_parquet_shard, train_path, target, ignore),
                                            rounds, ep, log=lambda m: print(f"[elastic] {m}", flush=True))
            result["elastic"] = report
        else:
            booster = Booster(params, device=device).train(
                DMatrix(Xtr, ytr), rounds, evals,
                tparams.get("early_stopping_rounds"), tparams.get("verbose_eval", False))
        if device.startswith("cuda"):
            torch.cuda.synchronize()
        result["train_seconds"] = time.time() - t0
        result["num_trees"] = booster.num_trees
        result["scores"] = getattr(booster, "last_scores", {})
        if rank == 0 and not args.no_save:
            booster.save_model(model_file)
    if not args.no_predict and rank == 0:
        booster = booster or Booster.load_model(model_file, device=device)
        name = "test" if "test" in splits else "train"
        Xp, yp = feature_frame(splits[name], target, ignore)
        pred = booster.predict(DMatrix(Xp))
        from cloudtik_amd.modeling.gbdt import evaluate_metric
        metric = tr_cfg.get("model_spec", {}).get("test_metric") or booster._default_metric()
        p = torch.as_tensor(pred).float()
        p = p[:, None] if p.dim() == 1 else p
        result["test_metric"] = {metric: evaluate_metric(metric, p, torch.as_tensor(yp.to_numpy()),
                                                         torch.ones(len(yp)))}
        if args.predict_output:
            np.savetxt(args.predict_output, pred, delimiter=",")
    if rank == 0:
        print(json.dumps(result, default=float), flush=True)
    return result


def main(argv=None):
    return run(parse_args(argv))


if __name__ == "__main__":
    sys.exit(0 if main() is not None else 1)
