"""``ai.modeling.graph_sage`` workflow: tabular data -> graph -> GraphSAGE link-prediction
training -> node embeddings -> tabular data with embedding columns (reference
graph_sage/modeling/run.py:504-700, build_graph.py, embeddings.py).

Two distributed modes (``cloudtik-run -np N``):

* ``--num-parts 1`` (default): the whole graph is resident on every GPU (288 GB HBM3E holds
  billion-edge graphs) and training is data-parallel over RCCL.
* ``--num-parts N`` (= world size): rank 0 partitions the graph (``distributed.py``, LDG),
  every rank loads its partition, samples across partitions with all-to-alls and holds a
  shard of the node embeddings -- the reference's partitioned DistGraph training without
  separate graph-server / sampler processes (``--num-servers``/``--num-samplers`` are
  accepted and ignored).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import yaml


def parse_args(argv=None):
    ap = argparse.ArgumentParser("ai.modeling.graph_sage", description=__doc__)
    a = ap.add_argument
    for flag in ("single-node", "no-process-data", "no-build-graph", "no-partition-graph", "no-train",
                 "no-predict", "heterogeneous", "inductive", "exclude-reverse-edges"):
        a(f"--{flag}", f"--{flag.replace('-', '_')}", action="store_true")
    a("--raw-data-path", "--raw_data_path")
    a("--processed-data-path", "--processed_data_path")
    a("--data-processing-config", "--data_processing_config")
    a("--model-file", "--model_file")
    a("--temp-dir", "--temp_dir", default="/tmp")
    a("--output-dir", "--output_dir", default="./output")
    a("--dataset-name", "--dataset_name", default="graph")
    a("--tabular2graph", required=False)
    a("--train-output", "--train_output")
    a("--predict-output", "--predict_output")
    a("--data-with-embeddings-name", "--data_with_embeddings_name", default="data_with_embeddings.csv")
    a("--hosts")
    a("--graph-name", "--graph_name", default="graph")
    a("--num-parts", "--num_parts", type=int, default=1)
    a("--num-hops", "--num_hops", type=int, default=1)
    a("--num-trainers", "--num_trainers", type=int, default=1)
    a("--num-samplers", "--num_samplers", type=int, default=0)
    a("--num-servers", "--num_servers", type=int, default=1)
    a("--num-server-threads", "--num_server_threads", type=int, default=1)
    a("--num-omp-threads", "--num_omp_threads", type=int, default=0)
    a("--num-epochs", "--num_epochs", type=int, default=2)
    a("--num-hidden", "--num_hidden", type=int, default=64)
    a("--num-layers", "--num_layers", type=int, default=2)
    a("--fan-out", "--fan_out", default="10,15")
    a("--batch-size", "--batch_size", type=int, default=1024)
    a("--batch-size-eval", "--batch_size_eval", type=int, default=100000)
    a("--eval-every", "--eval_every", type=int, default=1)
    a("--lr", type=float, default=5e-3)
    a("--log-every", "--log_every", type=int, default=20)
    a("--num-dl-workers", "--num_dl_workers", type=int, default=0)
    a("--relations", default=None)
    a("--node-feature", "--node_feature", default=None)
    a("--device", default=None)
    return ap.parse_args(argv)


def apply_embeddings(df, graph, emb: np.ndarray, node_columns):
    """Replace every node-id column by its embedding columns n<i>_c<j>_e<k>."""
    import pandas as pd
    types = list(dict.fromkeys(node_columns.values()))
    for i, t in enumerate(types):
        cols = [c for c, ty in node_columns.items() if ty == t]
        for j, c in enumerate(cols):
            idx = graph.node_index[t].get_indexer(df[c]) + graph.type_offset[t]
            e = pd.DataFrame(emb[idx], index=df.index).add_prefix(f"n{i}_c{j}_e")
            df = pd.concat([df.drop(columns=[c]), e], axis=1)
    return df


def run(args):
    import torch
    import torch.distributed as dist
    from cloudtik_amd.modeling.gbdt.data import process_data, read_table
    from cloudtik_amd.modeling.graph_sage import LinkPredictionTrainer, TrainConfig, build_graph

    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1 and not dist.is_initialized():
        if torch.cuda.is_available():
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    rank = dist.get_rank() if dist.is_initialized() else 0
    os.makedirs(args.output_dir, exist_ok=True)
    cfg = yaml.safe_load(open(args.tabular2graph)) if args.tabular2graph else None
    if cfg is None:
        raise SystemExit("--tabular2graph config is required")
    df = read_table(args.processed_data_path or args.raw_data_path)
    if not args.no_process_data and args.data_processing_config:
        splits = process_data(df, yaml.safe_load(open(args.data_processing_config)))
        import pandas as pd
        df = pd.concat(list(splits.values()))
    graph = build_graph(df, cfg)
    result = {"num_nodes": graph.num_nodes, "num_edges": graph.num_edges}
    model_file = args.model_file or os.path.join(args.output_dir, "graph_sage.pt")
    world = dist.get_world_size() if dist.is_initialized() else 1
    if args.num_parts > 1 and not args.single_node:
        return _run_partitioned(args, df, cfg, graph, result, model_file, rank, world)
    tc = TrainConfig(num_epochs=args.num_epochs, num_hidden=args.num_hidden, num_layers=args.num_layers,
                     fan_out=[int(x) for x in str(args.fan_out).split(",")], batch_size=args.batch_size,
                     batch_size_eval=args.batch_size_eval, eval_every=args.eval_every, lr=args.lr,
                     log_every=args.log_every, exclude_reverse_edges=True)
    trainer = LinkPredictionTrainer(graph, tc, device=args.device)
    if not args.no_train:
        result.update(trainer.train())
        if rank == 0:
            trainer.save(model_file)
    elif os.path.exists(model_file):
        trainer.model.load_state_dict(torch.load(model_file, weights_only=True)["state_dict"])
    if not args.no_predict and rank == 0:
        emb = trainer.embeddings().float().cpu().numpy()
        out = args.predict_output or os.path.join(args.output_dir, "node_embeddings.npy")
        np.save(out, emb)
        data_out = os.path.join(args.output_dir, args.data_with_embeddings_name)
        apply_embeddings(df, graph, emb, cfg["node_columns"]).to_csv(data_out, index=False)
        result["embeddings"] = out
        result["data_with_embeddings"] = data_out
    if rank == 0:
        print(json.dumps(result, default=float), flush=True)
    return result


def _run_partitioned(args, df, cfg, graph, result, model_file, rank, world):
    import torch
    import torch.distributed as dist
    from .distributed import DistGraph, DistLinkPredictionTrainer, DistTrainConfig, partition_graph

    if args.num_parts != world:
        raise SystemExit(f"--num-parts {args.num_parts} needs {args.num_parts} ranks (got {world})")
    part_dir = os.path.join(args.temp_dir, f"{args.graph_name}_parts")
    if rank == 0 and not (args.no_partition_graph and os.path.exists(os.path.join(part_dir, "partition.json"))):
        result["partition"] = partition_graph(graph, args.num_parts, part_dir)
    dist.barrier()
    device = args.device or (f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() else "cpu")
    dg = DistGraph(part_dir, rank, world, device)
    tc = DistTrainConfig(num_hidden=args.num_hidden, num_layers=args.num_layers,
                         fan_out=tuple(int(x) for x in str(args.fan_out).split(",")), batch_size=args.batch_size,
                         num_epochs=args.num_epochs, lr=args.lr)
    trainer = DistLinkPredictionTrainer(dg, tc)
    if not args.no_train:
        result.update(trainer.train())
        result["test_auc"] = trainer.evaluate(2)
        if rank == 0:
            trainer.save(model_file)
    emb = trainer.gather_embeddings() if not args.no_predict else None
    if emb is not None:
        emb = emb.numpy()
        out = args.predict_output or os.path.join(args.output_dir, "node_embeddings.npy")
        np.save(out, emb)
        data_out = os.path.join(args.output_dir, args.data_with_embeddings_name)
        apply_embeddings(df, graph, emb, cfg["node_columns"]).to_csv(data_out, index=False)
        result["embeddings"] = out
        result["data_with_embeddings"] = data_out
    if rank == 0:
        print(json.dumps(result, default=float), flush=True)
    return result


def main(argv=None):
    return run(parse_args(argv))


if __name__ == "__main__":
    sys.exit(0 if main() is not None else 1)
