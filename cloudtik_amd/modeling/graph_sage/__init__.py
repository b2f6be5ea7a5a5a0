from .graph import Block, Graph, build_graph, full_blocks, sample_blocks, sample_neighbors  # noqa: F401
from .model import EdgeDecoder, GraphSAGE, GraphSAGEModel, SAGEConv  # noqa: F401
from .trainer import LinkPredictionTrainer, TrainConfig  # noqa: F401
