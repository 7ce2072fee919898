"""cylon_amd.models: end-to-end pipelines built on the engine.

`etl_ddp` is the reference's Cylon -> PyTorch DDP tutorial
(cpp/src/tutorial/demo_pytorch_distributed.py) done MI355X-first: the join
result stays in HBM and becomes the training tensor without the reference's
`to_numpy()` host hop, and DDP runs on the same process group (RCCL).
"""
from .etl_ddp import ETLNetwork, join_features, train_ddp

__all__ = ["ETLNetwork", "join_features", "train_ddp"]
