"""Cylon ETL -> torch DDP training (M9).

Reference: cpp/src/tutorial/demo_pytorch_distributed.py:45-128 — each rank
reads user_device_tm_{r}.csv and user_usage_tm_{r}.csv, joins them (sort
join, device key column 0 = usage key column 3), takes columns 2:6 as features
and 6 as the target, and trains a 4 -> 1 -> 16 -> 1 MLP with DDP + SGD/MSE.
Here the joined table is turned into device tensors directly
(`utils.interop.to_tensor`), and the DDP process group is the one the
CylonContext already runs on (RCCL over xGMI on MI355X, gloo on CPU).
"""
from typing import Tuple

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ..data.table import Table
from ..utils.interop import to_tensor


class ETLNetwork(nn.Module):
    """The reference demo's network (4 -> 1 -> 16 -> 1, ReLU)."""

    def __init__(self, features: int = 4):
        super().__init__()
        self.hidden1 = nn.Linear(features, 1)
        self.hidden2 = nn.Linear(1, 16)
        self.output = nn.Linear(16, 1)

    def forward(self, x):
        x = F.relu(self.hidden1(x))
        x = F.relu(self.hidden2(x))
        return self.output(x)


def join_features(devices: Table, usage: Table, feature_cols=slice(2, 6), target_col: int = 6,
                  algorithm: str = "sort") -> Tuple[torch.Tensor, torch.Tensor]:
    """Join device and usage tables (device col 0 = usage col 3) and cut features / target."""
    joined = devices.join(usage, "inner", algorithm, left_on=[0], right_on=[3], left_prefix="d_",
                          right_prefix="u_")
    names = joined.column_names
    feats = names[feature_cols]
    x = to_tensor(joined, feats, dtype=torch.float32)
    y = to_tensor(joined, [names[target_col]], dtype=torch.float32)
    return x, y


def train_ddp(x: torch.Tensor, y: torch.Tensor, epochs: int = 20, lr: float = 1e-3, batch: int = 1,
              train_rows: int = 100, seed: int = 0):
    """DDP training loop of the reference demo; returns (model, last loss).  Uses the default
    process group when one is initialised (every rank must call it), else trains locally."""
    torch.manual_seed(seed)
    device = x.device
    model = ETLNetwork(x.shape[1]).to(device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        ids = [device.index] if device.type == "cuda" else None
        model = nn.parallel.DistributedDataParallel(model, device_ids=ids)
    opt = torch.optim.SGD(model.parameters(), lr=lr)
    loss_fn = nn.MSELoss()
    xt, yt = x[:train_rows], y[:train_rows]
    loss = torch.zeros((), device=device)
    for _ in range(epochs):
        for i in range(0, xt.shape[0], batch):
            pred = model(xt[i:i + batch])
            loss = loss_fn(pred, yt[i:i + batch])
            opt.zero_grad()
            loss.backward()
            opt.step()
    return model, float(loss.detach())
