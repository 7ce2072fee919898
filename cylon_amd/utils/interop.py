"""Zero-copy interop with torch / DLPack (hand tables to torch DDP
on-device instead of the reference demo's to_numpy host hop,
cpp/src/tutorial/demo_pytorch_distributed.py:88-104)."""
from typing import Dict, List

import torch
from torch.utils import dlpack

from ..data.table import Table


def to_dlpack(table: Table) -> Dict[str, object]:
    """Column name -> DLPack capsule of the device buffer (fixed-width columns)."""
    return {k: dlpack.to_dlpack(v) for k, v in table.to_torch().items()}


def from_dlpack(ctx, capsules: Dict[str, object]) -> Table:
    return Table.from_torch(ctx, {k: dlpack.from_dlpack(c) for k, c in capsules.items()})


def to_tensor(table: Table, columns: List[str] = None, dtype=torch.float32) -> torch.Tensor:
    """[rows, cols] tensor on the table's device (one device-side stack, no host copy)."""
    cols = table.to_torch()
    names = columns or list(cols.keys())
    return torch.stack([cols[c].to(dtype) for c in names], dim=1)
