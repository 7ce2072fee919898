"""Synthetic data generators (reference: cpp/src/experiments/generate_csv.py:16-31,
generate_files.py:44-71, cpp/src/examples/ra_test_inmem_datagen_example.cpp:95-139,
python/pycylon util generate_numeric_csv)."""
from typing import Optional

import numpy as np
import pandas as pd
import torch


def generate_numeric_csv(rows: int, columns: int, file_path: str, key_range_ratio: float = 0.99,
                         seed: Optional[int] = None):
    """int key column (uniform in [0, ratio*rows)) + (columns-1) floats in [0, 1) with 3 decimals."""
    rng = np.random.default_rng(seed)
    data = {"0": rng.integers(0, max(1, int(rows * key_range_ratio)), rows)}
    for c in range(1, columns):
        data[str(c)] = np.round(rng.random(rows), 3)
    pd.DataFrame(data).to_csv(file_path, index=False)
    return file_path


def random_table(ctx, rows: int, payload_cols: int = 3, key_range: Optional[int] = None, seed: int = 0,
                 key_dtype=torch.int64, payload_dtype=torch.float64):
    """Device-generated table of the reference benchmark shape (key + payload columns)."""
    from ..data.table import Table
    dev = ctx.device
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    kr = key_range if key_range is not None else max(1, int(0.99 * rows))
    cols = {"k": torch.randint(0, kr, (rows,), generator=g, device=dev, dtype=key_dtype)}
    for c in range(payload_cols):
        cols[f"v{c}"] = torch.rand(rows, generator=g, device=dev, dtype=payload_dtype)
    return Table.from_torch(ctx, cols)
