"""Building tables: from Python dicts, lists, numpy, pandas, Arrow and torch tensors, on the host
or straight into HBM (reference: python/examples/table_initialize.py, table_conversions.py).

    python examples/python/table_initialize.py [--device cpu|cuda:0]
"""
import numpy as np
import pandas as pd
import pyarrow as pa
import torch

from _common import device_from_argv, report
from cylon_amd import CylonContext, Table

dev = device_from_argv()
ctx = CylonContext(device=dev)

t_dict = Table.from_pydict(ctx, {"id": [1, 2, 3, 4], "score": [0.5, 1.5, 2.5, 3.5]})
t_list = Table.from_list(ctx, ["id", "score"], [[1, 2, 3, 4], [0.5, 1.5, 2.5, 3.5]])
t_np = Table.from_numpy(ctx, ["id", "score"], [np.arange(1, 5), np.arange(4) + 0.5])
t_pd = Table.from_pandas(ctx, pd.DataFrame({"id": [1, 2, 3, 4], "score": [0.5, 1.5, 2.5, 3.5]}))
t_arrow = Table.from_arrow(ctx, pa.table({"id": [1, 2, 3, 4], "score": [0.5, 1.5, 2.5, 3.5]}))
# a device tensor becomes a column without a copy (it already lives where the context computes)
t_torch = Table.from_torch(ctx, {"id": torch.arange(1, 5, device=dev), "score": torch.arange(4, device=dev) + 0.5})

for name, t in [("dict", t_dict), ("list", t_list), ("numpy", t_np), ("pandas", t_pd), ("arrow", t_arrow),
                ("torch", t_torch)]:
    assert t.to_pydict() == t_dict.to_pydict(), name
    report(f"rows_{name}", t.row_count)

# conversions back out
report("pandas_sum", float(t_arrow.to_pandas()["score"].sum()))
report("numpy_shape", "x".join(map(str, t_np.to_numpy().shape)))
report("torch_device", t_torch.to_torch()["id"].device.type)
report("arrow_columns", ",".join(t_pd.to_arrow().column_names))
