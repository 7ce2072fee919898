"""Checkpoint / spill of distributed tables (aux subsystem; the reference has none beyond
WriteCSV/WriteParquet, cpp/src/cylon/table.cpp:244-253,1117-1126).

Each rank writes its partition as an Arrow IPC file plus a JSON manifest; a reload
restores every partition onto the same rank (world size must match) and device."""
import json
import os

from ..data.table import Table
from ..io import read_arrow_ipc, write_arrow_ipc


def save_table(table: Table, directory: str, name: str = "table") -> str:
    ctx = table.context
    rank, world = ctx.get_rank(), ctx.get_world_size()
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, f"{name}.part{rank:05d}-of-{world:05d}.arrow")
    write_arrow_ipc(table, path)
    with open(os.path.join(directory, f"{name}.part{rank:05d}.json"), "w") as f:
        json.dump({"rank": rank, "world": world, "rows": table.row_count, "columns": table.column_names,
                   "file": os.path.basename(path)}, f)
    return path


def load_table(ctx, directory: str, name: str = "table") -> Table:
    rank, world = ctx.get_rank(), ctx.get_world_size()
    with open(os.path.join(directory, f"{name}.part{rank:05d}.json")) as f:
        meta = json.load(f)
    if meta["world"] != world:
        raise ValueError(f"checkpoint written by {meta['world']} ranks, loading with {world}")
    t = read_arrow_ipc(ctx, os.path.join(directory, meta["file"]))
    if t.row_count != meta["rows"]:
        raise ValueError("checkpoint row count mismatch")
    return t
