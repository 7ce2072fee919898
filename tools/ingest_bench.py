"""From-Arrow ingest throughput (host Arrow table -> HBM table), pinned staging vs pageable copy.

Builds one host Arrow table (int64 + float64 + nullable int64 + bool columns, --rows rows),
then times Table.from_arrow(ctx, table) on cuda:0 -- host staging, PCIe DMA, validity and
bool unpacking on the device, synchronised -- once per mode, alternating:
  staged:   io/h2d.cpp pinned ring (default)
  pageable: CYLON_STAGED_INGEST=0 (torch .to(device) from pageable numpy views)
Prints one JSON line per run: mode, seconds, host bytes moved, GB/s.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import pyarrow as pa
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cylon_amd import CylonContext, Table  # noqa: E402


def build(n: int) -> pa.Table:
    a = np.arange(n, dtype=np.int64)
    f = a.astype(np.float64) * 0.5
    valid = np.ones(n, dtype=bool)
    valid[::7] = False
    b = (a & 1) == 0
    return pa.table({"k": pa.array(a), "v": pa.array(f), "nk": pa.array(a, mask=~valid), "flag": pa.array(b)})


def host_bytes(t: pa.Table) -> int:
    return sum(buf.size for col in t.columns for chunk in col.chunks for buf in chunk.buffers() if buf is not None)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=1_000_000_000)
    p.add_argument("--reps", type=int, default=2)
    a = p.parse_args()
    ctx = CylonContext(device="cuda:0")
    t0 = time.perf_counter()
    tbl = build(a.rows)
    nbytes = host_bytes(tbl)
    print(json.dumps({"built_s": round(time.perf_counter() - t0, 2), "host_bytes": nbytes}), flush=True)
    for _ in range(a.reps):
        for mode in ("staged", "pageable"):
            os.environ["CYLON_STAGED_INGEST"] = "1" if mode == "staged" else "0"
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dt = Table.from_arrow(ctx, tbl)
            torch.cuda.synchronize()
            s = time.perf_counter() - t0
            assert dt.row_count == a.rows
            print(json.dumps({"mode": mode, "rows": a.rows, "seconds": round(s, 4), "bytes": nbytes,
                              "GB_per_s": round(nbytes / s / 1e9, 2)}), flush=True)
            del dt
            torch.cuda.empty_cache()
    # spot check: the staged copy is exact
    os.environ["CYLON_STAGED_INGEST"] = "1"
    small = tbl.slice(a.rows - 3_000_000, 3_000_000)
    back = Table.from_arrow(ctx, small).to_arrow()
    assert back.column("k").equals(small.column("k")) and back.column("flag").equals(small.column("flag"))
    assert back.column("nk").null_count == small.column("nk").null_count
    print(json.dumps({"check": "ok"}), flush=True)


if __name__ == "__main__":
    main()
