"""Multi-GPU runs of the secondary BASELINE.json configs (one process per GPU, RCCL):

  groupby : distributed hash group-by + sum, 1B rows / 10M int64 groups (config 4)
  sort    : distributed sample sort of 2B int64 rows (config 5)
  union   : distributed union of two join-shaped relations (reference headline #2)

Strong scaling: --rows is the global row count, split over the ranks; data is
generated in HBM on each rank.  Launch like bench.py: `--gpus N` without a torchrun
environment starts N ranks itself (bench.spawn_ranks, a child torchrun); under an
outer torchrun WORLD_SIZE must equal --gpus.
CYLON_BENCH_BACKEND=gloo-gpu runs the ranks over gloo (ranks may share one GPU:
rehearsal of the device code paths, not a timing of xGMI).
Prints one JSON line per config on rank 0 (max over ranks of the timed region).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import make_context, resolve_world  # noqa: E402  (imports no GPU code)

DEFAULT_ROWS = {"groupby": 1_000_000_000, "sort": 2_000_000_000, "union": 1_000_000_000}


def sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def timed(ctx, fn, steps, warmup):
    for _ in range(warmup):
        fn()
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    sync()
    ctx.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=ctx.device)
    if ctx.get_world_size() > 1:
        el = ctx.allreduce(el, "max")
    return float(el.item()) / steps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="groupby", choices=["groupby", "sort", "union"])
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--groups", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    world, _ = resolve_world(a.gpus, os.path.abspath(__file__), sys.argv[1:])
    from cylon_amd import Table
    ctx = make_context(world)
    rank, world = ctx.get_rank(), ctx.get_world_size()
    rows = a.rows or DEFAULT_ROWS[a.config]
    n = rows // world
    g = torch.Generator(device=ctx.device).manual_seed(100 + rank)
    dev = ctx.device
    if a.config == "groupby":
        t = Table.from_torch(ctx, {"g": torch.randint(0, a.groups, (n,), generator=g, device=dev),
                                   "x": torch.rand(n, generator=g, device=dev, dtype=torch.float64)})
        fn = lambda: t.groupby("g", {"x": "sum"}).row_count  # noqa: E731
    elif a.config == "sort":
        t = Table.from_torch(ctx, {"k": torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, device=dev)})
        fn = lambda: t.distributed_sort("k").row_count  # noqa: E731
    else:
        hi = int(0.99 * rows)

        def rel():
            return Table.from_torch(ctx, {"k": torch.randint(0, hi, (n,), generator=g, device=dev),
                                          **{f"v{i}": torch.rand(n, generator=g, device=dev, dtype=torch.float64)
                                             for i in range(3)}})
        L, R = rel(), rel()
        fn = lambda: L.distributed_union(R).row_count  # noqa: E731
    sec, local_out = timed(ctx, fn, a.steps, a.warmup)
    out_rows = torch.tensor([local_out], dtype=torch.int64, device=dev)
    if world > 1:
        out_rows = ctx.allreduce(out_rows, "sum")
    if rank == 0:
        rows_in = n * world * (2 if a.config == "union" else 1)
        print(json.dumps({"config": a.config, "n_gpus": world, "rows": rows, "ms": sec * 1e3,
                          "rows_per_s": rows_in / sec, "rows_out": int(out_rows.item()),
                          "backend": os.environ.get("CYLON_BENCH_BACKEND", "rccl" if world > 1 else "local")}),
              flush=True)
    ctx.finalize()


if __name__ == "__main__":
    main()
