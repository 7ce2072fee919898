"""Headline benchmark: distributed inner join, rows/s, on 1/2/4/8 MI355X.

Workload (BASELINE.json / BASELINE.md): two relations of 1B rows each in total,
the reference's benchmark shape (cpp/src/experiments/run_dist_scaling.py:
4 columns = int64 key + 3 float64 payload, keys uniform in [0, 0.99 * rows)).
Strong scaling like the reference: the total row count is fixed and split over
the N ranks.  Synthetic data is generated directly in HBM on each rank.

One timed step = one DistributedJoin (hash shuffle of both relations over
RCCL + local device hash join + materialisation of all 8 output columns).
metric value = (|L| + |R|) / step time, whole job.

Usage:
  python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--algorithm hash|sort]
  N > 1 is launched by torch.distributed.run (one process per GPU).
"""
import argparse
import json
import os
import sys
import time

import torch

REFERENCE_ROWS_PER_S = 4.0e8 / 2.3  # 2 x 200M rows in 2.3 s on 160 CPU cores (provisional row count)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--rows", type=int, default=1_000_000_000, help="rows per relation (total over all ranks)")
    p.add_argument("--payload-cols", type=int, default=3)
    p.add_argument("--algorithm", default="hash", choices=["hash", "sort"])
    p.add_argument("--key-ratio", type=float, default=0.99)
    p.add_argument("--profile-phases", action="store_true", help="print per-phase timings (extra syncs)")
    return p.parse_args()


def make_relation(ctx, rows_local, key_range, ncols, seed, device):
    from cylon_amd import Table
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    cols = {"k": torch.randint(0, key_range, (rows_local,), generator=g, device=device, dtype=torch.int64)}
    for c in range(ncols):
        cols[f"v{c}"] = torch.rand(rows_local, generator=g, device=device, dtype=torch.float64)
    return Table.from_torch(ctx, cols)


def sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cylon_amd import CylonContext, GlooConfig, RCCLConfig

    # CYLON_BENCH_BACKEND=gloo rehearses the multi-rank path on CPUs (tests only);
    # gloo-gpu keeps the tables in HBM (ranks may share one GPU) with gloo collectives
    backend = os.environ.get("CYLON_BENCH_BACKEND", "")
    cpu_rehearsal = backend == "gloo"
    if world > 1 and backend == "gloo-gpu":
        ndev = max(torch.cuda.device_count(), 1)
        ctx = CylonContext(config=GlooConfig(device=f"cuda:{int(os.environ.get('LOCAL_RANK', '0')) % ndev}"),
                           distributed=True)
    elif world > 1:
        ctx = CylonContext(config=GlooConfig() if cpu_rehearsal else RCCLConfig(), distributed=True)
    else:
        ctx = CylonContext(config=None, distributed=False, device="cpu" if cpu_rehearsal else "cuda:0")
    device = ctx.device
    n = world
    rows_local = args.rows // n
    key_range = max(1, int(args.key_ratio * args.rows))
    left = make_relation(ctx, rows_local, key_range, args.payload_cols, 1000 + rank, device)
    right = make_relation(ctx, rows_local, key_range, args.payload_cols, 2000 + rank, device)
    sync()

    def step():
        out = left.distributed_join(right, "inner", args.algorithm, on=[0], left_prefix="l_", right_prefix="r_")
        return out.row_count

    out_rows = 0
    for _ in range(args.warmup):
        out_rows = step()
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out_rows = step()
    sync()
    ctx.barrier()
    elapsed = time.perf_counter() - t0

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        t = ctx.allreduce(t, "max")
        rows_t = torch.tensor([out_rows], dtype=torch.int64, device=device)
        rows_t = ctx.allreduce(rows_t, "sum")
        out_rows = int(rows_t.item())
    elapsed = float(t.item())
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    rows_in = 2 * rows_local * n
    value = rows_in / (ms_per_step / 1000.0)
    if rank == 0:
        rec = {
            "metric": "rows/sec distributed inner-join, 1B×1B int64 keys, at 1/2/4/8 MI355X",
            "value": value,
            "unit": "rows/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": value / REFERENCE_ROWS_PER_S,
            "dtype": "int64 keys / float64 payload",
            "data": "synthetic (device-generated; keys uniform in [0, 0.99*rows), reference run_dist_scaling shape)",
            "config": {
                "model": f"distributed inner join ({args.algorithm}), int64 key + {args.payload_cols} float64 cols",
                "global_batch": args.rows,
                "seq_len": 1 + args.payload_cols,
                "parallelism": f"dp{n} (hash shuffle over RCCL)" if n > 1 else "dp1 (local join)",
                "rows_per_relation": args.rows,
                "output_rows": out_rows,
                "key_range": key_range,
            },
        }
        print(json.dumps(rec), flush=True)
    ctx.finalize()


if __name__ == "__main__":
    main()
