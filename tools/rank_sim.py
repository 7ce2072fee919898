"""Per-rank compute of the N-GPU headline join, simulated on one GPU.

For world W each rank holds rows/W rows per relation.  This times, on one
MI355X, what one rank does outside the RCCL transfer: the shuffle's hash
partition + partition-major reorder of both relations, and the local join of
the received rows (≈ rows/W per relation).  Usage: python tools/rank_sim.py [rows] [W ...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cylon_amd import CylonContext, Table  # noqa: E402
from cylon_amd._lib import C  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
SORT = "--sort" in sys.argv  # config 5: distributed sample sort of 2B int64 keys
rows = int(args[0]) if args else (2_000_000_000 if SORT else 1_000_000_000)
worlds = [int(x) for x in args[1:]] or [2, 4, 8]
XGMI_GBPS = 77.0  # per link per direction (MI355X: 7 links x ~153 GB/s bidirectional)
ctx = CylonContext(device="cuda:0")
hi = int(0.99 * rows)


def rel(n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return Table.from_torch(ctx, {"k": torch.randint(0, hi, (n,), generator=g, device="cuda"),
                                  **{f"v{i}": torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
                                     for i in range(3)}})


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
        del r
    return best * 1e3


def sort_sim(W, K=4):
    """Per-rank work of the pipelined DistributedSort on W ranks (ops/setops.cpp pipelined_sort):
    the local radix sort of rows/W keys, the exchange of (W-1)/W of them over W-1 links in K key
    sub-range chunks, and the merge of the W sorted runs each chunk brings (merge-path rounds).
    Chunk k's merge overlaps chunk k+1's transfer, so the tail after the local sort is about
    max(exchange, merge) + min(exchange, merge) / K instead of their sum."""
    n = rows // W
    g = torch.Generator(device="cuda").manual_seed(5)
    t = Table.from_torch(ctx, {"k": torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, device="cuda")})
    ts = timed(lambda: t.sort("k"))
    # what a rank receives: W sorted runs of ~n/W keys each (rank-ordered), merged into one
    runs = [Table.from_torch(ctx, {"k": torch.sort(torch.randint(-(1 << 62), 1 << 62, (n // W,), generator=g,
                                                                  device="cuda")).values}) for _ in range(W)]
    got = Table.merge(runs)
    tm = timed(lambda: C.merge_sorted_runs(got.native, [n // W] * W, 0, True))
    nbytes = n * 8 * (W - 1) / W
    txfer = nbytes / ((W - 1) * XGMI_GBPS * 1e9) * 1e3
    serial = ts + txfer + tm
    piped = ts + max(txfer, tm) + min(txfer, tm) / K
    print(f"SORT W={W} rows/rank={n}: local sort {ts:.1f} ms, exchange {nbytes / 1e9:.2f} GB over {W - 1} links "
          f"~{txfer:.1f} ms, merge of {W} runs {tm:.1f} ms => serial {serial:.1f} ms, pipelined (K={K}) "
          f"{piped:.1f} ms ({rows / piped * 1e3:.3g} rows/s/job)", flush=True)
    del t, runs, got
    torch.cuda.empty_cache()


if SORT:
    for W in worlds:
        sort_sim(W)
    sys.exit(0)

for W in worlds:
    n = rows // W
    L, R = rel(n, 1), rel(n, 2)

    def part():
        outs = []
        for t in (L, R):
            pid, counts = C.map_to_hash_partitions(t.native, [0], W)
            outs.append(C.partition_reorder(t.native, pid, W))
        return outs

    def part_fast():  # what the shuffle runs for an int64 key: one LDS-staged pass (W * 4 chunk partitions)
        return [C.shuffle_partition(t.native, [0], W * 4) for t in (L, R)]

    tp = timed(part)
    tpf = timed(part_fast)
    tj = timed(lambda: L.join(R, "inner", "hash", on=[0]))
    nbytes = 2 * n * 32 * (W - 1) / W
    print(f"W={W} rows/rank={n}: partition+reorder(both) generic {tp:.1f} ms, fast {tpf:.1f} ms, "
          f"local join {tj:.1f} ms, "
          f"bytes sent/rank {nbytes / 1e9:.2f} GB", flush=True)
    del L, R
    torch.cuda.empty_cache()
