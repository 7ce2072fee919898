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
                  [--how inner|left|right|outer] [--no-verify]

With --gpus N > 1 and no torchrun environment, bench.py starts
`torch.distributed.run --nproc-per-node N` on itself as a child process (one
rank per GPU, RCCL), the way the reference's run_dist_scaling.py:115-154 starts
`mpirun -np w`; the parent never touches the GPU.  Under an outer torchrun,
WORLD_SIZE must equal --gpus (a mismatch exits non-zero).

After the timed region the last timed step's output is checked against an
independent torch computation of the same join (key-count and payload-sum
identities, see verify_join; --no-verify skips it), and one extra traced step
reports per-phase milliseconds (max over ranks; not part of the metric).  At
N > 1 every rank reports its device, PCI bus id and the process group's world
size into the JSON line ("ranks"), so the record names the GPUs the ranks ran on.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

REFERENCE_ROWS_PER_S = 4.0e8 / 2.3  # 2 x 200M rows in 2.3 s on 160 CPU cores (provisional row count)
ROOT = os.path.dirname(os.path.abspath(__file__))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--rows", type=int, default=1_000_000_000, help="rows per relation (total over all ranks)")
    p.add_argument("--payload-cols", type=int, default=3)
    p.add_argument("--algorithm", default="hash", choices=["hash", "sort"])
    p.add_argument("--key-ratio", type=float, default=0.99)
    p.add_argument("--no-phases", action="store_true", help="skip the traced per-phase step after the timed region")
    p.add_argument("--how", default="inner", choices=["inner", "left", "right", "outer"])
    p.add_argument("--verify", action="store_true", help="(default) check the last output against torch, untimed")
    p.add_argument("--no-verify", action="store_true", help="skip the output check")
    p.add_argument("--sync-steps", action="store_true",
                   help="diagnostic: synchronise the device after every timed step (host never runs ahead)")
    p.add_argument("--force-shuffle", action="store_true",
                   help="with --gpus 1: run a world-1 RCCL context through the full shuffle + exchange path "
                        "(config force_shuffle=1) instead of the local join")
    return p.parse_args()


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(script: str, nproc: int, argv) -> int:
    """Run `script argv` as nproc torchrun ranks in a child process and return its exit code.
    Called before anything in this process initialises HIP (exec after a GPU touch is forbidden)."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), script, *argv]
    return subprocess.call(cmd, env=env)


def resolve_world(gpus: int, script: str, argv):
    """(world, rank) for this process, or exits: spawns the ranks when --gpus > 1 is asked for
    without a torchrun environment; refuses a WORLD_SIZE that disagrees with --gpus."""
    if "WORLD_SIZE" not in os.environ:
        if gpus > 1:
            sys.exit(spawn_ranks(script, gpus, argv))
        return 1, 0
    world = int(os.environ["WORLD_SIZE"])
    if world != gpus:
        print(f"error: --gpus {gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    return world, int(os.environ.get("RANK", "0"))


def make_context(world: int, force_shuffle: bool = False):
    """CYLON_BENCH_BACKEND=gloo rehearses the multi-rank path on CPUs (tests only); gloo-gpu keeps
    the tables in HBM (ranks may share one GPU) with gloo collectives; default = RCCL.
    force_shuffle at world 1: a distributed RCCL context of one rank whose operators take the
    shuffle path (RCCL self all-to-all), so the 1-GPU run measures the exchange machinery."""
    from cylon_amd import CylonContext, GlooConfig, RCCLConfig
    backend = os.environ.get("CYLON_BENCH_BACKEND", "")
    if world == 1 and force_shuffle:
        for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0"), ("MASTER_ADDR", "127.0.0.1")):
            os.environ.setdefault(k, v)
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        ctx = CylonContext(config=GlooConfig() if backend == "gloo" else RCCLConfig(), distributed=True)
        ctx.add_config("force_shuffle", "1")
        return ctx
    if world > 1 and backend == "gloo-gpu":
        ndev = max(torch.cuda.device_count(), 1)
        return CylonContext(config=GlooConfig(device=f"cuda:{int(os.environ.get('LOCAL_RANK', '0')) % ndev}"),
                            distributed=True)
    if world > 1:
        return CylonContext(config=GlooConfig() if backend == "gloo" else RCCLConfig(), distributed=True)
    return CylonContext(config=None, distributed=False, device="cpu" if backend == "gloo" else "cuda:0")


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


def max_over_ranks(ctx, d: dict) -> dict:
    """{name: value} -> {name: max over ranks} (names missing on a rank count as 0)."""
    if ctx.get_world_size() == 1:
        return d
    import torch.distributed as dist
    allv = [None] * ctx.get_world_size()
    dist.all_gather_object(allv, d)
    out = {}
    for part in allv:
        for k, v in part.items():
            out[k] = max(out.get(k, 0.0), v)
    return out


def verify_join(ctx, left, right, out, key_range, how="inner") -> dict:
    """Independent check of a join output by per-key identities (global key counts cL / cR by torch
    bincount, all-reduced over ranks; per-row gathers of them, no weighted histogram -- a float64
    atomic histogram serialises on a hot key; reference join/join_utils.cpp:126-181 for outer rows):
      rows        = sum_k cL(k) cR(k)  [+ sum_k cL(k) [cR(k) = 0] (left, outer)]
                                       [+ sum_k cR(k) [cL(k) = 0] (right, outer)]
      null l / r  = the unmatched right / left rows above, and their payload bytes are zero
      sum l_k     = sum over left rows i of k_i * (cR(k_i) [+ [cR(k_i) = 0]])  (l_k == r_k where both exist)
      sum l_v0    = sum over left rows i of v_i * (cR(k_i) [+ [cR(k_i) = 0]])
      sum r_v0    = sum over right rows j of w_j * (cL(k_j) [+ [cL(k_j) = 0]])"""
    return verify_join_against(ctx, out, join_expectation(ctx, left, right, key_range, how), how)


def join_expectation(ctx, left, right, key_range, how="inner"):
    """The verify_join identities' expected values, from the inputs alone (so a caller can take them
    before a retain = false join releases its inputs)."""
    lt, rt = left.to_torch(), right.to_torch()
    dev = lt["k"].device
    f64 = torch.float64
    cL = torch.bincount(lt["k"], minlength=key_range)
    cR = torch.bincount(rt["k"], minlength=key_range)
    if ctx.get_world_size() > 1:
        cL.copy_(ctx.allreduce(cL, "sum"))
        cR.copy_(ctx.allreduce(cR, "sum"))
    keep_l = how in ("left", "outer")
    keep_r = how in ("right", "outer")
    inner = (cL.to(f64) * cR.to(f64)).sum()
    un_l = (cL * (cR == 0)).sum().to(f64) if keep_l else torch.zeros((), dtype=f64, device=dev)
    un_r = (cR * (cL == 0)).sum().to(f64) if keep_r else torch.zeros((), dtype=f64, device=dev)

    def mult(c_other, keys, keep):  # output rows of each input row
        m = c_other.index_select(0, keys)
        return (m + (m == 0)).to(f64) if keep else m.to(f64)
    ml = mult(cR, lt["k"], keep_l)
    mr = mult(cL, rt["k"], keep_r)
    part = torch.stack([(lt["k"].to(f64) * ml).sum(), (lt["v0"] * ml).sum(), (rt["v0"] * mr).sum()])
    del ml, mr, cL, cR
    if ctx.get_world_size() > 1:
        part = ctx.allreduce(part, "sum")
    return torch.cat([torch.stack([inner + un_l + un_r, un_r, un_l]), part])


def verify_join_against(ctx, out, expect, how="inner") -> dict:
    ocols = {c.name: c for c in out.native.columns()}
    dev = expect.device
    f64 = torch.float64

    def col(name):
        c = ocols[name]
        v = c.validity
        return c.data, (torch.ones(c.data.shape[0], dtype=torch.bool, device=dev) if v is None else v.to(torch.bool))
    lkd, lkv = col("l_k")
    rkd, rkv = col("r_k")
    lvd, lvv = col("l_v0")
    rvd, rvv = col("r_v0")
    both = lkv & rkv
    mism = ((lkd != rkd) & both).sum().to(f64)
    null_payload = (lvd.abs() * (~lvv)).sum() + (rvd.abs() * (~rvv)).sum()  # null slots hold zeros
    got = torch.stack([torch.tensor(float(out.row_count), dtype=f64, device=dev), (~lkv).sum().to(f64),
                       (~rkv).sum().to(f64), (lkd.to(f64) * lkv).sum(), (lvd * lvv).sum(), (rvd * rvv).sum(), mism,
                       null_payload.to(f64)])
    if ctx.get_world_size() > 1:
        got = ctx.allreduce(got, "sum")
    e, g = expect.cpu().tolist(), got.cpu().tolist()
    rel = [abs(a - b) / max(abs(a), 1.0) for a, b in zip(e, g[:6])]
    ok = g[0] == e[0] and g[1] == e[1] and g[2] == e[2] and g[6] == 0 and g[7] == 0 and rel[3] < 1e-12 and \
        rel[4] < 1e-9 and rel[5] < 1e-9
    return {"ok": bool(ok), "how": how, "rows": int(g[0]), "expected_rows": int(e[0]),
            "null_left_rows": int(g[1]), "expected_null_left_rows": int(e[1]),
            "null_right_rows": int(g[2]), "expected_null_right_rows": int(e[2]),
            "key_mismatch_rows": int(g[6]), "null_payload_abs_sum": g[7],
            "rel_err_sum_k": rel[3], "rel_err_sum_l_v0": rel[4], "rel_err_sum_r_v0": rel[5]}


def rank_record(ctx) -> list:
    """[{rank, device, pci_bus_id, world_size}] of every rank (all-gathered; rank 0 prints it)."""
    import torch.distributed as dist
    rec = {"rank": ctx.get_rank(), "world_size_pg": dist.get_world_size() if dist.is_initialized() else 1,
           "backend": dist.get_backend() if dist.is_initialized() else None}
    if torch.cuda.is_available():
        d = torch.cuda.current_device()
        props = torch.cuda.get_device_properties(d)
        rec.update({"device": d, "name": props.name,
                    "pci_bus_id": f"{getattr(props, 'pci_domain_id', 0):04x}:{getattr(props, 'pci_bus_id', 0):02x}:"
                                  f"{getattr(props, 'pci_device_id', 0):02x}",
                    "uuid": str(getattr(props, "uuid", ""))})
    else:
        rec["device"] = "cpu"
    if ctx.get_world_size() == 1:
        return [rec]
    allv = [None] * ctx.get_world_size()
    dist.all_gather_object(allv, rec)
    return allv


def main():
    args = parse()
    world, rank = resolve_world(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    sys.path.insert(0, ROOT)
    ctx = make_context(world, args.force_shuffle)
    device = ctx.device
    n = world
    rows_local = args.rows // n
    key_range = max(1, int(args.key_ratio * args.rows))
    left = make_relation(ctx, rows_local, key_range, args.payload_cols, 1000 + rank, device)
    right = make_relation(ctx, rows_local, key_range, args.payload_cols, 2000 + rank, device)
    sync()

    def step():
        return left.distributed_join(right, args.how, args.algorithm, on=[0], left_prefix="l_", right_prefix="r_")

    out = None
    for _ in range(args.warmup):
        out = step()
        out = None
    ctx.barrier()
    sync()
    alloc0 = torch.cuda.memory_stats() if torch.cuda.is_available() else {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = None  # the previous output is released before the next join allocates
        out = step()
        if args.sync_steps:
            sync()
    sync()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    out_rows = out.row_count if out is not None else 0
    # caching-allocator activity inside the timed region: a retry frees every cached block
    # (device synchronise + hipFree) and mallocs again -- the cost of running at the memory limit
    alloc1 = torch.cuda.memory_stats() if torch.cuda.is_available() else {}
    allocator = {"alloc_retries": int(alloc1.get("num_alloc_retries", 0) - alloc0.get("num_alloc_retries", 0)),
                 "device_mallocs": int(alloc1.get("num_device_alloc", 0) - alloc0.get("num_device_alloc", 0)),
                 "device_frees": int(alloc1.get("num_device_free", 0) - alloc0.get("num_device_free", 0)),
                 "peak_reserved_gb": round(alloc1.get("reserved_bytes.all.peak", 0) / 2**30, 1),
                 "peak_allocated_gb": round(alloc1.get("allocated_bytes.all.peak", 0) / 2**30, 1)}

    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        t = ctx.allreduce(t, "max")
        rows_t = torch.tensor([out_rows], dtype=torch.int64, device=device)
        rows_t = ctx.allreduce(rows_t, "sum")
        out_rows = int(rows_t.item())
    elapsed = float(t.item())

    verify = None
    if not args.no_verify and out is not None:
        verify = verify_join(ctx, left, right, out, key_range, args.how)
    out = None
    ranks = rank_record(ctx)

    phases = None
    counters = {}
    if not args.no_phases:
        from cylon_amd.utils import trace
        trace.enable_tracing(True)
        trace.reset_tracing()
        ctx.barrier()
        sync()
        t1 = time.perf_counter()
        step()
        sync()
        traced_ms = 1000.0 * (time.perf_counter() - t1)
        ph = {k: v[0] for k, v in trace.phases().items()}
        ph["step_total"] = traced_ms
        counters = {k: v for k, v in trace.counters().items() if k.startswith("shuffle.")}
        trace.enable_tracing(False)
        phases = {k: round(v, 3) for k, v in sorted(max_over_ranks(ctx, ph).items())}

    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    rows_in = 2 * rows_local * n
    value = rows_in / (ms_per_step / 1000.0)
    if rank == 0:
        rec = {
            "metric": ("rows/sec distributed inner-join, 1B×1B int64 keys, at 1/2/4/8 MI355X" if args.how == "inner"
                       else f"rows/sec distributed {args.how}-join, 1B×1B int64 keys (not the headline)"),
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
                "model": f"distributed {args.how} join ({args.algorithm}), int64 key + {args.payload_cols} float64 cols",
                "global_batch": args.rows,
                "seq_len": 1 + args.payload_cols,
                "parallelism": (f"dp{n} (hash shuffle over {'RCCL' if os.environ.get('CYLON_BENCH_BACKEND', '') == '' else os.environ['CYLON_BENCH_BACKEND']})"
                                if n > 1 or args.force_shuffle else "dp1 (local join)"),
                "rows_per_relation": args.rows,
                "output_rows": out_rows,
                "key_range": key_range,
            },
        }
        if phases is not None:
            rec["phases_ms_max_over_ranks"] = phases
        if verify is not None:
            rec["verify"] = verify
        rec["ranks"] = ranks
        rec["allocator_timed_region"] = allocator
        if args.sync_steps:
            rec["sync_steps"] = True
        if args.force_shuffle:
            rec["force_shuffle"] = True
        if counters:
            rec["shuffle_counters_rank0"] = counters
        print(json.dumps(rec), flush=True)
    ctx.finalize()
    if verify is not None and not verify["ok"]:
        sys.exit(3)


if __name__ == "__main__":
    main()
