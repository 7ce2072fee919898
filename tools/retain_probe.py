"""retain = false and bounded memory.  Per step: fresh device inputs of the
bench's shape (make_relation, untimed), the expected verify identities taken from them (untimed),
optionally retain_memory(False) on both, then ONE timed join, its peak reserved / allocated memory
(the allocator's peak over the join alone) and the bench's exact verify of the output.

usage: python tools/retain_probe.py [--rows N] [--payload-cols P] [--steps K] [--warmup W]
                                    [--retain 0|1] [--how inner]
Prints one JSON line per step and a summary line (median ms over the timed steps, max peak)."""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from cylon_amd import CylonContext  # noqa: E402
from cylon_amd._lib import C  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=1_000_000_000)
    p.add_argument("--payload-cols", type=int, default=3)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--retain", type=int, default=0)
    p.add_argument("--how", default="inner")
    a = p.parse_args()
    ctx = CylonContext(device="cuda:0")
    key_range = int(0.99 * a.rows)
    recs = []
    for s in range(a.warmup + a.steps):
        left = bench.make_relation(ctx, a.rows, key_range, a.payload_cols, 1000, "cuda")
        right = bench.make_relation(ctx, a.rows, key_range, a.payload_cols, 2000, "cuda")
        expect = bench.join_expectation(ctx, left, right, key_range, a.how)
        if not a.retain:
            left.retain_memory(False)
            right.retain_memory(False)
        torch.cuda.synchronize()
        base_alloc = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        st0 = torch.cuda.memory_stats()
        C.trace_enable(True)
        C.trace_reset()
        t0 = time.perf_counter()
        out = left.join(right, a.how, "hash", on=["k"], left_prefix="l_", right_prefix="r_")
        torch.cuda.synchronize()
        ms = 1000.0 * (time.perf_counter() - t0)
        cnt = {k: v for k, v in dict(C.trace_counters()).items() if k.startswith("join.")}
        C.trace_enable(False)
        st = torch.cuda.memory_stats()
        rec = {"step": s, "timed": s >= a.warmup, "ms": round(ms, 2), "retain": bool(a.retain),
               "rows": a.rows, "payload_cols": a.payload_cols,
               "inputs_gb": round(2 * a.rows * 8 * (1 + a.payload_cols) / 2**30, 1),
               "peak_reserved_gb": round(st.get("reserved_bytes.all.peak", 0) / 2**30, 1),
               "peak_allocated_gb": round(st.get("allocated_bytes.all.peak", 0) / 2**30, 1),
               "allocated_before_gb": round(base_alloc / 2**30, 1),
               "alloc_retries": int(st.get("num_alloc_retries", 0) - st0.get("num_alloc_retries", 0)),
               "device_mallocs": int(st.get("num_device_alloc", 0) - st0.get("num_device_alloc", 0)),
               "inputs_left_rows": [left.row_count, right.row_count], "counters": cnt}
        rec["verify"] = bench.verify_join_against(ctx, out, expect, a.how)
        print(json.dumps(rec), flush=True)
        recs.append(rec)
        del out, left, right, expect  # (no empty_cache: the next step's blocks come from the cache, as
        # in the bench's timed loop -- re-mapping ~170 GB with hipMalloc costs seconds)
    timed = [r for r in recs if r["timed"]]
    print(json.dumps({"summary": True, "retain": bool(a.retain), "rows": a.rows, "payload_cols": a.payload_cols,
                      "median_ms": round(statistics.median(r["ms"] for r in timed), 2),
                      "all_ms": [r["ms"] for r in timed],
                      "max_peak_reserved_gb": max(r["peak_reserved_gb"] for r in timed),
                      "max_peak_allocated_gb": max(r["peak_allocated_gb"] for r in timed),
                      "verify_ok": all(r["verify"]["ok"] for r in timed)}), flush=True)


if __name__ == "__main__":
    main()
