"""GPU numerics tests: every HIP kernel path against its CPU twin / a pandas oracle."""
import numpy as np
import pandas as pd
import pyarrow as pa
import pytest
import torch

from cylon_amd import C, Table

pytestmark = pytest.mark.gpu


def _pair(gpu_ctx, ctx, at):
    return Table(at, gpu_ctx), Table(at, ctx)


def _rows(df):
    return sorted(map(tuple, df.astype(object).where(pd.notnull(df), None).itertuples(index=False)),
                  key=lambda r: tuple((x is None, str(x)) for x in r))


def test_extension_is_native_and_on_gpu(gpu_ctx):
    assert C.__file__.endswith(".so")
    t = Table(pa.table({"a": [1, 2, 3]}), gpu_ctx)
    assert t.device.startswith("cuda")


def test_lds_atomics_return_in_lane_order(gpu_ctx):
    """Precondition of the radix passes' wave-atomic stable ranking: same-address LDS atomics of
    one wave64 instruction return in lane order (the passes self-check this once per process and
    fall back to ballot ranking otherwise; here 256 blocks x 4096 rounds = 6.7e7 lane-ops)."""
    assert C.lds_lane_order_violations("cuda:0", 256, 4096) == 0


@pytest.mark.parametrize("rank", [1, 2])
def test_radix_sort_stable_under_both_rankings(gpu_ctx, monkeypatch, rank):
    """The row-moving sort (stable LSD passes) under each stable ranking method (1 = wave-atomic,
    2 = ballots, forced with rp_set_ranking; 0 re-probes the device afterwards): ties keep their
    input order."""
    rng = np.random.default_rng(3)
    n = 400_000
    k = rng.integers(-300, 300, n)
    t = Table(pa.table({"k": k, "p": np.arange(n)}), gpu_ctx)
    monkeypatch.setenv("CYLON_RADIX_SORT_MIN_ROWS", "1")
    C.rp_set_ranking(rank)
    try:
        s = t.sort("k").to_pandas()
    finally:
        C.rp_set_ranking(0)
    assert np.array_equal(s["p"].to_numpy(), np.lexsort((np.arange(n), k))), "unstable"


@pytest.mark.parametrize("nparts", [1, 2, 3, 4, 7, 8, 64, 1000])
def test_partition_ids_and_split_match_cpu(gpu_ctx, ctx, nparts):
    rng = np.random.default_rng(nparts)
    n = 100_003
    at = pa.table({"i": rng.integers(-2**40, 2**40, n), "f": rng.random(n),
                   "s": [f"k{x}" for x in rng.integers(0, 999, n)],
                   "i8": pa.array(rng.integers(-100, 100, n), pa.int8())})
    g, c = _pair(gpu_ctx, ctx, at)
    for cols in ([0], [1], [2], [3], [0, 1, 2, 3]):
        pg, hg = C.map_to_hash_partitions(g.native, cols, nparts)
        pc, hc = C.map_to_hash_partitions(c.native, cols, nparts)
        assert hg == hc
        assert torch.equal(pg.cpu(), pc)
    parts_g = g.hash_partition([0, 2], nparts)
    parts_c = c.hash_partition([0, 2], nparts)
    for a, b in zip(parts_g, parts_c):
        assert a.to_arrow().equals(b.to_arrow())  # stable split: identical order


@pytest.mark.parametrize("n", [0, 1, 63, 64, 4097, 1_000_000])
def test_mask_compaction_and_gather(gpu_ctx, ctx, n):
    rng = np.random.default_rng(n)
    at = pa.table({"x": rng.integers(0, 10, n),
                   "y": pa.array([None if v < 0.1 else v for v in rng.random(n)], pa.float64())
                   if n < 5000 else rng.random(n)})
    g, c = _pair(gpu_ctx, ctx, at)
    mask = torch.from_numpy(rng.random(n) < 0.3)
    assert g.filter_mask(mask).to_arrow().equals(c.filter_mask(mask).to_arrow())
    idx = torch.from_numpy(rng.integers(-1, max(n, 1), n))
    if n:
        assert g.take(idx).to_arrow().equals(c.take(idx).to_arrow())


@pytest.mark.parametrize("algorithm", ["hash", "sort"])
@pytest.mark.parametrize("how", ["inner", "left", "right", "outer"])
def test_join_gpu_vs_cpu(gpu_ctx, ctx, algorithm, how):
    rng = np.random.default_rng(7)
    a = pa.table({"k": rng.integers(0, 3000, 20000), "s": [f"s{x}" for x in rng.integers(0, 50, 20000)],
                  "v": rng.random(20000)})
    b = pa.table({"k": rng.integers(0, 3000, 9000), "s": [f"s{x}" for x in rng.integers(0, 50, 9000)],
                  "w": rng.random(9000)})
    for on in (["k"], ["k", "s"]):
        res = []
        for cx in (gpu_ctx, ctx):
            res.append(Table(a, cx).join(Table(b, cx), how, algorithm, on=on, left_prefix="l_",
                                         right_prefix="r_").to_pandas())
        assert _rows(res[0]) == _rows(res[1])


@pytest.mark.parametrize("n", [2_000_000, 6_000_000])
def test_large_join_count_matches_pandas(gpu_ctx, n):
    # 2M: sorted (atomic-free) build + two-pass probe; 6M: sorted build + single-pass emit probe
    g = torch.Generator(device="cuda").manual_seed(3)
    k1 = torch.randint(0, int(0.99 * n), (n,), generator=g, device="cuda")
    k2 = torch.randint(0, int(0.99 * n), (n,), generator=g, device="cuda")
    l = Table.from_torch(gpu_ctx, {"k": k1, "v": torch.rand(n, device="cuda", dtype=torch.float64)})
    r = Table.from_torch(gpu_ctx, {"k": k2, "w": torch.rand(n, device="cuda", dtype=torch.float64)})
    for alg in ("hash", "sort"):
        out = l.join(r, "inner", alg, on=[0], left_prefix="l_", right_prefix="r_")
        a = pd.Series(k1.cpu().numpy()).value_counts()
        b = pd.Series(k2.cpu().numpy()).value_counts()
        expect = int((a * b.reindex(a.index).fillna(0)).sum())
        assert out.row_count == expect
        o = out.to_torch()
        assert torch.equal(o["l_k"], o["r_k"])


@pytest.mark.parametrize("dtype", ["int64", "int32", "int8", "uint16", "float64", "float32", "string"])
@pytest.mark.parametrize("asc", [True, False])
def test_sort_gpu_vs_cpu(gpu_ctx, ctx, dtype, asc):
    rng = np.random.default_rng(11)
    n = 50_000
    if dtype == "string":
        col = pa.array([None if x % 97 == 0 else f"w{x * 7919 % 1000}x" * (1 + x % 3) for x in range(n)])
    elif dtype.startswith("float"):
        vals = rng.normal(size=n).astype(dtype)
        vals[::101] = np.nan
        vals[::103] = -0.0
        col = pa.array(vals)
    else:
        info = np.iinfo(dtype)
        col = pa.array(rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True))
    at = pa.table({"a": col, "b": rng.integers(0, 5, n), "i": np.arange(n)})
    g, c = _pair(gpu_ctx, ctx, at)
    sg = g.sort(["a", "b"], ascending=[asc, True]).to_arrow()
    sc = c.sort(["a", "b"], ascending=[asc, True]).to_arrow()
    pd.testing.assert_frame_equal(sg.to_pandas(), sc.to_pandas())  # NaN-aware (Table.equals is not)
    # oracle on the order of the non-null values
    pdf = at.to_pandas()
    ref = pdf.sort_values(["a", "b"], ascending=[asc, True], kind="stable", na_position="last")
    if dtype.startswith("float"):
        got = sg.column("a").to_numpy(zero_copy_only=False)
        exp = ref["a"].to_numpy()
        nn = ~np.isnan(exp)
        assert np.array_equal(got[nn], exp[nn])
    else:
        assert sg.column("a").to_pylist() == ref["a"].where(pd.notnull(ref["a"]), None).tolist()


def test_radix_sort_large_int64(gpu_ctx):
    n = 3_000_000
    k = torch.randint(-2**62, 2**62, (n,), device="cuda")
    t = Table.from_torch(gpu_ctx, {"k": k})
    s = t.sort("k").to_torch()["k"]
    assert torch.equal(s, torch.sort(k).values)


@pytest.mark.parametrize("case", ["uniform63", "small_range_ties", "skewed", "desc", "one_chunk"])
def test_lookback_sort_passes_match_stable_torch_sort(gpu_ctx, monkeypatch, case):
    """Look-back LSD passes (2 all-8-byte columns: key + payload; chunk plans counted by the previous
    pass, offsets from a decoupled look-back) vs torch's stable sort; payload order = stability.
    Balanced chunks run XCD-local (look-back words in one L2), skewed ones (
    90 % one key) let every XCD take any chunk's tiles with written-through words."""
    n = 5_000_000
    g = torch.Generator(device="cuda").manual_seed(21)
    if case in ("uniform63", "desc"):
        k = torch.randint(-2**62, 2**62, (n,), generator=g, device="cuda")
    elif case == "small_range_ties":
        k = torch.randint(-3000, 3000, (n,), generator=g, device="cuda") * 977
    elif case == "skewed":  # 90 % one key: one chunk / one digit holds most rows (36 bits: 4 x 9-bit digits)
        k = torch.randint(0, 1 << 36, (n,), generator=g, device="cuda")
        k[torch.rand(n, generator=g, device="cuda") < 0.9] = 123456789
    else:  # 3 x 8-bit digits, the first one < 32: every row lands in chunk 0 of the second pass
        a = torch.randint(0, 32, (n,), generator=g, device="cuda")
        b = torch.randint(0, 1 << 16, (n,), generator=g, device="cuda")
        k = ((a | (b << 8)) << 3) + (1 << 50)
    v = torch.arange(n, device="cuda")
    t = Table.from_torch(gpu_ctx, {"k": k, "v": v})
    asc = case != "desc"
    monkeypatch.setenv("CYLON_RADIX_SORT_MIN_ROWS", "1")
    C.trace_enable(True)
    C.trace_reset()
    out = t.sort("k", ascending=asc).to_torch()
    torch.cuda.synchronize()
    c = dict(C.trace_counters())
    C.trace_enable(False)
    assert c.get("sort.radix.lookback", 0) == 1, c
    assert c.get("sort.radix.lookback_timeout_fallback", 0) == 0, c
    ref_k, idx = torch.sort(k, stable=True, descending=not asc)
    assert torch.equal(out["k"], ref_k)
    assert torch.equal(out["v"], v[idx])


@pytest.mark.parametrize("case", ["uniform63", "desc", "ties", "uint64", "skewed", "narrow_span"])
def test_msd_keys_only_sort_matches_torch(gpu_ctx, monkeypatch, case):
    """Keys-only int sorts: two MSD slot passes + the LDS segment sort (kernels/seg_sort.hip) vs
    torch.sort.  Skewed top digits overflow a slot and the LSD passes sort instead; a span narrower
    than the MSD digits never takes the MSD path."""
    n = 6_000_000
    g = torch.Generator(device="cuda").manual_seed(23)
    dt = torch.int64
    if case in ("uniform63", "desc"):
        k = torch.randint(-2**62, 2**62, (n,), generator=g, device="cuda")
    elif case == "ties":  # ~3.8M distinct keys over 33 bits: equal keys inside partitions (more copies per
        # key widen the partition-size spread beyond the slots' Poisson margin: the LSD fallback)
        k = torch.randint(-3000000, 3000000, (n,), generator=g, device="cuda") * 977
    elif case == "uint64":
        k = torch.randint(0, 2**63 - 1, (n,), generator=g, device="cuda").to(torch.uint64)
        dt = torch.uint64
    elif case == "skewed":  # 90 % one key: its partition outgrows every slot
        k = torch.randint(0, 1 << 40, (n,), generator=g, device="cuda")
        k[torch.rand(n, generator=g, device="cuda") < 0.9] = 123456789
    else:  # keys in [0, 1024): 10 varying bits, fewer than the 11 MSD bits
        k = torch.randint(0, 1024, (n,), generator=g, device="cuda")
    t = Table.from_torch(gpu_ctx, {"k": k})
    asc = case != "desc"
    monkeypatch.setenv("CYLON_RADIX_SORT_MIN_ROWS", "1")
    C.trace_enable(True)
    C.trace_reset()
    out = t.sort("k", ascending=asc).to_torch()["k"]
    torch.cuda.synchronize()
    c = dict(C.trace_counters())
    C.trace_enable(False)
    if dt == torch.uint64:  # torch sorts uint64 as unsigned only via int64 + bias
        ref = (torch.sort(k.view(torch.int64) ^ (-(2**63)))[0] ^ (-(2**63))).view(torch.uint64)
        assert torch.equal(out.view(torch.int64), ref.view(torch.int64))
    else:
        assert torch.equal(out, torch.sort(k, descending=not asc).values)
    if case == "skewed":
        assert c.get("sort.radix.msd_slot_overflow", 0) == 1 and c.get("sort.radix.msd", 0) == 0, c
    elif case == "narrow_span":
        assert c.get("sort.radix.msd", 0) == 0, c
    else:
        assert c.get("sort.radix.msd", 0) == 1, c


@pytest.mark.parametrize("op", ["groupby", "unique", "union"])
def test_partition_lookback_passes_match_exact(gpu_ctx, monkeypatch, op):
    """Look-back passes of the stable two-pass hash partitions (group-by, set ops): 12M rows need more
    than 10 partition bits, i.e. two passes; the result equals the exact-histogram passes
    (CYLON_PARTITION_LOOKBACK=0)."""
    n = 12_000_000
    g = torch.Generator(device="cuda").manual_seed(23)
    k = torch.randint(0, 1_600_000, (n,), generator=g, device="cuda")
    x = torch.randint(0, 3, (n,), generator=g, device="cuda").to(torch.float64)
    t = Table.from_torch(gpu_ctx, {"k": k, "x": x})
    t2 = Table.from_torch(gpu_ctx, {"k": k[: n // 2] + 7, "x": x[: n // 2]})
    monkeypatch.setenv("CYLON_RADIX_GROUPBY_MIN_ROWS", "1")
    monkeypatch.setenv("CYLON_RADIX_SETOP_MIN_ROWS", "1")
    res = []
    for lb in ("1", "0"):
        monkeypatch.setenv("CYLON_PARTITION_LOOKBACK", lb)
        C.trace_enable(True)
        C.trace_reset()
        if op == "groupby":
            df = t.local_groupby("k", {"x": ["sum", "count"]}).to_pandas().sort_values("k")
        elif op == "unique":
            df = t.unique().to_pandas().sort_values(["k", "x"])
        else:
            df = t.union(t2).to_pandas().sort_values(["k", "x"])
        c = dict(C.trace_counters())
        C.trace_enable(False)
        if lb == "1":
            assert c.get("partition.radix.lookback", 0) >= 1, c
            assert c.get("partition.radix.lookback_timeout_fallback", 0) == 0, c
        res.append(df.reset_index(drop=True))
    pd.testing.assert_frame_equal(res[0], res[1])
    # the CPU twin as an independent third oracle (a shared GPU encoding bug would pass the A/B)
    tc, t2c = t.to_cpu(), t2.to_cpu()
    if op == "groupby":
        cpu = tc.local_groupby("k", {"x": ["sum", "count"]}).to_pandas().sort_values("k")
    elif op == "unique":
        cpu = tc.unique().to_pandas().sort_values(["k", "x"])
    else:
        cpu = tc.union(t2c).to_pandas().sort_values(["k", "x"])
    pd.testing.assert_frame_equal(res[0], cpu.reset_index(drop=True), check_dtype=False)


def _sorted_df(t):
    df = t.to_pandas()
    return df.sort_values(list(df.columns), kind="stable").reset_index(drop=True)


@pytest.mark.parametrize("case", ["int64", "int32_nullable", "dups", "skew_fallback", "left_smaller"])
def test_radix_join_matches_global_table_join(gpu_ctx, ctx, monkeypatch, case):
    """K5 LDS radix join (partitioned, fused materialisation) vs the global-table join."""
    rng = np.random.default_rng(11)
    nl, nr = 300_000, 200_000
    if case == "left_smaller":
        nl, nr = nr, nl
    hi = 20000 if case == "dups" else int(0.9 * max(nl, nr))
    kl, kr = rng.integers(0, hi, nl), rng.integers(0, hi, nr)
    if case == "skew_fallback":
        kr[:10_000] = 7  # one build partition > LDS table capacity -> global fallback
    kt = pa.int32() if case == "int32_nullable" else pa.int64()
    mask_u = rng.random(nl) < 0.1 if case == "int32_nullable" else None
    mask_b = rng.random(nr) < 0.2 if case == "int32_nullable" else None
    a = pa.table({"k": pa.array(kl, kt), "v": rng.random(nl),
                  "u": pa.array(rng.integers(-300, 300, nl), pa.int16(), mask=mask_u)})
    b = pa.table({"w": pa.array(rng.random(nr), pa.float32()), "k": pa.array(kr, kt),
                  "b": pa.array(rng.random(nr) < 0.5, mask=mask_b)})
    L, R = Table(a, gpu_ctx), Table(b, gpu_ctx)
    on = dict(left_on=["k"], right_on=["k"], left_prefix="l_", right_prefix="r_")
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", "1")
    got = L.join(R, "inner", "hash", **on)
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", str(1 << 62))
    ref = L.join(R, "inner", "hash", **on)
    assert got.column_names == ref.column_names
    pd.testing.assert_frame_equal(_sorted_df(got), _sorted_df(ref))
    cpu = Table(a, ctx).join(Table(b, ctx), "inner", "hash", **on)  # CPU twin: third oracle
    pd.testing.assert_frame_equal(_sorted_df(got), _sorted_df(cpu), check_dtype=False)


@pytest.mark.parametrize("case", ["int64_many_groups", "int32_nullable", "few_groups", "min_key", "wide_aggs",
                                  "null_keys", "null_keys_int16"])
def test_radix_groupby_matches_global(gpu_ctx, ctx, monkeypatch, case):
    """K8 LDS radix group-by (HLL sizing, partitioned LDS aggregation) vs the global-table path."""
    rng = np.random.default_rng(5)
    n = 400_000
    groups = {"int64_many_groups": 150_000, "int32_nullable": 20_000, "few_groups": 7, "min_key": 5000,
              "wide_aggs": 3000, "null_keys": 40_000, "null_keys_int16": 300}[case]
    k = rng.integers(-groups, groups, n)
    if case == "min_key":
        k[::97] = np.iinfo(np.int64).min
    kt = {"int32_nullable": pa.int32(), "null_keys_int16": pa.int16()}.get(case, pa.int64())
    fmask = rng.random(n) < 0.1 if case == "int32_nullable" else None
    kmask = rng.random(n) < 0.05 if case.startswith("null_keys") else None  # null keys: one group
    if case == "null_keys":
        k[:3] = [np.iinfo(np.int64).min, 7, 0]  # the null group goes above the max (INT64_MIN is a key)
    t = pa.table({"k": pa.array(k, kt, mask=kmask), "f": pa.array(rng.standard_normal(n), mask=fmask),
                  "i": pa.array(rng.integers(-1000, 1000, n), pa.int32())})
    T = Table(t, gpu_ctx)
    aggs = {"f": ["sum", "count", "min", "max", "mean"], "i": ["sum", "min"]} if case == "wide_aggs" else \
        {"f": ["sum", "mean"], "i": ["max", "count"]}
    res = []
    for thr in ("1", str(1 << 62)):
        monkeypatch.setenv("CYLON_RADIX_GROUPBY_MIN_ROWS", thr)
        C.trace_enable(True)
        C.trace_reset()
        df = T.local_groupby("k", aggs).to_pandas()
        c = dict(C.trace_counters())
        C.trace_enable(False)
        if thr == "1" and case.startswith("null_keys"):
            assert c.get("groupby.radix.groups", 0) > 0, c  # the radix path took the nullable key
        res.append(df.sort_values("k").reset_index(drop=True))
    pd.testing.assert_frame_equal(res[0], res[1], check_exact=False, rtol=1e-9, atol=1e-9)
    cpu = Table(t, ctx).local_groupby("k", aggs).to_pandas()  # CPU twin: third oracle
    pd.testing.assert_frame_equal(res[0], cpu.sort_values("k").reset_index(drop=True), check_exact=False,
                                  rtol=1e-9, atol=1e-9, check_dtype=False)


@pytest.mark.parametrize("dtype", ["int64", "float64", "int32", "uint16", "float32", "uint64", "int64_full",
                                   "int64_equal", "int64_offset", "int64_offset_odd"])
@pytest.mark.parametrize("asc", [True, False])
def test_radix_row_sort_matches_index_sort(gpu_ctx, monkeypatch, dtype, asc):
    """Row-moving LSD sort (all columns through LDS-staged passes) vs index sort + gather; stable on ties.
    uint64 keys >= 2^63 and full-range int64 keys (INT64_MIN / INT64_MAX present) take the last pass's
    XOR-on-store path; all-equal keys take the zero-varying-bits branch."""
    rng = np.random.default_rng(9)
    n = 300_000
    if dtype == "uint64":
        k = rng.integers(0, 1 << 63, n, dtype=np.uint64) | (rng.integers(0, 2, n, dtype=np.uint64) << np.uint64(63))
        k[:5] = [0, (1 << 64) - 1, 1 << 63, (1 << 63) - 1, 1]
    elif dtype == "int64_full":
        k = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, n, dtype=np.int64)
        k[:4] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, 0, -1]
        k[4:2000] = k[2000:3996]  # ties
    elif dtype == "int64_equal":
        k = np.full(n, -77, dtype=np.int64)
    elif dtype == "int64_offset":  # far from zero, low 3 bits constant: digits of image - min from bit 3
        k = 10**15 + 8 * rng.integers(0, 100_000, n, dtype=np.int64)
    elif dtype == "int64_offset_odd":  # digits of image - min from bit 0 (the prologue histogram rotated)
        k = -(10**15) + 12345 + rng.integers(0, 3_000_000, n, dtype=np.int64)
    elif dtype.startswith("float"):
        k = rng.standard_normal(n).astype(dtype)
        k[::101] = np.nan
        k[::103] = -0.0
    elif dtype == "uint16":
        k = rng.integers(0, 60000, n).astype(dtype)
    else:
        k = rng.integers(-5000, 5000, n).astype(dtype)  # many ties: stability visible in the payload
    t = pa.table({"p": pa.array(np.arange(n)), "k": k,
                  "q": pa.array(rng.random(n), mask=rng.random(n) < 0.2),
                  "b": pa.array(rng.random(n) < 0.5, mask=rng.random(n) < 0.1)})  # packed bytes
    T = Table(t, gpu_ctx)
    res = []
    for thr in ("1", str(1 << 62)):
        monkeypatch.setenv("CYLON_RADIX_SORT_MIN_ROWS", thr)
        res.append(T.sort("k", ascending=asc).to_pandas())
    pd.testing.assert_frame_equal(res[0], res[1])


# ---------------------------------------------------------------------------
# correctness at bench scale, against independent torch computations
# ---------------------------------------------------------------------------
def _bench_module():
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("cylon_bench", os.path.join(os.path.dirname(__file__), "..",
                                                                              "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("algorithm", ["hash", "sort"])
def test_join_100m_payload_identities(gpu_ctx, algorithm):
    """100M x 100M join (the radix / range LDS paths at scale): row count, key sum and both payload
    sums equal the per-key identities computed independently with torch.bincount (bench.verify_join)."""
    n = 100_000_000
    bm = _bench_module()
    key_range = int(0.99 * n)
    left = bm.make_relation(gpu_ctx, n, key_range, 3, 11, "cuda:0")
    right = bm.make_relation(gpu_ctx, n, key_range, 3, 12, "cuda:0")
    out = left.distributed_join(right, "inner", algorithm, on=[0], left_prefix="l_", right_prefix="r_")
    v = bm.verify_join(gpu_ctx, left, right, out, key_range)
    assert v["ok"], v
    del out
    torch.cuda.empty_cache()


def test_groupby_1b_rows_sums_match_index_add(gpu_ctx):
    """Config 4 shape (1B rows / 10M groups, the radix group-by): every group sum equals torch index_add."""
    n, groups = 1_000_000_000, 10_000_000
    g = torch.Generator(device="cuda").manual_seed(4)
    keys = torch.randint(0, groups, (n,), generator=g, device="cuda")
    x = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
    t = Table.from_torch(gpu_ctx, {"g": keys, "x": x})
    res = t.local_groupby("g", {"x": "sum"}).to_torch()
    ks, sums = list(res.values())[:2]
    ref = torch.zeros(groups, dtype=torch.float64, device="cuda").index_add_(0, keys, x)
    assert ks.numel() == int((torch.bincount(keys, minlength=groups) > 0).sum())
    assert torch.allclose(sums, ref[ks], rtol=1e-9, atol=1e-9)
    del t, keys, x, res, ref
    torch.cuda.empty_cache()


def test_sort_2b_rows_sorted_permutation(gpu_ctx):
    """Config 5 shape (2B int64 rows, the row-moving radix sort): output non-decreasing and the
    same multiset as the input (count, wrapping sum, wrapping sum of squares)."""
    n = 2_000_000_000
    g = torch.Generator(device="cuda").manual_seed(5)
    k = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, device="cuda")
    s = Table.from_torch(gpu_ctx, {"k": k}).sort("k").to_torch()["k"]
    assert s.numel() == n
    assert bool((s[1:] >= s[:-1]).all())
    assert int(s.sum()) == int(k.sum()) and int((s * s).sum()) == int((k * k).sum())
    del s, k
    torch.cuda.empty_cache()


@pytest.mark.parametrize("algorithm", ["hash", "sort"])
def test_radix_join_packed_validity_matches_cpu(gpu_ctx, ctx, monkeypatch, algorithm):
    """Nullable 8-byte payloads on both sides: validity travels packed (8 bytes per row) through the
    radix / range partition passes and the write kernel, then unpacks into the output columns."""
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", "1024")
    rng = np.random.default_rng(31)
    n = 200_000

    def side(prefix, nulls):
        cols = {"k": pa.array(rng.integers(0, 150_000, n))}
        for i, p in enumerate(nulls):
            cols[f"{prefix}{i}"] = pa.array(rng.random(n), mask=rng.random(n) < p)
        cols[f"{prefix}i"] = pa.array(rng.integers(-5, 5, n), mask=rng.random(n) < 0.3)
        return pa.table(cols)
    a, b = side("a", [0.1, 0.0, 0.5]), side("b", [0.2, 0.9])
    res = []
    for cx in (gpu_ctx, ctx):
        res.append(Table(a, cx).join(Table(b, cx), "inner", algorithm, on=["k"], left_prefix="l_",
                                     right_prefix="r_").to_pandas())
    assert len(res[0]) == len(res[1]) > 0
    assert _rows(res[0]) == _rows(res[1])


@pytest.mark.parametrize("mode", ["fused", "fused_rerun", "fused_nullable"])
def test_radix_join_fused_count_matches_exact(gpu_ctx, monkeypatch, mode):
    """Fused count (sampled output estimate + per-partition atomic claims in the write kernel) vs the
    exact count kernel + scan; fused_rerun scales the estimate down so the write kernel overflows its
    allocation, reports the exact total and runs again; nullable payloads use the packed words."""
    rng = np.random.default_rng(21)
    n = 3_000_000
    kl, kr = rng.integers(0, int(0.9 * n), n), rng.integers(0, int(0.9 * n), n)
    mask = rng.random(n) < 0.2 if mode == "fused_nullable" else None
    a = pa.table({"k": kl, "v": pa.array(rng.random(n), mask=mask), "i": rng.integers(-9, 9, n)})
    b = pa.table({"k": kr, "w": rng.random(n)})
    L, R = Table(a, gpu_ctx), Table(b, gpu_ctx)
    on = dict(left_on=["k"], right_on=["k"], left_prefix="l_", right_prefix="r_")
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", "1024")
    monkeypatch.setenv("CYLON_RJ_FUSED_MIN_PARTS", "64")
    if mode == "fused_rerun":
        monkeypatch.setenv("CYLON_RJ_ESTIMATE_SCALE", "0.5")
    from cylon_amd._lib import C
    C.trace_enable(True)
    C.trace_reset()
    got = L.join(R, "inner", "hash", **on)
    c = dict(C.trace_counters())
    C.trace_enable(False)
    assert c.get("join.radix.estimated_rows", 0) > 0, c  # the fused path ran
    assert (c.get("join.radix.estimate_rerun", 0) == 1) == (mode == "fused_rerun"), c
    monkeypatch.setenv("CYLON_RJ_EXACT_COUNT", "1")
    ref = L.join(R, "inner", "hash", **on)
    assert got.row_count == ref.row_count == c["join.radix.rows_out"]
    pd.testing.assert_frame_equal(_sorted_df(got), _sorted_df(ref))


@pytest.mark.parametrize("count_mode", ["fused", "exact"])
def test_radix_join_ranking_guard_falls_back(gpu_ctx, monkeypatch, count_mode):
    """The LSD partition passes after the first must keep the order they receive (wave-atomic
    stable ranking).  CYLON_RP_DEBUG_UNSTABLE=1 breaks that on purpose (block-atomic ranking in
    every pass): the passes' ranking guard -- inside each bucket run of a sorted tile the input rows
    must ascend -- flags it, and the join falls back to the global-table path with a correct result."""
    rng = np.random.default_rng(8)
    n = 6_000_000  # 11 partition bits: two LSD passes
    a = pa.table({"k": rng.integers(0, n, n), "v": rng.random(n)})
    b = pa.table({"k": rng.integers(0, n, n), "w": rng.random(n)})
    L, R = Table(a, gpu_ctx), Table(b, gpu_ctx)
    on = dict(left_on=["k"], right_on=["k"], left_prefix="l_", right_prefix="r_")
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", "1024")
    monkeypatch.setenv("CYLON_RJ_SLOT", "0")  # the guard watches the exact LSD passes (slot mode has no stable pass)
    if count_mode == "fused":
        monkeypatch.setenv("CYLON_RJ_FUSED_MIN_PARTS", "64")
    else:
        monkeypatch.setenv("CYLON_RJ_EXACT_COUNT", "1")
    from cylon_amd._lib import C
    ref = L.join(R, "inner", "hash", **on)
    monkeypatch.setenv("CYLON_RP_DEBUG_UNSTABLE", "1")
    C.trace_enable(True)
    C.trace_reset()
    got = L.join(R, "inner", "hash", **on)
    c = dict(C.trace_counters())
    C.trace_enable(False)
    monkeypatch.delenv("CYLON_RP_DEBUG_UNSTABLE")
    C.rp_set_ranking(0)  # the guard switched the device to ballot ranking: probe again
    assert c.get("join.radix.order_violation_fallback", 0) == 1, c
    assert got.row_count == ref.row_count
    pd.testing.assert_frame_equal(_sorted_df(got), _sorted_df(ref))


@pytest.mark.parametrize("dtype", ["int64", "float64"])
def test_verify_sort_config(gpu_ctx, dtype):
    """config verify_sort=1: the sorted result is checked in order-image space (nulls last)."""
    from cylon_amd._lib import C
    rng = np.random.default_rng(2)
    n = 5_000_000
    k = rng.integers(-10**9, 10**9, n).astype(dtype)
    t = Table(pa.table({"k": pa.array(k, mask=rng.random(n) < 0.01), "p": np.arange(n)}), gpu_ctx)
    gpu_ctx.add_config("verify_sort", "1")
    C.trace_enable(True)
    C.trace_reset()
    try:
        for asc in (True, False):
            t.sort("k", ascending=asc)
        c = dict(C.trace_counters())
    finally:
        gpu_ctx.add_config("verify_sort", "0")
        C.trace_enable(False)
    assert c.get("sort.verified", 0) == 2, c


@pytest.mark.parametrize("op", ["join", "sort", "union", "groupby"])
def test_xcd_tile_schedule_matches_chunk_schedule(gpu_ctx, monkeypatch, op):
    """XCD-tile radix passes (wave-atomic ranking: per-tile histograms or look-back offsets, tiles
    claimed in order per XCD) against the per-block-chunk histogram schedule the ballot ranking runs
    for 1-2 column passes (rp_set_ranking(2): 512-thread blocks): identical results, including the
    stable order of the row sort."""
    rng = np.random.default_rng(23)
    n = 3_000_000  # > 256 tiles per pass: every XCD chunk is non-trivial
    a = pa.table({"k": rng.integers(0, n // 3, n), "v": rng.random(n), "i": rng.integers(-50, 50, n)})
    b = pa.table({"k": rng.integers(0, n // 3, n), "v": rng.random(n), "i": rng.integers(-50, 50, n)})
    A, B = Table(a, gpu_ctx), Table(b, gpu_ctx)
    for k, v in (("CYLON_RADIX_JOIN_MIN_ROWS", "1024"), ("CYLON_RADIX_SORT_MIN_ROWS", "1024"),
                 ("CYLON_RADIX_GROUPBY_MIN_ROWS", "1024")):
        monkeypatch.setenv(k, v)
    res = []
    for mode in (2, 1):
        C.rp_set_ranking(mode)
        if op == "join":
            res.append(_sorted_df(A.join(B, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_")))
        elif op == "sort":
            res.append(A.sort("i").to_pandas())  # many ties: the order within them must match exactly
        elif op == "union":
            res.append(_sorted_df(A.union(B)))
        else:
            res.append(A.local_groupby("k", {"v": ["sum"], "i": ["max"]}).to_pandas()
                       .sort_values("k").reset_index(drop=True))
    C.rp_set_ranking(0)
    if op == "groupby":
        pd.testing.assert_frame_equal(res[0], res[1], check_exact=False, rtol=1e-12, atol=1e-12)
    else:
        pd.testing.assert_frame_equal(res[0], res[1])
