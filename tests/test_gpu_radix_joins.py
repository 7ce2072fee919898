"""LDS radix join (kernels/radix_join.hip k_rj_count / k_rj_write) beyond the inner single-key
headline shape: outer joins (unmatched probe rows, unmatched build rows through the LDS matched
flags, both), several key columns (exact composite key or a verified 64-bit hash), var-width
payload columns (gathered by row number after the join) and the sampled-estimate skew check.
Every case is compared with the CPU twin of the same join (reference: join/hash_join.cpp:21-186,
join/join_utils.cpp:126-181)."""
import numpy as np
import pandas as pd
import pyarrow as pa
import pytest
import torch

from cylon_amd import Table
from cylon_amd._lib import C

pytestmark = pytest.mark.gpu


def _canon(df):
    df = df[sorted(df.columns)]
    return df.sort_values(list(df.columns), kind="mergesort", na_position="last").reset_index(drop=True)


def _join(gpu_ctx, ctx, a, b, how, on, monkeypatch, algorithm="hash"):
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", "1024")
    kw = dict(left_on=on, right_on=on, left_prefix="l_", right_prefix="r_")
    C.trace_enable(True)
    C.trace_reset()
    got = Table(a, gpu_ctx).join(Table(b, gpu_ctx), how, algorithm, **kw)
    c = dict(C.trace_counters())
    C.trace_enable(False)
    exp = Table(a, ctx).join(Table(b, ctx), how, algorithm, **kw)
    return got.to_pandas(), exp.to_pandas(), c


@pytest.mark.parametrize("how", ["left", "right", "outer"])
@pytest.mark.parametrize("left_small", [True, False])
def test_radix_outer_join_matches_cpu(gpu_ctx, ctx, monkeypatch, how, left_small):
    """The smaller side is built in LDS: left_small makes the left side the build side (so a LEFT
    join preserves build rows: matched flags), else the probe side (lone unmatched probe rows)."""
    rng = np.random.default_rng(5)
    nl, nr = (300_000, 500_000) if left_small else (500_000, 300_000)
    a = pa.table({"k": rng.integers(0, 600_000, nl), "v": rng.random(nl),
                  "i": pa.array(rng.integers(-9, 9, nl), mask=rng.random(nl) < 0.1)})
    b = pa.table({"k": rng.integers(0, 600_000, nr), "w": rng.random(nr)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["k"], monkeypatch)
    assert c.get("join.radix.outer", 0) > 0, c
    assert c["join.radix.rows_out"] == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "left", "outer"])
@pytest.mark.parametrize("nkeys", [1, 2])
def test_radix_join_nullable_int_keys(gpu_ctx, ctx, monkeypatch, how, nkeys):
    """Nullable integer keys join on the radix path as an exact composite whose null code (one past
    the largest valid field) makes nulls match nulls, as on the CPU twin (docs/semantics.md); the
    unpacked key columns come back null there."""
    rng = np.random.default_rng(16)
    n = 300_000

    def side(seed_off):
        k = rng.integers(-50_000, 150_000, n)
        km = np.zeros(n, bool)
        km[rng.choice(n, 40, replace=False)] = True  # 40 null keys a side: 1600 null-null rows
        cols = {"k": pa.array(k, mask=km)}
        if nkeys == 2:
            g = rng.integers(0, 4, n).astype(np.int16)
            gm = np.zeros(n, bool)
            gm[rng.choice(n, 25, replace=False)] = True
            cols["g"] = pa.array(g, mask=gm)
        cols["v" if seed_off == 0 else "w"] = rng.random(n)
        return pa.table(cols)

    a, b = side(0), side(1)
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["k", "g"][:nkeys], monkeypatch)
    assert c.get("join.radix.composite_key", 0) == 1, c
    assert list(got.columns) == list(exp.columns)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "left", "outer"])
def test_radix_join_composite_two_keys(gpu_ctx, ctx, monkeypatch, how):
    """Two int keys -> one exact composite (composite_key_pack); the proxy tables carry it in place
    of the key columns and composite_key_unpack rebuilds them (null where the side is absent)."""
    rng = np.random.default_rng(6)
    n = 400_000
    a = pa.table({"k": rng.integers(0, 200_000, n), "g": rng.integers(-3, 3, n).astype(np.int32),
                  "v": rng.random(n)})
    b = pa.table({"k": rng.integers(0, 200_000, n), "g": rng.integers(-3, 3, n).astype(np.int32),
                  "w": rng.random(n)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["k", "g"], monkeypatch)
    assert c.get("join.radix.composite_key", 0) == 1 and c.get("join.radix.composite_unpacked", 0) == 4, c
    assert list(got.columns) == list(exp.columns)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


def test_radix_join_composite_mixed_widths_var_payload(gpu_ctx, ctx, monkeypatch):
    """Three keys of widths 8 / 4 / 1 (signed, signed, unsigned) with negative minima, keys not
    leading the column order, and a string payload (composite proxy + row-number gather)."""
    rng = np.random.default_rng(16)
    n = 300_000
    def mk(seed_off, tag):
        r = np.random.default_rng(60 + seed_off)
        return pa.table({"s": [f"{tag}{x}" for x in r.integers(0, 500, n)],
                         "k": r.integers(-(1 << 40), -(1 << 40) + 90_000, n),
                         "x": r.random(n),
                         "h": r.integers(-70_000, -69_990, n).astype(np.int32),
                         "u": r.integers(250, 256, n).astype(np.uint8)})
    a, b = mk(0, "a"), mk(1, "b")
    got, exp, c = _join(gpu_ctx, ctx, a, b, "left", ["k", "h", "u"], monkeypatch)
    assert c.get("join.radix.composite_key", 0) == 1 and c.get("join.radix.var_gather", 0) == 1, c
    assert list(got.columns) == list(exp.columns)
    assert len(exp) > n
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


def test_radix_join_hashed_keys_verified(gpu_ctx, ctx, monkeypatch):
    """Key spans too wide to pack into 63 bits: a 64-bit row hash partitions and matches, and the
    output's key columns are compared (a collision would send the join to the exact path)."""
    rng = np.random.default_rng(7)
    n = 300_000
    big = rng.integers(-(1 << 62), 1 << 62, 50_000)
    a = pa.table({"k": rng.choice(big, n), "g": rng.choice(big, n) >> 20, "v": rng.random(n)})
    b = pa.table({"k": rng.choice(big, n), "g": rng.choice(big, n) >> 20, "w": rng.random(n)})
    b = pa.table({"k": pa.concat_arrays([a["k"].combine_chunks()[:1000], b["k"].combine_chunks()[1000:]]),
                  "g": pa.concat_arrays([a["g"].combine_chunks()[:1000], b["g"].combine_chunks()[1000:]]),
                  "w": b["w"]})
    got, exp, c = _join(gpu_ctx, ctx, a, b, "inner", ["k", "g"], monkeypatch)
    assert c.get("join.radix.hashed_key", 0) == 1 and c.get("join.radix.hash_collision_fallback", 0) == 0, c
    assert len(exp) >= 1000
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "left", "outer"])
def test_radix_join_var_width_payload(gpu_ctx, ctx, monkeypatch, how):
    rng = np.random.default_rng(8)
    n = 200_000
    a = pa.table({"k": rng.integers(0, 250_000, n), "s": [f"a{x}" for x in rng.integers(0, 999, n)],
                  "v": rng.random(n)})
    b = pa.table({"k": rng.integers(0, 250_000, n), "t": pa.array([f"bb{x}" for x in rng.integers(0, 99, n)],
                                                                mask=rng.random(n) < 0.05)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["k"], monkeypatch)
    assert c.get("join.radix.var_gather", 0) == 1, c
    assert list(got.columns) == list(exp.columns)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


def test_radix_outer_sort_algorithm_uses_radix(gpu_ctx, ctx, monkeypatch):
    rng = np.random.default_rng(9)
    n = 300_000
    a = pa.table({"k": rng.integers(0, 400_000, n), "v": rng.random(n)})
    b = pa.table({"k": rng.integers(0, 400_000, n), "w": rng.random(n)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, "outer", ["k"], monkeypatch, algorithm="sort")
    assert c.get("join.radix.outer", 0) == 3, c
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


def test_radix_join_hot_key_sample_is_counted_exactly(gpu_ctx, monkeypatch):
    """a hot probe key in a sampled partition must not inflate the fused output
    estimate 32x; the skew check counts such a sample exactly (or the estimate path reruns)."""
    rng = np.random.default_rng(10)
    nb, npr = 1_000_000, 2_000_000
    hot = np.arange(16) * 7919 + 5
    bk = np.concatenate([rng.integers(0, 1_000_000, nb - 16 * 100), np.repeat(hot, 100)])
    pk = np.concatenate([rng.integers(0, 1_000_000, npr - 16 * 3000), np.repeat(hot, 3000)])
    a = pa.table({"k": bk, "v": rng.random(nb)})
    b = pa.table({"k": pk, "w": rng.random(npr)})
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", "1024")
    monkeypatch.setenv("CYLON_RJ_FUSED_MIN_PARTS", "64")
    C.trace_enable(True)
    C.trace_reset()
    got = Table(a, gpu_ctx).join(Table(b, gpu_ctx), "inner", "hash", on=["k"])
    c = dict(C.trace_counters())
    C.trace_enable(False)
    exp = len(pd.DataFrame({"k": bk}).merge(pd.DataFrame({"k": pk}), on="k"))
    assert got.row_count == exp
    if c.get("join.radix.estimated_rows"):  # the fused estimate was used: it must not be inflated
        assert c["join.radix.estimated_rows"] < 3 * exp, c


# ---- slot-mode partitions (radix_slot_rows_pass): MSD second pass into fixed-size partition slots
@pytest.mark.parametrize("how", ["inner", "left", "outer"])
def test_radix_join_slot_partitions_match_cpu(gpu_ctx, ctx, monkeypatch, how):
    """CYLON_RJ_EXTRA_BITS=4 gives 2^12+ partitions at 1M rows, so both sides take the two-pass
    slot mode (high digit with exact offsets, then the low digit into slots without a histogram);
    nullable payloads travel as packed validity words through the slots."""
    monkeypatch.setenv("CYLON_RJ_EXTRA_BITS", "4")
    rng = np.random.default_rng(31)
    nl, nr = 1_000_000, 1_200_000
    a = pa.table({"k": rng.integers(0, 1_500_000, nl), "v": rng.random(nl),
                  "i": pa.array(rng.integers(-9, 9, nl), mask=rng.random(nl) < 0.1)})
    b = pa.table({"k": rng.integers(0, 1_500_000, nr), "w": rng.random(nr)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["k"], monkeypatch)
    assert c.get("join.radix.slot_sides", 0) == 2 and c.get("join.radix.slot_overflow", 0) == 0, c
    assert c["join.radix.rows_out"] == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


def test_radix_join_slot_overflow_repartitions_exactly(gpu_ctx, ctx, monkeypatch):
    """A hot probe key fills one partition far beyond its slot: that side is partitioned again
    with exact offsets (join.radix.slot_overflow) and the result is unchanged."""
    monkeypatch.setenv("CYLON_RJ_EXTRA_BITS", "4")
    rng = np.random.default_rng(32)
    nl, nr = 800_000, 1_000_000
    kr = rng.integers(0, 1_000_000, nr)
    kr[: 20_000] = 4242  # one partition receives 20k extra probe rows (slot ~ 400)
    a = pa.table({"k": rng.integers(0, 1_000_000, nl), "v": rng.random(nl)})
    b = pa.table({"k": kr, "w": rng.random(nr)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, "inner", ["k"], monkeypatch)
    assert c.get("join.radix.slot_overflow", 0) >= 1, c
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("left_small", [True, False])
@pytest.mark.parametrize("share", ["1", "0"])
def test_radix_inner_join_shared_key_column(gpu_ctx, ctx, monkeypatch, left_small, share):
    """Inner joins on one integer key column per side write the probe side's key column once and
    give the build side's output key column the same buffer (join.radix.shared_key_column); the
    key sits behind a nullable payload column so the build column list's index shift is exercised.
    CYLON_RJ_SHARE_KEY=0 writes both columns; the results are equal either way."""
    monkeypatch.setenv("CYLON_RJ_SHARE_KEY", share)
    rng = np.random.default_rng(41)
    nl, nr = (300_000, 500_000) if left_small else (500_000, 300_000)
    a = pa.table({"i": pa.array(rng.integers(-9, 9, nl), mask=rng.random(nl) < 0.1),
                  "k": rng.integers(0, 600_000, nl), "v": rng.random(nl)})
    b = pa.table({"w": rng.random(nr), "k": rng.integers(0, 600_000, nr)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, "inner", ["k"], monkeypatch)
    assert c.get("join.radix.shared_key_column", 0) == (1 if share == "1" else 0), c
    assert c["join.radix.rows_out"] == len(exp)
    assert (got["l_k"].to_numpy() == got["r_k"].to_numpy()).all()
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


def test_shared_key_column_to_torch_is_copy_on_second_name(gpu_ctx, monkeypatch):
    """The inner join's two key columns share one device buffer natively; to_torch() hands the
    second name a copy, so an in-place write through one tensor leaves the other (and the table)
    unchanged."""
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", "1024")
    monkeypatch.setenv("CYLON_RJ_SHARE_KEY", "1")
    rng = np.random.default_rng(43)
    a = pa.table({"k": rng.integers(0, 200_000, 300_000), "v": rng.random(300_000)})
    b = pa.table({"k": rng.integers(0, 200_000, 300_000), "w": rng.random(300_000)})
    out = Table(a, gpu_ctx).join(Table(b, gpu_ctx), "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_")
    cols = {c.name: c for c in out.native.columns()}
    assert cols["l_k"].data.data_ptr() == cols["r_k"].data.data_ptr()  # shared natively
    t = out.to_torch()
    assert t["l_k"].data_ptr() != t["r_k"].data_ptr()
    before = t["r_k"].clone()
    t["l_k"].add_(1)
    assert torch.equal(t["r_k"], before)
    t["l_k"].sub_(1)  # (l_k is the table's own buffer: restore it)
    assert torch.equal(t["l_k"], t["r_k"])


# ---- LDS radix group-by (kernels/radix_groupby.hip) beyond one integer key + SUM/COUNT/MIN/MAX/MEAN
def _groupby_both(T, keys, aggs, monkeypatch):
    """[radix path, GPU global-table path] results and counters; both are also checked against the
    CPU twin of the group-by (kernels/cpu_groupby.cpp, an independent implementation), so an
    encoding bug shared by the two GPU paths (composite key, float canonical bits, null code) fails."""
    res, counters = [], []
    for thr in ("1", str(1 << 62)):  # radix path, then the global-table path
        monkeypatch.setenv("CYLON_RADIX_GROUPBY_MIN_ROWS", thr)
        C.trace_enable(True)
        C.trace_reset()
        df = T.local_groupby(keys, aggs).to_pandas()
        counters.append(dict(C.trace_counters()))
        C.trace_enable(False)
        res.append(df.sort_values(keys).reset_index(drop=True))
    cpu = T.to_cpu().local_groupby(keys, aggs).to_pandas().sort_values(keys).reset_index(drop=True)
    assert list(cpu.columns) == list(res[0].columns)
    pd.testing.assert_frame_equal(res[0], cpu, check_exact=False, rtol=1e-8, atol=1e-8, check_dtype=False)
    return res, counters


@pytest.mark.parametrize("case", ["six_planes", "eight_planes"])
def test_radix_groupby_many_accumulators(gpu_ctx, monkeypatch, case):
    """5-8 accumulator planes (the 8-plane LDS table; idle planes are counts of their own): sums,
    means, min / max and VAR / STD over three columns -- against the CPU twin and the global path."""
    rng = np.random.default_rng(14)
    n = 500_000
    t = pa.table({"k": rng.integers(0, 40_000, n), "x": rng.standard_normal(n) * 10.0,
                  "y": pa.array(rng.integers(-1000, 1000, n), mask=rng.random(n) < 0.03),
                  "z": rng.random(n)})
    T = Table(t, gpu_ctx)
    aggs = ({"x": ["sum", "var"], "y": ["max", "mean"]} if case == "six_planes"
            else {"x": ["std", "min"], "y": ["mean", "max"], "z": ["sum"]})
    res, cnt = _groupby_both(T, ["k"], aggs, monkeypatch)
    assert cnt[0].get("groupby.radix.groups", 0) == len(res[0]), cnt[0]


@pytest.mark.parametrize("case", ["var_std", "two_keys", "float_key", "two_keys_var", "two_keys_nulls"])
def test_radix_groupby_extended(gpu_ctx, monkeypatch, case):
    """VAR / STDDEV through the M2 accumulator (second in-block pass over a partition's rows), two
    integer keys through an exact composite key, a float key through canonical bits -- against
    the global-table path."""
    rng = np.random.default_rng(12)
    n = 600_000
    nulls = case == "two_keys_nulls"  # nullable keys: a null code per key field of the composite
    t = pa.table({"k": pa.array(rng.integers(0, 50_000, n), mask=(rng.random(n) < 0.01) if nulls else None),
                  "g": pa.array(rng.integers(-4, 4, n).astype(np.int16), mask=(rng.random(n) < 0.02) if nulls else None),
                  "x": pa.array(rng.standard_normal(n) + 100.0, mask=rng.random(n) < 0.05),
                  "f": np.round(rng.standard_normal(n), 1)})
    T = Table(t, gpu_ctx)
    keys, aggs = {"var_std": (["k"], {"x": ["sum", "mean", "std"]}),
                  "two_keys": (["k", "g"], {"x": ["sum", "max"], "f": ["count"]}),
                  "float_key": (["f"], {"x": ["sum", "min"], "k": ["max"]}),
                  "two_keys_var": (["k", "g"], {"x": ["var", "mean"]}),
                  "two_keys_nulls": (["k", "g"], {"x": ["sum", "count"], "f": ["max"]})}[case]
    res, cnt = _groupby_both(T, keys, aggs, monkeypatch)
    assert cnt[0].get("groupby.radix.groups", 0) == len(res[0]), cnt[0]
    if len(keys) > 1:
        assert cnt[0].get("groupby.radix.composite_key", 0) == 1, cnt[0]
    pd.testing.assert_frame_equal(res[0], res[1], check_exact=False, rtol=1e-8, atol=1e-8)


@pytest.mark.parametrize("fmt", ["s{:06d}", "key-{:09d}", "key-{:020d}", "key-{:011d}/bin"])
def test_radix_groupby_string_word_key(gpu_ctx, monkeypatch, fmt):
    """A fixed-length string key groups on the LDS radix path by its invertible word key: words
    1..W-1 ride along as MIN / MAX accumulators (equal in every group = exact), and the output key
    bytes are rebuilt from the key and the MIN words.  7 bytes (one word), 13 (unaligned), 24
    (three aligned words) and 19-byte binary; against the global path and the CPU twin."""
    rng = np.random.default_rng(14)
    n = 600_000
    ids = rng.integers(0, 40_000, n)
    vals = [fmt.format(x).encode() for x in ids] if fmt.endswith("/bin") else [fmt.format(x) for x in ids]
    t = pa.table({"s": pa.array(vals), "x": rng.standard_normal(n), "k": rng.integers(-50, 50, n)})
    res, cnt = _groupby_both(Table(t, gpu_ctx), ["s"], {"x": ["sum", "mean"], "k": ["max"]}, monkeypatch)
    assert cnt[0].get("groupby.radix.word_key", 0) == 1, cnt[0]
    assert cnt[0].get("groupby.radix.groups", 0) == len(res[0]) == len(np.unique(ids)), cnt[0]
    pd.testing.assert_frame_equal(res[0], res[1], check_exact=False, rtol=1e-8, atol=1e-8)


@pytest.mark.parametrize("case", ["var_8_32", "var_1_100_binary", "fixed_40_too_wide"])
def test_radix_groupby_hashed_string_key(gpu_ctx, monkeypatch, case):
    """Variable-length string / binary keys (and fixed-length keys whose MIN / MAX words would not fit
    the 8 accumulator planes) group on the LDS radix path by a 64-bit hash of the bytes, verified by
    MIN == MAX of an independent 64-bit hash per group; the output key is each group's first row's
    bytes.  Against the global path and the CPU twin."""
    rng = np.random.default_rng(15)
    n = 600_000
    ids = rng.integers(0, 40_000, n)
    if case == "fixed_40_too_wide":
        vals = [f"key-{x:036d}" for x in ids]
    else:
        lo, hi = (8, 32) if case == "var_8_32" else (1, 100)
        vals = _var_strings(rng, ids, lo, hi, binary=case.endswith("binary"))
    t = pa.table({"s": pa.array(vals), "x": rng.standard_normal(n), "k": rng.integers(-50, 50, n)})
    res, cnt = _groupby_both(Table(t, gpu_ctx), ["s"], {"x": ["sum", "mean"], "k": ["max"]}, monkeypatch)
    assert cnt[0].get("groupby.radix.hashed_string_key", 0) == 1, cnt[0]
    assert cnt[0].get("groupby.radix.word_key_too_wide", 0) == (1 if case == "fixed_40_too_wide" else 0), cnt[0]
    assert cnt[0].get("groupby.radix.groups", 0) == len(res[0]) == len(np.unique(ids)), cnt[0]
    pd.testing.assert_frame_equal(res[0], res[1], check_exact=False, rtol=1e-8, atol=1e-8)


@pytest.mark.parametrize("case", ["median_alone", "sum_q25_nullable", "int_values_two_q", "two_keys_q90",
                                  "mixed_group_sizes"])
def test_radix_groupby_quantile(gpu_ctx, monkeypatch, case):
    """QUANTILE on the LDS radix path: (group key, value) rows partitioned by the key hash and sorted
    per partition in LDS, each group's quantile by the global path's type-2 rule (nulls excluded; a
    group whose values are all null gets a null quantile), LEFT-joined to the other aggregates.
    Against the global path and the CPU twin."""
    rng = np.random.default_rng(17)
    n = 700_000
    k = rng.integers(0, 30_000, n)
    if case == "mixed_group_sizes":  # ~230-row groups (counted per row) next to 1-row and ~30-row ones
        k = np.where(rng.random(n) < 0.5, rng.integers(0, 1_500, n),
                     np.where(rng.random(n) < 0.5, rng.integers(100_000, 300_000, n), rng.integers(-6_000, 0, n)))
    xmask = (rng.random(n) < 0.05) | (k % 1009 == 0)  # nulls, and groups whose x is all null
    t = pa.table({"k": k, "g": rng.integers(-3, 3, n).astype(np.int16),
                  "x": pa.array(np.round(rng.standard_normal(n) * 100.0, 1),
                               mask=xmask if case in ("sum_q25_nullable", "mixed_group_sizes") else None),
                  "i": rng.integers(-1000, 1000, n).astype(np.int32)})
    keys, aggs = {"median_alone": (["k"], {"x": ["median"]}),
                  "sum_q25_nullable": (["k"], {"x": ["sum", ("quantile", 0.25)]}),
                  "int_values_two_q": (["k"], {"i": [("quantile", 0.5), ("quantile", 0.9)], "x": ["max"]}),
                  "two_keys_q90": (["k", "g"], {"x": [("quantile", 0.9), "mean"]}),
                  "mixed_group_sizes": (["k"], {"x": [("quantile", 0.75), "sum", "min", "max", "count", "mean"]})}[case]
    res, cnt = _groupby_both(Table(t, gpu_ctx), keys, aggs, monkeypatch)
    nq = 2 if case == "int_values_two_q" else 1
    assert cnt[0].get("groupby.radix.quantile", 0) == nq, cnt[0]
    assert cnt[0].get("groupby.radix.quantile_overflow_fallback", 0) == 0, cnt[0]
    # SUM / COUNT / MEAN / MIN / MAX of the quantile's own float64 column come from the quantile kernel
    fused = {"sum_q25_nullable": 1, "two_keys_q90": 1, "mixed_group_sizes": 5}.get(case, 0)
    assert cnt[0].get("groupby.radix.quantile_fused_aggs", 0) == fused, cnt[0]
    # quantiles, min / max / count are order statistics and counts: equal to 1e-12.  Sums and means
    # add a group's values in an order that differs between the paths (and, for groups counted by
    # LDS atomics, between runs): ~230 values of magnitude <= ~500 that cancel to ~0.4 can differ by
    # a few 1e-12 absolute, so those columns get an absolute tolerance of 1e-8
    summed = [c for c in res[0].columns if c.startswith(("sum_", "mean_"))]
    pd.testing.assert_frame_equal(res[0].drop(columns=summed), res[1].drop(columns=summed), check_exact=False,
                                  rtol=1e-12, atol=1e-12)
    if summed:
        pd.testing.assert_frame_equal(res[0][summed], res[1][summed], check_exact=False, rtol=1e-12, atol=1e-8)


@pytest.mark.parametrize("case", ["with_sum", "alone", "two_keys"])
def test_radix_groupby_nunique(gpu_ctx, monkeypatch, case):
    """NUNIQUE on the radix path: distinct (keys, x) pairs by a radix group-by, counted per key, LEFT
    joined to the other aggregates (a group whose x is all null counts 0) -- against the global path."""
    rng = np.random.default_rng(13)
    n = 600_000
    k = rng.integers(0, 40_000, n)
    g = rng.integers(0, 6, n).astype(np.int32)
    gmask = (rng.random(n) < 0.1) | (k % 997 == 0)  # nulls, and some groups with every value null
    t = pa.table({"k": k, "h": rng.integers(-2, 2, n).astype(np.int16), "g": pa.array(g, mask=gmask),
                  "x": rng.random(n)})
    T = Table(t, gpu_ctx)
    keys, aggs = {"with_sum": (["k"], {"g": ["nunique"], "x": ["sum", "max"]}),
                  "alone": (["k"], {"g": "nunique"}),
                  "two_keys": (["k", "h"], {"x": ["mean"], "g": ["nunique"]})}[case]
    res, cnt = _groupby_both(T, keys, aggs, monkeypatch)
    assert cnt[0].get("groupby.radix.nunique_columns", 0) == 1, cnt[0]
    assert list(res[0].columns) == list(res[1].columns)
    pd.testing.assert_frame_equal(res[0], res[1], check_exact=False, rtol=1e-9, atol=1e-9, check_dtype=False)


@pytest.mark.parametrize("nacc", [2, 3])
def test_radix_groupby_3m_rows_1m_groups(gpu_ctx, monkeypatch, nacc):
    """The round-3 fault shape: 3M rows / ~1M groups with two and three accumulators (the <2, 2048>
    and <3, 2048> LDS tables)."""
    rng = np.random.default_rng(23)
    n = 3_000_000
    t = pa.table({"k": rng.integers(0, n // 3, n), "v": rng.random(n), "i": rng.integers(-50, 50, n)})
    T = Table(t, gpu_ctx)
    aggs = {2: {"v": ["sum"], "i": ["max"]}, 3: {"v": ["sum", "max"], "i": ["max"]}}[nacc]
    res, cnt = _groupby_both(T, ["k"], aggs, monkeypatch)
    assert cnt[0].get("groupby.radix.groups", 0) == len(res[0]) > 900_000, cnt[0]
    pd.testing.assert_frame_equal(res[0], res[1], check_exact=False, rtol=1e-9, atol=1e-9)


def _zipf_ranks(rng, n, s, key_range):
    u = rng.random(n)
    r = np.floor(np.maximum(u, 1e-300) ** (-1.0 / (s - 1.0)))
    r = np.minimum(r, 2.0**62).astype(np.int64) % key_range
    return (r * 0x9E3779B1) % key_range


@pytest.mark.parametrize("how", ["inner", "left", "right", "outer"])
@pytest.mark.parametrize("shape", ["hotbuild", "zipfprobe"])
def test_radix_join_skewed_partitions_split(gpu_ctx, ctx, monkeypatch, how, shape):
    """Skew is handled per partition (kernel_decls.inc RJSplit): hot build keys beyond the LDS
    capacity are joined in build chunks, a hot probe partition in probe chunks; the rest of the join
    stays on the per-partition path and nothing falls back to the global table.  Outer joins defer a
    split side's unmatched rows to emission items.  Against the CPU twin at 2M x 2M."""
    rng = np.random.default_rng(41)
    n = 2_000_000
    kr = int(0.99 * n)
    lk = rng.integers(0, kr, n)
    rk = rng.integers(0, kr, n)
    if shape == "hotbuild":  # right = build side (equal sizes): 8 hot keys x 6k duplicates
        pos = rng.choice(n, 8 * 6000, replace=False)
        rk[pos] = np.repeat(np.arange(8) * (kr // 8) + 3, 6000)
    else:  # probe (left) keys Zipf(1.1): the hottest key holds ~6.7 % of the rows
        lk = _zipf_ranks(rng, n, 1.1, kr)
    a = pa.table({"k": lk, "v": rng.random(n)})
    b = pa.table({"k": rk, "w": rng.random(n), "i": pa.array(rng.integers(-5, 5, n), mask=rng.random(n) < 0.05)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["k"], monkeypatch)
    assert c.get("join.radix.split_partitions", 0) > 0, c
    assert c.get("join.radix.overflow_fallback", 0) == 0, c
    assert c["join.radix.rows_out"] == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "left", "right", "outer"])
def test_radix_join_forced_small_build_chunks(gpu_ctx, ctx, monkeypatch, how):
    """CYLON_RJ_SPLIT_ROWS=64 splits every partition with more than 64 build rows into 64-row build
    chunks: most partitions run as items, both outer sides deferred (many chunks per partition)."""
    rng = np.random.default_rng(43)
    nl, nr = 400_000, 300_000
    a = pa.table({"k": rng.integers(0, 200_000, nl), "v": rng.random(nl)})
    b = pa.table({"k": rng.integers(0, 200_000, nr), "w": rng.random(nr)})
    monkeypatch.setenv("CYLON_RJ_SPLIT_ROWS", "64")
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["k"], monkeypatch)
    assert c.get("join.radix.split_items", 0) > 100, c
    assert c["join.radix.rows_out"] == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("case", ["narrow_far_from_zero", "wide_fallback", "uint64_top"])
@pytest.mark.parametrize("how", ["inner", "outer"])
def test_radix_join_narrowed_keys(gpu_ctx, ctx, monkeypatch, case, how):
    """Narrowed partition keys (kernel_decls.inc NarrowKeys): keys within 2^31 of the left table's
    first key travel as uint32 offsets (also far from zero, and for uint64 keys near 2^64); keys
    spanning more than 2^32 are detected by the first pass and joined as int64 keys."""
    rng = np.random.default_rng(47)
    n = 1_500_000
    if case == "narrow_far_from_zero":
        lo, span, typ = -(1 << 62), 1 << 30, pa.int64()
    elif case == "wide_fallback":
        lo, span, typ = -(1 << 40), 1 << 41, pa.int64()
    else:
        lo, span, typ = (1 << 63) + (1 << 62), 1 << 29, pa.uint64()
    ka = rng.integers(0, span // 2, n).astype(np.uint64) * 2 + np.uint64(lo % (1 << 64))
    kb = rng.integers(0, span // 2, n).astype(np.uint64) * 2 + np.uint64(lo % (1 << 64))
    kb[: n // 3] = ka[rng.integers(0, n, n // 3)]  # plenty of matches
    if typ == pa.int64():
        ka, kb = ka.view(np.int64), kb.view(np.int64)
    a = pa.table({"k": pa.array(ka, typ), "v": rng.random(n)})
    b = pa.table({"k": pa.array(kb, typ), "w": rng.random(n)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["k"], monkeypatch)
    if case == "wide_fallback":
        assert c.get("join.radix.narrow_fallback", 0) == 1, c
    elif case == "narrow_far_from_zero":
        assert c.get("join.radix.narrow_keys", 0) == 1 and c.get("join.radix.narrow_fallback", 0) == 0, c
    # (uint64 keys join through their 64-bit image, which is not the column itself: not narrowed)
    assert c["join.radix.rows_out"] == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "left", "outer"])
@pytest.mark.parametrize("keys", [["s"], ["s", "k"]])
def test_radix_join_string_keys(gpu_ctx, ctx, monkeypatch, how, keys):
    """String keys on the LDS radix path: the row hash of the key columns is partitioned and matched
    in LDS; the fixed-length (13-byte) key strings travel as two int64 word columns (no gather by row
    number) and every output row's key words are compared (a 64-bit collision would be dropped /
    fall back).  Against the CPU twin."""
    monkeypatch.setenv("CYLON_RJ_SHARE_KEY", "1")
    rng = np.random.default_rng(53)
    n = 1_200_000
    ids_a = rng.integers(0, 900_000, n)
    ids_b = rng.integers(0, 900_000, n)
    a = pa.table({"s": pa.array([f"key-{x:09d}" for x in ids_a]), "k": ids_a % 7, "v": rng.random(n)})
    b = pa.table({"s": pa.array([f"key-{x:09d}" for x in ids_b]), "k": ids_b % 7, "w": rng.random(n)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, keys, monkeypatch)
    assert c.get("join.radix.var_key", 0) >= 1 and c.get("join.radix.hashed_key", 0) == 1, c
    assert c.get("join.radix.hash_collision_fallback", 0) == 0, c
    assert c.get("join.radix.word_columns", 0) == 2 and c.get("join.radix.var_gather", 0) == 0, c
    # inner on the string alone: the build side's word-key column is the probe side's (radix_join)
    # and the right key column is the verified left one's buffers
    assert c.get("join.radix.shared_key_column", 0) == (2 if how == "inner" and keys == ["s"] else 0), c
    assert c["join.radix.rows_out"] == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "outer"])
@pytest.mark.parametrize("fmt", ["s{:06d}", "key-{:020d}", "key-{:011d}/bin"])
def test_radix_join_string_word_key(gpu_ctx, ctx, monkeypatch, how, fmt):
    """One fixed-length string key per side joins on its invertible word key (hash.hpp word_key_*):
    7-byte strings (one word: the key IS the string, no verification), 24 bytes (three aligned
    words: word 0 rebuilt from the key after the join) and 19-byte binary (unaligned tail word).
    Output key bytes must round-trip exactly.  Against the CPU twin."""
    rng = np.random.default_rng(61)
    n = 1_000_000
    ids_a, ids_b = rng.integers(0, 800_000, n), rng.integers(0, 800_000, n)
    enc = (lambda v: [fmt.format(x).encode() for x in v]) if fmt.endswith("/bin") else \
        (lambda v: [fmt.format(x) for x in v])
    a = pa.table({"s": pa.array(enc(ids_a)), "v": rng.random(n)})
    b = pa.table({"s": pa.array(enc(ids_b)), "w": rng.random(n)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["s"], monkeypatch)
    assert c.get("join.radix.hashed_key", 0) == 1 and c.get("join.radix.var_gather", 0) == 0, c
    assert c.get("join.radix.narrow_fallback", 0) == 0 and c.get("join.radix.hash_collision_fallback", 0) == 0, c
    assert c["join.radix.rows_out"] == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "left", "outer"])
@pytest.mark.parametrize("retain", [True, False])
def test_radix_join_memory_bounded_chunks(gpu_ctx, ctx, monkeypatch, how, retain):
    """Bounded memory: with a device budget (config memory_budget_mb) below the join's working set
    + output, the radix join runs in key-hash chunks into one output sink (join.radix.memory_chunks)
    and gives the CPU twin's result.  retain = false: one chunk-major pass per side (the input is
    released after it) makes every chunk a contiguous slice (join.radix.chunk_pass); a wide side
    moves in column groups whose input buffers are released group by group."""
    rng = np.random.default_rng(59)
    n = 3_000_000
    a = pa.table({"k": rng.integers(0, 2_000_000, n), "v": rng.random(n),
                  "u": pa.array(rng.integers(-9, 9, n), mask=rng.random(n) < 0.1),
                  "x": rng.random(n), "y": rng.integers(-7, 7, n).astype(np.int32)})
    b = pa.table({"k": rng.integers(0, 2_000_000, n), "w": rng.random(n), "i": rng.integers(-5, 5, n)})
    gpu_ctx.add_config("memory_budget_mb", "260")
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", "1024")
    kw = dict(left_on=["k"], right_on=["k"], left_prefix="l_", right_prefix="r_")
    try:
        L, R = Table(a, gpu_ctx), Table(b, gpu_ctx)
        L.retain_memory(retain)
        R.retain_memory(retain)
        C.trace_enable(True)
        C.trace_reset()
        got = L.join(R, how, "hash", **kw).to_pandas()
        c = dict(C.trace_counters())
        C.trace_enable(False)
    finally:
        gpu_ctx.add_config("memory_budget_mb", "")
    exp = Table(a, ctx).join(Table(b, ctx), how, "hash", **kw).to_pandas()
    assert c.get("join.radix.memory_chunks", 0) >= 2, c
    assert c.get("join.radix.chunk_pass", 0) == (0 if retain else 2), c
    # retain = false: the left side's 5 moving buffers go in two column groups (stable passes)
    assert c.get("join.radix.chunk_pass_groups", 0) == (0 if retain else 2), c
    assert (L.row_count, R.row_count) == ((n, n) if retain else (0, 0))
    assert len(got) == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how,first_pass,skew", [("inner", True, False), ("left", True, False), ("outer", True, False),
                                                  ("inner", False, False), ("left", False, False), ("outer", False, False),
                                                  ("inner", True, True), ("outer", True, True)])
def test_radix_join_memory_bounded_first_pass_chunks(gpu_ctx, ctx, monkeypatch, how, first_pass, skew):
    """Bounded memory, retain = false, non-nullable int64-key tables: the chunks are ranges of the join's
    own first radix pass (join.radix.first_pass_chunks; per chunk only the second pass + the LDS join,
    into one sink) -- or, with CYLON_RJ_FIRST_PASS_CHUNKS=0, the chunk-major pass.  Both equal the CPU
    twin; a wide side moves in stable column groups."""
    rng = np.random.default_rng(61)
    n = 3_000_000
    ka = rng.integers(0, 2_000_000, n)
    kb = rng.integers(0, 2_000_000, n)
    if skew:  # one hot key: its partition outgrows its slot in the second pass (widened, then split items)
        ka[rng.random(n) < 0.002] = 777  # ~6000 rows against a ~1000-row slot
        kb[:20] = 777
    a = pa.table({"k": ka, "v": rng.random(n), "x": rng.random(n),
                  "y": rng.integers(-7, 7, n).astype(np.int32), "z": rng.random(n)})
    b = pa.table({"k": kb, "w": rng.random(n), "i": rng.integers(-5, 5, n)})
    gpu_ctx.add_config("memory_budget_mb", "260")
    monkeypatch.setenv("CYLON_RADIX_JOIN_MIN_ROWS", "1024")
    monkeypatch.setenv("CYLON_RJ_FIRST_PASS_CHUNKS", "1" if first_pass else "0")
    monkeypatch.setenv("CYLON_RJ_EXTRA_BITS", "2")  # 12 partition bits: two levels at 3M rows
    kw = dict(left_on=["k"], right_on=["k"], left_prefix="l_", right_prefix="r_")
    try:
        L, R = Table(a, gpu_ctx), Table(b, gpu_ctx)
        L.retain_memory(False)
        R.retain_memory(False)
        C.trace_enable(True)
        C.trace_reset()
        got = L.join(R, how, "hash", **kw).to_pandas()
        c = dict(C.trace_counters())
        C.trace_enable(False)
    finally:
        gpu_ctx.add_config("memory_budget_mb", "")
    exp = Table(a, ctx).join(Table(b, ctx), how, "hash", **kw).to_pandas()
    assert c.get("join.radix.memory_chunks", 0) >= 2, c
    assert (c.get("join.radix.first_pass_chunks", 0) >= 2) == first_pass, c
    assert c.get("join.radix.chunk_pass", 0) == (0 if first_pass else 2), c
    if skew and first_pass:
        assert c.get("join.radix.slot_overflow", 0) >= 1, c
    assert (L.row_count, R.row_count) == (0, 0)
    assert len(got) == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "outer"])
def test_radix_join_memory_bounded_chunks_string_key(gpu_ctx, ctx, monkeypatch, how):
    """Bounded memory with a 16-byte string key: the key-hash chunks split the proxies (word key +
    word 1 + payload) and each chunk joins into the sink without narrowing the word key."""
    rng = np.random.default_rng(67)
    n = 2_000_000
    ids_a, ids_b = rng.integers(0, 1_500_000, n), rng.integers(0, 1_500_000, n)
    a = pa.table({"s": pa.array([f"k{x:015d}" for x in ids_a]), "v": rng.random(n)})
    b = pa.table({"s": pa.array([f"k{x:015d}" for x in ids_b]), "w": rng.random(n)})
    gpu_ctx.add_config("memory_budget_mb", "150")
    try:
        got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["s"], monkeypatch)
    finally:
        gpu_ctx.add_config("memory_budget_mb", "")
    assert c.get("join.radix.memory_chunks", 0) >= 2, c
    assert c.get("join.radix.narrow_fallback", 0) == 0, c
    assert len(got) == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


def _var_strings(rng, ids, lo, hi, binary=False):
    """Keys of random length in [lo, hi] that are a function of the id (equal ids <=> equal keys):
    the id's digits, then filler bytes up to a length drawn from the id."""
    out = []
    for x in ids:
        ln = lo + (int(x) * 2654435761 % (hi - lo + 1))
        s = (f"{x:d}#" + "abcdefghijklmnopqrstuvwxyz0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ" * 2)[:max(ln, 0)]
        if ln < len(f"{x:d}#"):  # too short for the id: a prefix would alias ids -- keep the id whole
            s = f"{x:d}"
        out.append(s.encode() if binary else s)
    return out


@pytest.mark.parametrize("how", ["inner", "left", "outer"])
@pytest.mark.parametrize("kind", ["string_8_32", "binary_1_40", "string_0_64"])
def test_radix_join_variable_length_keys(gpu_ctx, ctx, monkeypatch, how, kind):
    """Variable-length string / binary keys (rows <= 64 bytes) travel as zero-padded words + a length
    column under the padded word key (no row-number gather of the key bytes): empty strings, one-word
    keys, unaligned tails, 5-8 words.  Output key bytes must round-trip exactly; against the CPU twin."""
    rng = np.random.default_rng(71)
    n = 1_000_000
    lo, hi = {"string_8_32": (8, 32), "binary_1_40": (1, 40), "string_0_64": (0, 64)}[kind]
    ids_a, ids_b = rng.integers(0, 700_000, n), rng.integers(0, 700_000, n)
    bin_ = kind.startswith("binary")
    a = pa.table({"s": pa.array(_var_strings(rng, ids_a, lo, hi, bin_)), "v": rng.random(n)})
    b = pa.table({"s": pa.array(_var_strings(rng, ids_b, lo, hi, bin_)), "w": rng.random(n)})
    if kind == "string_0_64":  # a few empty keys on both sides (they match each other)
        a = a.set_column(0, "s", pa.array([("" if i % 9973 == 0 else s) for i, s in enumerate(a["s"].to_pylist())]))
        b = b.set_column(0, "s", pa.array([("" if i % 7919 == 0 else s) for i, s in enumerate(b["s"].to_pylist())]))
    if bin_:  # zero bytes inside keys (a trailing one too): the length column must travel
        fix = (lambda x: x[:2] + b"\x00" + x[2:] if x[:1] in (b"1", b"2") else (x + b"\x00" if x[:1] == b"3" else x))
        a = a.set_column(0, "s", pa.array([fix(x) for x in a["s"].to_pylist()]))
        b = b.set_column(0, "s", pa.array([fix(x) for x in b["s"].to_pylist()]))
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["s"], monkeypatch)
    # text keys (no zero byte): the padding encodes the length (text mode); binary keys carry it
    mode = "join.radix.var_word_key" if bin_ else "join.radix.var_word_key_text"
    assert c.get(mode, 0) == 1 and c.get("join.radix.var_gather", 0) == 0, c
    assert c.get("join.radix.hash_collision_fallback", 0) == 0, c
    assert c.get("join.radix.shared_key_column", 0) == (2 if how == "inner" else 0), c
    assert c["join.radix.rows_out"] == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "outer"])
@pytest.mark.parametrize("case", ["no_words_knob", "longer_than_64"])
def test_radix_join_variable_length_keys_gather_path(gpu_ctx, ctx, monkeypatch, how, case):
    """The hashed-key path of variable-length keys: the 64-bit row hash is partitioned and matched,
    the key bytes are gathered by row number after the join (var_gather) and every output row's keys
    are compared byte-wise (rows_equal).  Taken for keys longer than 64 bytes, or with
    CYLON_RJ_VAR_WORDS=0.  Against the CPU twin."""
    rng = np.random.default_rng(73)
    n = 600_000
    ids_a, ids_b = rng.integers(0, 400_000, n), rng.integers(0, 400_000, n)
    lo, hi = (4, 30) if case == "no_words_knob" else (50, 90)
    if case == "no_words_knob":
        monkeypatch.setenv("CYLON_RJ_VAR_WORDS", "0")
    a = pa.table({"s": pa.array(_var_strings(rng, ids_a, lo, hi)), "v": rng.random(n)})
    b = pa.table({"s": pa.array(_var_strings(rng, ids_b, lo, hi)), "w": rng.random(n)})
    got, exp, c = _join(gpu_ctx, ctx, a, b, how, ["s"], monkeypatch)
    assert c.get("join.radix.var_word_key", 0) == 0 and c.get("join.radix.var_word_key_text", 0) == 0, c
    assert c.get("join.radix.var_gather", 0) == 1, c
    assert c.get("join.radix.hashed_key", 0) == 1 and c.get("join.radix.hash_collision_fallback", 0) == 0, c
    assert c["join.radix.rows_out"] == len(exp)
    pd.testing.assert_frame_equal(_canon(got), _canon(exp), check_dtype=False)


@pytest.mark.parametrize("how", ["inner", "left"])
def test_radix_join_retain_false_releases_inputs(gpu_ctx, monkeypatch, how):
    """retain = false (reference table.cpp:150-154): each input's buffers are released as soon as
    its partition passes fit (the other side's passes and the output then reuse the memory), so the
    join's peak allocation drops by about the inputs' size; the inputs are empty afterwards and the
    result equals the retained join's."""
    n = 20_000_000

    def run(retain):
        g = torch.Generator(device="cuda").manual_seed(3)
        sides = []
        for _ in range(2):
            cols = {"k": torch.randint(0, int(0.99 * n), (n,), generator=g, device="cuda")}
            for i in range(3):
                cols[f"v{i}"] = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
            t = Table.from_torch(gpu_ctx, cols)
            del cols
            t.retain_memory(retain)
            sides.append(t)
        L, R = sides
        del sides
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        C.trace_enable(True)
        C.trace_reset()
        out = L.join(R, how, "hash", on=["k"], left_prefix="l_", right_prefix="r_")
        torch.cuda.synchronize()
        c = dict(C.trace_counters())
        C.trace_enable(False)
        peak = torch.cuda.max_memory_allocated() - base
        t = out.to_torch()
        sums = {name: float(x.double().sum()) for name, x in t.items() if not name.startswith("r_v")}
        sums["rows"] = out.row_count
        return sums, peak, c, (L.row_count, R.row_count)

    kept, peak_kept, c_kept, rows_kept = run(True)
    rel, peak_rel, c_rel, rows_rel = run(False)
    assert c_kept.get("join.radix.released_inputs", 0) == 0 and rows_kept == (n, n)
    assert c_rel.get("join.radix.released_inputs", 0) == 2 and rows_rel == (0, 0), c_rel
    # (row order inside a radix-joined table is not fixed: float sums compare to rounding)
    assert rel.keys() == kept.keys() and all(rel[x] == pytest.approx(kept[x], rel=1e-12) for x in kept), (rel, kept)
    input_bytes = 2 * n * 32
    assert peak_kept - peak_rel >= 0.5 * input_bytes, (peak_kept, peak_rel)
