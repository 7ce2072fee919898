"""Regression tests for round-2 review findings: sort order of DECIMAL and
FIXED_SIZE_LIST columns (numeric, not byte order), LIST sort keys refused,
decimal precision/scale round trip, Arrow-compatible safe int -> float casts."""
from decimal import Decimal

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pytest

from cylon_amd import Table


def _decimal_values():
    vals = [Decimal("1.00"), Decimal("2.56"), Decimal("-1.00"), Decimal("-300.25"), Decimal("0.00"),
            Decimal("99999999999999.99"), Decimal("-99999999999999.99"), Decimal("2.55"), None, Decimal("1.01")]
    return vals


@pytest.mark.parametrize("asc", [True, False])
def test_sort_by_decimal_is_numeric(ctx, asc):
    vals = _decimal_values()
    at = pa.table({"d": pa.array(vals, pa.decimal128(18, 2)), "i": np.arange(len(vals))})
    out = Table(at, ctx).sort("d", ascending=asc).to_arrow()
    assert out.schema.field("d").type == pa.decimal128(18, 2)  # precision / scale survive
    got = out.column("d").to_pylist()
    nn = sorted([v for v in vals if v is not None], reverse=not asc)
    assert got == nn + [None]


def test_sort_by_decimal256(ctx):
    vals = [Decimal(x) for x in ("5", "-7", "123456789012345678901234567890", "-2", "0")]
    at = pa.table({"d": pa.array(vals, pa.decimal256(40, 0))})
    got = Table(at, ctx).sort("d").to_arrow().column("d").to_pylist()
    assert got == sorted(vals)


def test_sort_by_fixed_size_list_is_elementwise(ctx):
    rows = [[1, 300], [1, -2], [-5, 7], [256, 0], [1, 1], [0, 0]]
    at = pa.table({"l": pa.array(rows, pa.list_(pa.int32(), 2)), "i": np.arange(len(rows))})
    got = Table(at, ctx).sort("l").to_arrow().column("l").to_pylist()
    assert got == sorted(rows)
    got = Table(at, ctx).sort("l", ascending=False).to_arrow().column("l").to_pylist()
    assert got == sorted(rows, reverse=True)


def test_sort_by_list_column_refused(ctx):
    at = pa.table({"l": pa.array([[1, 2], [3]], pa.list_(pa.int64())), "i": [0, 1]})
    with pytest.raises(Exception, match="list"):
        Table(at, ctx).sort("l")


def test_decimal_roundtrip_keeps_scale(ctx):
    at = pa.table({"d": pa.array([Decimal("1.25"), None, Decimal("-3.50")], pa.decimal128(7, 2))})
    assert Table(at, ctx).to_arrow().equals(at)


@pytest.mark.parametrize("target", ["float64", "float32"])
def test_safe_int_to_float_cast_matches_arrow(ctx, target):
    big = 2 ** 53 + 1 if target == "float64" else 2 ** 24 + 1
    at = pa.table({"x": pa.array([1, big, -3], pa.int64())})
    with pytest.raises(pa.ArrowInvalid):
        pc.cast(at.column("x"), getattr(pa, target)(), safe=True)
    with pytest.raises(pa.ArrowInvalid):
        Table(at, ctx).astype(target)
    ok = Table(at, ctx).astype(target, safe=False).to_arrow().column("x")
    assert ok.equals(pc.cast(at.column("x"), getattr(pa, target)(), safe=False))
    small = pa.table({"x": pa.array([1, -(2 ** 20), 7], pa.int64())})
    assert Table(small, ctx).astype(target).to_arrow().column("x").equals(
        pc.cast(small.column("x"), getattr(pa, target)()))


def test_uint64_casts_follow_arrow(ctx):
    at = pa.table({"x": pa.array([1, 2 ** 63 + 5, 3], pa.uint64())})
    for target in (pa.int64(), pa.float64()):
        try:
            exp = pc.cast(at.column("x"), target, safe=True)
        except pa.ArrowInvalid:
            with pytest.raises(pa.ArrowInvalid):
                Table(at, ctx).astype(str(target) if target != pa.float64() else "float64")
            continue
        got = Table(at, ctx).astype(str(target)).to_arrow().column("x")
        assert got.equals(exp)
