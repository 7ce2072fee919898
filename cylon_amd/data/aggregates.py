"""Aggregation op enum and helpers (reference: python/pycylon/data/aggregates.pyx:17-40,
cpp/src/cylon/compute/aggregate_kernels.hpp:40-50).

COUNT counts the non-null values of the aggregated column (pandas ``count``), in
``groupby`` and in the scalar ``Table.count`` alike.  The reference's scalar Count
is the same (Arrow COUNT_NON_NULL); its group-by COUNT counts rows, nulls included.
Results are identical on columns without nulls."""
from .._lib import C

AggregationOp = C.AggregationOp

AggregationOpString = {
    "sum": AggregationOp.SUM,
    "cnt": AggregationOp.COUNT,
    "count": AggregationOp.COUNT,
    "min": AggregationOp.MIN,
    "max": AggregationOp.MAX,
    "var": AggregationOp.VAR,
    "nunique": AggregationOp.NUNIQUE,
    "mean": AggregationOp.MEAN,
    "quantile": AggregationOp.QUANTILE,
    "median": AggregationOp.QUANTILE,
    "std": AggregationOp.STDDEV,
}


def resolve_op(op):
    if isinstance(op, AggregationOp):
        return op
    if isinstance(op, int):
        return AggregationOp(op)
    try:
        return AggregationOpString[str(op).lower()]
    except KeyError:
        raise ValueError(f"unknown aggregation op '{op}'") from None


def parse_agg(table, agg: dict):
    """{col: op | [ops]} -> parallel lists (cols, op ids, quantiles, ddofs)."""
    cols, ops, qs, ddofs = [], [], [], []
    for col, spec in agg.items():
        ci = table._resolve_column(col)
        specs = spec if isinstance(spec, (list, tuple)) else [spec]
        for s in specs:
            q, ddof = 0.5, 1
            if isinstance(s, tuple):  # ('quantile', 0.9) or ('var', 0)
                s, arg = s
                if str(s).lower() == "quantile":
                    q = float(arg)
                else:
                    ddof = int(arg)
            cols.append(ci)
            ops.append(int(resolve_op(s)))
            qs.append(q)
            ddofs.append(ddof)
    return cols, ops, qs, ddofs
