"""Elementwise compute on device columns (K15; reference: python/pycylon/data/compute.pyx:43-813).

The reference evaluates these operators in Python/Cython over pyarrow.compute or
numpy on the host.  Here fixed-width columns stay on the table's device and the
operators run as device tensor expressions (ROCm kernels on MI355X), with the
validity byte-mask propagated explicitly.  Variable-width (string) columns are
evaluated by Arrow compute on the host, as in the reference.

Engine selection keeps the reference's `compute_engine` config key: "arrow"
forces the host Arrow path, anything else uses the device path.
"""
import operator
from typing import Any, Callable, List, Optional

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import torch

from .._lib import C
from . import arrow_bridge as ab

T = C.Type

_CMP = {operator.eq: "equal", operator.ne: "not_equal", operator.lt: "less", operator.gt: "greater",
        operator.le: "less_equal", operator.ge: "greater_equal"}
_ARITH = {operator.add: "add", operator.sub: "subtract", operator.mul: "multiply", operator.truediv: "divide"}


def is_var(col) -> bool:
    return col.offsets is not None


def col_values(col) -> torch.Tensor:
    """Typed value tensor of a fixed-width column (bool as torch.bool)."""
    t = col.data
    if col.type.type == T.BOOL:
        return t.to(torch.bool)
    return t


def col_valid(col) -> Optional[torch.Tensor]:
    v = col.validity
    return None if v is None else v.to(torch.bool)


def make_col(name: str, values: torch.Tensor, valid: Optional[torch.Tensor] = None, like=None):
    vt = None if valid is None else valid.to(torch.uint8).contiguous()
    if (like is not None and not is_var(like) and like.type.type != T.BOOL and values.dtype != torch.bool
            and ab.torch_dtype(like.type) == values.dtype):
        data = values.contiguous()
        return C.Column(name, like.type, data.numel(), data, None, vt)
    return ab.column_from_tensor(name, values, vt)


def _and_valid(a, b):
    if a is None:
        return b
    if b is None:
        return a
    return a & b


def _arrow_col(col) -> pa.Array:
    return ab.column_to_arrow(col)


def _from_arrow(name, arr, device):
    return ab.column_from_arrow(name, arr, device)


def _scalar_for(col, value):
    if isinstance(value, (bool, int, float, np.number)):
        return value
    raise TypeError(f"unsupported scalar {value!r} for column {col.name}")


def binary_op(table, other, op: Callable, engine: str = "device"):
    """Elementwise op between a table and a scalar or an equally shaped table."""
    from .table import Table
    cols = table.native.columns()
    dev = table.device
    other_cols = other.native.columns() if isinstance(other, Table) else None
    if other_cols is not None and len(other_cols) != len(cols):
        raise ValueError("tables must have the same number of columns")
    out = []
    for i, c in enumerate(cols):
        oc = other_cols[i] if other_cols is not None else None
        use_arrow = engine == "arrow" or is_var(c) or (oc is not None and is_var(oc)) or isinstance(other, str)
        if use_arrow:
            fn = _CMP.get(op) or _ARITH.get(op) or {operator.and_: "and_kleene", operator.or_: "or_kleene"}.get(op)
            rhs = _arrow_col(oc) if oc is not None else other
            res = getattr(pc, fn)(_arrow_col(c), rhs)
            out.append(_from_arrow(c.name, res, dev))
            continue
        a = col_values(c)
        va = col_valid(c)
        if oc is not None:
            b = col_values(oc)
            vb = col_valid(oc)
        else:
            b = _scalar_for(c, other)
            vb = None
        if op is operator.truediv:
            res = a.to(torch.float64) / (b.to(torch.float64) if torch.is_tensor(b) else float(b))
        else:
            res = op(a, b)
        out.append(make_col(c.name, res, _and_valid(va, vb), like=c if res.dtype == a.dtype else None))
    return table._wrap(C.Table(table.native.context(), out))


def unary_op(table, fn: Callable, name: str = "", engine: str = "device"):
    cols = table.native.columns()
    out = []
    for c in cols:
        if is_var(c) or engine == "arrow":
            res = getattr(pc, {"neg": "negate", "invert": "invert"}[name])(_arrow_col(c))
            out.append(_from_arrow(c.name, res, table.device))
            continue
        v = col_values(c)
        out.append(make_col(c.name, fn(v), col_valid(c), like=c))
    return table._wrap(C.Table(table.native.context(), out))


def is_null(table, invert: bool = False):
    out = []
    for c in table.native.columns():
        n = c.length
        v = col_valid(c)
        isn = torch.zeros(n, dtype=torch.bool, device=c.data.device) if v is None else ~v
        if not is_var(c) and c.type.type in (T.FLOAT, T.DOUBLE, T.HALF_FLOAT):
            isn = isn | torch.isnan(c.data)
        out.append(make_col(c.name, ~isn if invert else isn))
    return table._wrap(C.Table(table.native.context(), out))


def _var_scalar(c, value, device):
    """One-row device column of c's type holding value (None if value does not convert)."""
    try:
        arr = pa.array([value], type=ab.to_arrow_type(c.type))
    except (pa.ArrowInvalid, pa.ArrowTypeError, TypeError, ValueError):
        return None
    return ab.column_from_arrow(c.name, arr, device)


def _select_var(c, other, cond, device):
    """K15 device select of a string / binary column (kernels/select.hip): cond ? c : other, where
    other is None (null), a scalar (broadcast) or a column of c's type; None when other does not
    fit (the caller then uses Arrow's host kernels)."""
    if other is None:
        b = None
    elif isinstance(other, C.Column):
        if not is_var(other) or other.type.type != c.type.type or other.length not in (1, c.length):
            return None
        b = other
    else:
        b = _var_scalar(c, other, device)
        if b is None:
            return None
    return C.select_var(c, b, cond.to(torch.uint8))


def fill_null(table, value):
    out = []
    for c in table.native.columns():
        if c.validity is None and (is_var(c) or c.type.type not in (T.FLOAT, T.DOUBLE)):
            out.append(c)
            continue
        if is_var(c):
            res = _select_var(c, value, c.validity, table.device) if value is not None else c
            out.append(res if res is not None else _from_arrow(c.name, pc.fill_null(_arrow_col(c), value),
                                                               table.device))
            continue
        v = col_values(c)
        mask = col_valid(c)
        fill = torch.full_like(v, value)
        isn = (~mask if mask is not None else torch.zeros_like(v, dtype=torch.bool))
        if v.is_floating_point():
            isn = isn | torch.isnan(v)
        out.append(make_col(c.name, torch.where(isn, fill, v), None, like=c))
    return table._wrap(C.Table(table.native.context(), out))


def where(table, condition, other=None):
    """Keep values where condition (bool table, same shape, or one column) holds, else other/null."""
    from .table import Table
    ccols = condition.native.columns()
    out = []
    for i, c in enumerate(table.native.columns()):
        cond = ccols[i] if len(ccols) > 1 else ccols[0]
        cv = col_values(cond)
        cvv = col_valid(cond)
        if cvv is not None:
            cv = cv & cvv
        if is_var(c):
            rhs = other.native.column(i) if isinstance(other, Table) else other
            res = _select_var(c, rhs, cv, table.device)
            if res is None:  # other of another type: Arrow's host if_else (casts / raises like pandas)
                rhs = other.to_arrow().column(i) if isinstance(other, Table) else other
                res = _from_arrow(c.name, pc.if_else(pa.array(cv.cpu().numpy()), _arrow_col(c), rhs), table.device)
            out.append(res)
            continue
        v = col_values(c)
        valid = col_valid(c)
        if other is None:
            nv = cv if valid is None else (valid & cv)
            out.append(make_col(c.name, v, nv, like=c))
        else:
            ov = col_values(other.native.column(i)) if isinstance(other, Table) else torch.full_like(v, other)
            out.append(make_col(c.name, torch.where(cv, v, ov), valid, like=c))
    return table._wrap(C.Table(table.native.context(), out))


def is_in(table, values, skip_null: bool = True):
    """Membership test per column; values: list/set (all columns), dict (per column name) or Table."""
    from .table import Table
    out = []
    for i, c in enumerate(table.native.columns()):
        if isinstance(values, dict):
            vals = values.get(c.name, [])
        elif isinstance(values, Table):
            vals = values.to_arrow().column(i).to_pylist()
        else:
            vals = list(values)
        if is_var(c):
            vals = [v for v in vals if isinstance(v, (str, bytes))]
        else:
            vals = [v for v in vals if not isinstance(v, (str, bytes))]
        if is_var(c):  # device hash join of the column against the distinct value set
            n = c.length
            res = torch.zeros(n, dtype=torch.bool, device=c.data.device)
            if vals and n:
                vs = pa.array(vals, type=ab.to_arrow_type(c.type)).unique()
                vt = C.Table(table.native.context(), [ab.column_from_arrow("v", vs, table.device)])
                lt = C.Table(table.native.context(), [c])
                li, _ = C.join_indices(lt, vt, "inner", "hash", [0], [0])
                res[li.to(res.device)] = True
            valid = col_valid(c)
            if valid is not None:
                res = res & valid
            out.append(make_col(c.name, res))
            continue
        v = col_values(c)
        vs = torch.tensor([x for x in vals if x is not None], dtype=v.dtype, device=v.device) if vals else \
            torch.empty(0, dtype=v.dtype, device=v.device)
        res = torch.isin(v, vs)
        valid = col_valid(c)
        if valid is not None:
            res = res & valid
        out.append(make_col(c.name, res))
    return table._wrap(C.Table(table.native.context(), out))


def _device_cast(c, target: pa.DataType, safe: bool):
    """Numeric -> numeric casts on the column's device (torch), with Arrow's safe-cast checks:
    float -> int must be integral and in range, int -> narrower int must be in range, int -> float
    must lie within the float's exact integer range (2^53 / 2^24).  uint64 sources go to Arrow."""
    src = ab.to_arrow_type(c.type)
    num = lambda t: pa.types.is_integer(t) or pa.types.is_floating(t)  # noqa: E731
    try:
        # K15 string <-> number casts on the device (kernels/strcast.hip); None: the host parser
        if is_var(c):
            # uint64 targets: the device parser reads int64, Arrow's host cast takes the full range
            if pa.types.is_string(src) and num(target) and target not in (pa.float16(), pa.uint64()):
                return C.cast_string_to_number(c, ab.to_cylon_type(target))
            return None
        if pa.types.is_string(target) and pa.types.is_integer(src) and src != pa.uint64() and c.type.type != T.BOOL:
            return C.cast_integer_to_string(c, ab.to_cylon_type(target))
    except C.CylonError as e:
        raise pa.ArrowInvalid(str(e)) from None
    if c.type.type == T.BOOL:
        return None
    if not (num(src) and num(target)) or target == pa.float16() or src == pa.float16():
        return None
    if src == pa.uint64():  # torch has no full uint64 min/max/compare support: Arrow's host kernels
        return None
    ct = ab.to_cylon_type(target)
    tdt = ab.torch_dtype(ct)
    v = c.data
    valid = col_valid(c)
    if safe and pa.types.is_integer(target):
        live = v if valid is None else v[valid]
        if live.numel():
            info = np.iinfo(target.to_pandas_dtype())
            if pa.types.is_floating(src):
                if not bool(torch.all(torch.isfinite(live)) and torch.all(live == torch.trunc(live))):
                    raise pa.ArrowInvalid(f"column {c.name}: float values would be truncated")
                lo, hi = float(live.min()), float(live.max())
            else:
                lo, hi = int(live.min()), int(live.max())
            if lo < info.min or hi > info.max:
                raise pa.ArrowInvalid(f"column {c.name}: integer value out of range for {target}")
    if safe and pa.types.is_floating(target) and pa.types.is_integer(src):
        # Arrow's safe int -> float cast refuses integers beyond the float's exact range
        live = v if valid is None else v[valid]
        lim = 2 ** 53 if target == pa.float64() else 2 ** 24
        if live.numel() and (int(live.min()) < -lim or int(live.max()) > lim):
            raise pa.ArrowInvalid(f"column {c.name}: integer value not in range: {-lim} to {lim}")
    out = v.to(tdt)
    return C.Column(c.name, ct, c.length, out.contiguous(), None,
                    None if c.validity is None else c.validity.contiguous())


def cast(table, dtype, safe: bool = True):
    """astype: dtype may be a single type or {column: type}.  Numeric -> numeric, string -> number
    and integer -> string casts run on the table's device; everything else (float -> string,
    dates, hex / special-value strings) goes through Arrow's cast kernels on the host."""
    from ..types import to_arrow
    cols = table.native.columns()
    targets = [dtype.get(c.name) if isinstance(dtype, dict) else dtype for c in cols]
    dev = [None if t is None else _device_cast(c, to_arrow(t), safe) for c, t in zip(cols, targets)]
    if all(t is None or d is not None for t, d in zip(targets, dev)):
        out = [c if d is None else d for c, d in zip(cols, dev)]
        return table._wrap(C.Table(table.native.context(), out))
    at = table.to_arrow()
    arrays, names = [], []
    for name, col in zip(at.column_names, at.columns):
        t = dtype.get(name) if isinstance(dtype, dict) else dtype
        arrays.append(col if t is None else pc.cast(col, to_arrow(t), safe=safe))
        names.append(name)
    from .table import Table
    return Table(pa.Table.from_arrays(arrays, names=names), table.context)


def apply_map(table, func: Callable):
    at = table.to_arrow()
    arrays = [pa.array([func(x) for x in col.to_pylist()]) for col in at.columns]
    from .table import Table
    return Table(pa.Table.from_arrays(arrays, names=at.column_names), table.context)


def unique_values(table, column=0) -> List[Any]:
    return table.to_arrow().column(column).unique().to_pylist()


def nunique(table, column=0) -> int:
    return len(unique_values(table, column))


# ---------------------------------------------------------------------------
# Reference entry points (python/pycylon/data/compute.pyx), mapped onto the
# device engine above.  Same names and argument order as pycylon.
# ---------------------------------------------------------------------------
def comparison_compute_op_iter(array, other, op):
    """compute.pyx:78 — elementwise comparison of a 1-D array with a scalar."""
    return np.asarray([op(x, other) for x in np.asarray(array)], dtype=bool)


def comparison_compute_np_op(array, other, op):
    """compute.pyx:108 — vectorised comparison of a numpy array with a scalar."""
    return op(np.asarray(array), other)


def table_compare_ar_op(table, other, op):
    """compute.pyx:127 — comparison through the Arrow (host) engine."""
    return binary_op(table, other, op, engine="arrow")


def table_compare_np_op(table, other, op):
    """compute.pyx:164 — the reference's numpy engine; here the device engine."""
    return binary_op(table, other, op, engine="device")


def table_compare_op(table, other, op, engine="arrow"):
    """compute.pyx:198."""
    return binary_op(table, other, op, engine=engine)


def invert(table):
    """compute.pyx:226 — logical not of bool columns (other types raise, as in the reference)."""
    for c in table.native.columns():
        if c.type.type != T.BOOL:
            raise ValueError(f"Invert only support for bool types, but found {c.type}")
    return unary_op(table, torch.logical_not, "invert")


def neg(table):
    """compute.pyx:246 — negation of numeric columns."""
    return unary_op(table, torch.neg, "neg")


def division_op(table, op, value):
    """compute.pyx:267 — table / scalar (op: operator.truediv or operator.floordiv)."""
    return binary_op(table, value, op)


def math_op(table, op, value, engine="device"):
    """compute.pyx:441 — table (+ - * /) scalar or table."""
    return binary_op(table, value, op, engine="arrow" if engine == "arrow" else "device")


def math_op_numpy(table, op, value):
    """compute.pyx:299."""
    return math_op(table, op, value, "numpy")


def math_op_arrow(table, op, value):
    """compute.pyx:347."""
    return math_op(table, op, value, "arrow")


def math_op_c_numpy(table, op, value):
    """compute.pyx:373."""
    return math_op(table, op, value, "numpy")


def unique(table):
    """compute.pyx:454 — per column, the number of distinct values (a one-row table)."""
    from .table import Table
    return Table.from_pydict(table.context, {name: [nunique(table, i)] for i, name in enumerate(table.column_names)})


def compare_array_like_values(l_org_ar, l_cmp_ar, skip_null=True):
    """compute.pyx:509 — membership of each value of l_org_ar in l_cmp_ar (pyarrow arrays)."""
    return pc.is_in(l_org_ar, options=pc.SetLookupOptions(value_set=pa.array(l_cmp_ar), skip_nulls=skip_null))


def drop_na(table, how: str, axis=0):
    """compute.pyx:714."""
    return table.dropna(axis=axis, how=how)


def infer_map(table, func):
    """compute.pyx:792 — func applied to every column as a numpy array; one output column each."""
    from .table import Table
    arrays = [pa.array(np.asarray(func(col.to_numpy(zero_copy_only=False))))
              for col in table.to_arrow().combine_chunks().itercolumns()]
    return Table.from_arrow(table.context, pa.Table.from_arrays(arrays, names=table.column_names))
