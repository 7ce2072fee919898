"""pycylon-compatible Table (reference: python/pycylon/data/table.pyx:75-2531).

A Table is a handle on a native, device-resident table (cylon_amd._C.Table):
columns live in HBM on the context's MI355X (or in host memory for CPU
contexts) and every relational operator runs in the native engine.
"""
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import pyarrow as pa
import torch

from .._lib import C
from ..ctx.context import CylonContext
from . import arrow_bridge as ab
from .table_pandas import PandasOpsMixin

_JOIN_TYPES = {"inner": "inner", "left": "left", "right": "right", "outer": "outer", "full_outer": "outer",
               "fullouter": "outer"}


def _ensure_ctx(ctx: Optional[CylonContext]) -> CylonContext:
    if ctx is None:
        return default_context()
    return ctx


_DEFAULT_CTX = None


def default_context() -> CylonContext:
    global _DEFAULT_CTX
    if _DEFAULT_CTX is None:
        _DEFAULT_CTX = CylonContext(config=None, distributed=False)
    return _DEFAULT_CTX


class SortOptions:
    """reference: python/pycylon/data/table.pyx:2512 / cylon/table.hpp:388-393"""

    def __init__(self, num_bins: int = 0, num_samples: int = 0):
        self.num_bins = int(num_bins)
        self.num_samples = int(num_samples)


class Table(PandasOpsMixin):
    def __init__(self, pyarrow_table=None, context: Optional[CylonContext] = None, _native=None):
        self._ctx = _ensure_ctx(context)
        if _native is not None:
            self._t = _native
        elif pyarrow_table is not None:
            self._t = ab.table_from_arrow(self._ctx._ctx, pyarrow_table, self._ctx.device)
        else:
            self._t = C.Table(self._ctx._ctx, [])
        self._index = None

    # ------------------------------------------------------------------ wrapping
    def _wrap(self, native) -> "Table":
        return Table(context=self._ctx, _native=native)

    @property
    def native(self):
        return self._t

    @property
    def context(self) -> CylonContext:
        return self._ctx

    # ------------------------------------------------------------ constructors
    @staticmethod
    def from_arrow(context: CylonContext, pyarrow_table: pa.Table) -> "Table":
        return Table(pyarrow_table, context)

    @staticmethod
    def from_pandas(context: CylonContext = None, df=None, preserve_index=False, nthreads=None, columns=None,
                    safe=False) -> "Table":
        if df is None and context is not None and not isinstance(context, CylonContext):
            context, df = None, context
        at = pa.Table.from_pandas(df, preserve_index=preserve_index, nthreads=nthreads, columns=columns, safe=safe)
        return Table(at, context)

    @staticmethod
    def from_pydict(context: CylonContext, dictionary: dict) -> "Table":
        return Table(pa.Table.from_pydict(dictionary), context)

    @staticmethod
    def from_list(context: CylonContext, col_names: List[str], data_list: List) -> "Table":
        return Table(pa.Table.from_arrays([pa.array(d) for d in data_list], names=col_names), context)

    @staticmethod
    def from_numpy(context: CylonContext, col_names: List[str], ar_list: List[np.ndarray]) -> "Table":
        return Table(pa.Table.from_arrays([pa.array(a) for a in ar_list], names=col_names), context)

    @staticmethod
    def from_torch(context: CylonContext, columns: Dict[str, torch.Tensor]) -> "Table":
        """Zero-copy from device tensors (DLPack-free: the tensors become the column buffers)."""
        ctx = _ensure_ctx(context)
        cols = [ab.column_from_tensor(k, v.to(ctx.device)) for k, v in columns.items()]
        return Table(context=ctx, _native=C.Table(ctx._ctx, cols))

    # ------------------------------------------------------------- conversions
    def to_arrow(self) -> pa.Table:
        return ab.table_to_arrow(self._t)

    def to_pandas(self):
        return self.to_arrow().to_pandas()

    def to_pydict(self, with_index=False):
        return self.to_arrow().to_pydict()

    def to_numpy(self, order: str = "F", zero_copy_only: bool = True, writable: bool = False):
        cols = [c.to_numpy(zero_copy_only=False) for c in self.to_arrow().columns]
        return np.array(cols).T.copy(order=order) if cols else np.empty((0, 0))

    # ---- Arrow PyCapsule interfaces ---------------------------------------------
    def __arrow_c_stream__(self, requested_schema=None):
        """Host Arrow C stream (pyarrow / polars / duckdb consumers)."""
        return self.to_arrow().__arrow_c_stream__(requested_schema)

    def __arrow_c_device_array__(self, requested_schema=None, **kwargs):
        """Arrow C Device Data Interface: a struct array whose buffers stay where the table
        lives (ARROW_DEVICE_ROCM in HBM, zero-copy for values / offsets / list children;
        bitmaps and packed booleans produced on the device; sync_event = a hipEvent_t)."""
        if requested_schema is not None:
            raise NotImplementedError("schema requests are not supported")
        return C.export_device_table(self._t)

    @staticmethod
    def from_arrow_device(context: CylonContext, obj) -> "Table":
        """Zero-copy import of an object exposing __arrow_c_device_array__ (or the capsule pair)."""
        ctx = _ensure_ctx(context)
        caps = obj.__arrow_c_device_array__() if hasattr(obj, "__arrow_c_device_array__") else obj
        return Table(context=ctx, _native=C.import_device_table(ctx._ctx, caps[0], caps[1]))

    def to_torch(self) -> Dict[str, torch.Tensor]:
        """Columns as device tensors (zero-copy, fixed width columns only).  Columns of one table
        may share a buffer natively (an inner join's two key columns hold the same values,
        docs/semantics.md); the second and later names of a shared buffer come back as copies, so an
        in-place write through one returned tensor never changes another."""
        out, seen = {}, set()
        for c in self._t.columns():
            if c.offsets is not None:
                raise TypeError(f"column {c.name} is variable width")
            d = c.data
            key = (d.device, d.untyped_storage().data_ptr()) if d.numel() else None
            if key is not None and key in seen:
                d = d.clone()
            elif key is not None:
                seen.add(key)
            out[c.name] = d
        return out

    def to_csv(self, path, csv_write_options=None):
        from ..io import write_csv
        write_csv(self, path, csv_write_options)

    def to_device(self, device: str) -> "Table":
        return self._wrap(self._t.to(device))

    def to_cpu(self) -> "Table":
        return self.to_device("cpu")

    # -------------------------------------------------------------- properties
    @property
    def column_names(self) -> List[str]:
        return self._t.column_names()

    @property
    def column_count(self) -> int:
        return self._t.num_columns()

    @property
    def row_count(self) -> int:
        return self._t.rows()

    @property
    def shape(self):
        return (self.row_count, self.column_count)

    @property
    def device(self) -> str:
        return self._t.device()

    def retain_memory(self, retain: bool):
        self._t.retain_memory(retain)

    def is_retain(self) -> bool:
        return self._t.is_retain()

    def clear(self):
        self._t.clear()

    def __len__(self):
        return self.row_count

    # ---------------------------------------------------------- column helpers
    def _resolve_column(self, c) -> int:
        if isinstance(c, (int, np.integer)):
            if not 0 <= int(c) < self.column_count:
                raise IndexError(f"column index {c} out of range")
            return int(c)
        idx = self._t.column_index(str(c))
        if idx < 0:
            raise KeyError(f"column '{c}' not found in {self.column_names}")
        return idx

    def _resolve_columns(self, cols) -> List[int]:
        if cols is None:
            return list(range(self.column_count))
        if isinstance(cols, (int, str, np.integer)):
            cols = [cols]
        return [self._resolve_column(c) for c in cols]

    def _resolve_join_columns(self, table: "Table", kwargs):
        left_on, right_on, on = kwargs.get("left_on"), kwargs.get("right_on"), kwargs.get("on")
        if left_on is not None and right_on is not None:
            lc, rc = self._resolve_columns(left_on), table._resolve_columns(right_on)
        elif on is not None:
            lc, rc = self._resolve_columns(on), table._resolve_columns(on)
        else:
            raise TypeError("kwargs 'on' or 'left_on' and 'right_on' must be provided")
        if not lc or len(lc) != len(rc):
            raise ValueError("Provided Column Names or Column Indices not valid.")
        return lc, rc

    # --------------------------------------------------------------- relational
    def join(self, table: "Table", join_type: str = "inner", algorithm: str = "sort", **kwargs) -> "Table":
        lc, rc = self._resolve_join_columns(table, kwargs)
        jt = _JOIN_TYPES[join_type.lower()]
        return self._wrap(C.join(self._t, table._t, jt, algorithm.lower(), lc, rc, kwargs.get("left_prefix", ""),
                                 kwargs.get("right_prefix", "")))

    def distributed_join(self, table: "Table", join_type: str = "inner", algorithm: str = "sort",
                         **kwargs) -> "Table":
        lc, rc = self._resolve_join_columns(table, kwargs)
        jt = _JOIN_TYPES[join_type.lower()]
        return self._wrap(C.distributed_join(self._t, table._t, jt, algorithm.lower(), lc, rc,
                                             kwargs.get("left_prefix", ""), kwargs.get("right_prefix", "")))

    # set operations (distinct semantics over all columns; reference table.pyx:383-430)
    def union(self, table: "Table") -> "Table":
        return self._wrap(C.union(self._t, table._t))

    def distributed_union(self, table: "Table") -> "Table":
        return self._wrap(C.distributed_union(self._t, table._t))

    def subtract(self, table: "Table") -> "Table":
        return self._wrap(C.subtract(self._t, table._t))

    def distributed_subtract(self, table: "Table") -> "Table":
        return self._wrap(C.distributed_subtract(self._t, table._t))

    def intersect(self, table: "Table") -> "Table":
        return self._wrap(C.intersect(self._t, table._t))

    def distributed_intersect(self, table: "Table") -> "Table":
        return self._wrap(C.distributed_intersect(self._t, table._t))

    def unique(self, columns: List = None, keep: str = "first", inplace=False) -> Optional["Table"]:
        out = self._wrap(C.unique(self._t, self._resolve_columns(columns), keep == "first"))
        if inplace:
            self._t = out._t
            return None
        return out

    def distributed_unique(self, columns: List = None, keep: str = "first", inplace=False):
        out = self._wrap(C.distributed_unique(self._t, self._resolve_columns(columns), keep == "first"))
        if inplace:
            self._t = out._t
            return None
        return out

    # aggregates (global across ranks, reference table.pyx:548-586)
    def _agg_op(self, column, op, quantile=0.5, ddof=1) -> "Table":
        from .aggregates import resolve_op
        return self._wrap(C.aggregate(self._t, self._resolve_column(column), int(resolve_op(op)), quantile, ddof,
                                      True))

    def sum(self, column):
        return self._agg_op(column, "sum")

    def count(self, column):
        return self._agg_op(column, "count")

    def min(self, column):
        return self._agg_op(column, "min")

    def max(self, column):
        return self._agg_op(column, "max")

    def mean(self, column):
        return self._agg_op(column, "mean")

    def var(self, column, ddof=1):
        return self._agg_op(column, "var", ddof=ddof)

    def std(self, column, ddof=1):
        return self._agg_op(column, "std", ddof=ddof)

    def nunique(self, column):
        return self._agg_op(column, "nunique")

    def quantile(self, column, q=0.5):
        return self._agg_op(column, "quantile", quantile=q)

    def groupby(self, index, agg: dict, algorithm: str = "hash") -> "Table":
        """Distributed group-by (reference table.pyx:587-647 -> DistributedHashGroupBy).

        agg: {column: op | [ops]} with ops as names ('sum','cnt'/'count','min','max','mean','var','std',
        'nunique','quantile'/'median') or AggregationOp values.
        """
        from .aggregates import parse_agg
        if not agg or not isinstance(agg, dict):
            raise ValueError("agg should be non-empty and dict type")
        keys = self._resolve_columns(index)
        cols, ops, qs, ddofs = parse_agg(self, agg)
        fn = C.distributed_hash_groupby if algorithm == "hash" else C.distributed_pipeline_groupby
        return self._wrap(fn(self._t, keys, cols, ops, qs, ddofs))

    def local_groupby(self, index, agg: dict, algorithm: str = "hash") -> "Table":
        from .aggregates import parse_agg
        keys = self._resolve_columns(index)
        cols, ops, qs, ddofs = parse_agg(self, agg)
        fn = C.hash_groupby if algorithm == "hash" else C.pipeline_groupby
        return self._wrap(fn(self._t, keys, cols, ops, qs, ddofs))

    def distributed_sort(self, order_by=None, ascending: Union[bool, List[bool]] = True,
                         sort_options: SortOptions = None) -> "Table":
        cols = self._resolve_columns(order_by if order_by is not None else 0)
        asc = [bool(a) for a in ascending] if isinstance(ascending, (list, tuple)) else [bool(ascending)] * len(cols)
        so = sort_options or SortOptions()
        return self._wrap(C.distributed_sort(self._t, cols, asc, so.num_bins, so.num_samples))

    def project(self, columns: List) -> "Table":
        return self._wrap(C.project(self._t, self._resolve_columns(columns)))

    @staticmethod
    def merge(tables: List["Table"], ctx: CylonContext = None) -> "Table":
        if not tables:
            raise ValueError("merge needs at least one table")
        return tables[0]._wrap(C.merge([t._t for t in tables]))

    def sort(self, order_by=None, ascending: Union[bool, List[bool]] = True) -> "Table":
        cols = self._resolve_columns(order_by if order_by is not None else 0)
        asc = [bool(a) for a in ascending] if isinstance(ascending, (list, tuple)) else [bool(ascending)]
        return self._wrap(C.sort(self._t, cols, asc))

    def shuffle(self, hash_columns: List = None) -> "Table":
        return self._wrap(C.shuffle(self._t, self._resolve_columns(hash_columns)))

    def hash_partition(self, hash_columns: List, num_partitions: int) -> List["Table"]:
        return [self._wrap(t) for t in C.hash_partition(self._t, self._resolve_columns(hash_columns),
                                                         int(num_partitions))]

    def take(self, indices) -> "Table":
        idx = torch.as_tensor(indices, dtype=torch.int64)
        return self._wrap(C.gather(self._t, idx.to(self.device)))

    def filter_mask(self, mask) -> "Table":
        m = torch.as_tensor(mask)
        if m.dtype != torch.uint8:
            m = m.to(torch.uint8)
        return self._wrap(C.filter_by_mask(self._t, m.to(self.device)))

    def slice(self, offset: int, length: int) -> "Table":
        return self._wrap(C.slice(self._t, int(offset), int(length)))

    # ------------------------------------------------------------------ display
    def to_string(self, row_limit: int = 10):
        return self.to_arrow().slice(0, row_limit).to_pandas().to_string()

    def __repr__(self):
        return self.to_string()

    def show(self, row1=-1, row2=-1, col1=-1, col2=-1):
        at = self.to_arrow()
        if row1 >= 0 and row2 >= 0:
            at = at.slice(row1, row2 - row1)
        if col1 >= 0 and col2 >= 0:
            at = at.select(list(range(col1, col2)))
        print(at.to_pandas().to_string())
