"""pandas-style Table operators (reference: python/pycylon/data/table.pyx:1025-2411).

Mask/elementwise operators run on the table's device (data/compute.py);
row-selection results go through the native filter (K11) and gather (K4).
"""
import operator
from typing import Callable, Dict, List, Optional, Union

import numpy as np
import pyarrow as pa
import torch

from .._lib import C
from ..indexing.index import (BaseIndex, ILocIndexer, IndexingSchema, LocIndexer, RangeIndex, build_index)
from . import compute


class PandasOpsMixin:
    # ------------------------------------------------------------------ index
    @property
    def index(self) -> BaseIndex:
        idx = getattr(self, "_index", None)
        if idx is None or len(idx) != self.row_count:
            idx = RangeIndex.of_length(self.row_count, self.device)
            self._index = idx
        return idx

    def get_index(self) -> BaseIndex:
        return self.index

    @property
    def indexing_schema(self):
        return self.index.get_schema()

    @indexing_schema.setter
    def indexing_schema(self, schema):
        self._index = build_index(self.index.get_index_array(), schema, self.device)

    def set_index(self, key, indexing_schema: IndexingSchema = IndexingSchema.LINEAR, drop: bool = False):
        """key: column name/position (its values become the index), a list/array of values, or an index."""
        if isinstance(key, BaseIndex):
            self._index = key
            return self
        if isinstance(key, (str, int, np.integer)) and not isinstance(key, bool):
            ci = self._resolve_column(key)
            values = self.to_arrow().column(ci)
            if drop:
                keep = [i for i in range(self.column_count) if i != ci]
                self._t = C.project(self._t, keep)
            self._index = build_index(values, indexing_schema, self.device)
            return self
        self._index = build_index(pa.array(list(key)), indexing_schema, self.device)
        return self

    def reset_index(self, drop_index: bool = False):
        idx = self.index
        if not drop_index and not isinstance(idx, RangeIndex):
            at = self.to_arrow()
            at = at.add_column(0, "index", idx.get_index_array())
            self._t = type(self)(at, self.context)._t
        self._index = RangeIndex.of_length(self.row_count, self.device)
        return self

    @property
    def loc(self) -> LocIndexer:
        return LocIndexer(self)

    @property
    def iloc(self) -> ILocIndexer:
        return ILocIndexer(self)

    # ----------------------------------------------------------- item access
    def __getitem__(self, key):
        from .table import Table
        if isinstance(key, slice):
            start = 0 if key.start is None else key.start
            stop = self.row_count if key.stop is None else min(key.stop, self.row_count)
            out = self.slice(start, max(0, stop - start))
            out._index = self.index.take(torch.arange(start, max(start, stop)))
            return out
        if isinstance(key, (int, np.integer)) and not isinstance(key, bool):
            out = self.slice(int(key), 1)
            out._index = self.index.take(torch.tensor([int(key)]))
            return out
        if isinstance(key, str):
            out = self.project([key])
            out._index = self.index
            return out
        if isinstance(key, (list, tuple)):
            out = self.project(list(key))
            out._index = self.index
            return out
        if isinstance(key, Table):
            if key.column_count == 1:
                return self.filter_mask(compute.col_values(key.native.column(0)).to(torch.uint8) &
                                        (compute.col_valid(key.native.column(0)).to(torch.uint8)
                                         if key.native.column(0).validity is not None else 1))
            return compute.where(self, key)
        raise ValueError(f"Unsupported Key Type in __getitem__ {type(key)}")

    def __setitem__(self, key, value):
        from .table import Table
        if not isinstance(key, str):
            raise ValueError(f"__setitem__ key must be a column name, got {type(key)}")
        if isinstance(value, Table):
            if value.column_count != 1:
                raise ValueError("Given table has more than 1 columns")
            col = value.native.column(0).with_name(key)
            if col.length != self.row_count:
                raise ValueError("column length differs from table rows")
        elif np.isscalar(value):
            col = compute.make_col(key, torch.full((self.row_count,), value, device=self.device)) \
                if not isinstance(value, str) else \
                type(self)(pa.table({key: pa.array([value] * self.row_count)}), self.context).native.column(0)
        elif torch.is_tensor(value):
            col = compute.make_col(key, value.to(self.device))
        else:
            arr = pa.array(value)
            col = type(self)(pa.table({key: arr}), self.context).native.column(0)
        cols = list(self._t.columns())
        names = [c.name for c in cols]
        if key in names:
            cols[names.index(key)] = col
        else:
            cols.append(col)
        idx = self.index
        self._t = C.Table(self._t.context(), cols)
        self._index = idx

    # -------------------------------------------------------------- operators
    def _engine(self):
        return self.context.get_config("compute_engine", "device") or "device"

    def __eq__(self, other):
        return compute.binary_op(self, other, operator.eq, self._engine())

    def __ne__(self, other):
        return compute.binary_op(self, other, operator.ne, self._engine())

    def __lt__(self, other):
        return compute.binary_op(self, other, operator.lt, self._engine())

    def __gt__(self, other):
        return compute.binary_op(self, other, operator.gt, self._engine())

    def __le__(self, other):
        return compute.binary_op(self, other, operator.le, self._engine())

    def __ge__(self, other):
        return compute.binary_op(self, other, operator.ge, self._engine())

    def __or__(self, other):
        return compute.binary_op(self, other, operator.or_, self._engine())

    def __and__(self, other):
        return compute.binary_op(self, other, operator.and_, self._engine())

    def __invert__(self):
        return compute.unary_op(self, lambda v: ~v, "invert", self._engine())

    def __neg__(self):
        return compute.unary_op(self, lambda v: -v, "neg", self._engine())

    def __add__(self, other):
        return compute.binary_op(self, other, operator.add, self._engine())

    def __sub__(self, other):
        return compute.binary_op(self, other, operator.sub, self._engine())

    def __mul__(self, other):
        return compute.binary_op(self, other, operator.mul, self._engine())

    def __truediv__(self, other):
        return compute.binary_op(self, other, operator.truediv, self._engine())

    __hash__ = object.__hash__

    # ---------------------------------------------------------- transforms
    def drop(self, column_names: List[str], inplace=False):
        drop = set(self._resolve_columns(column_names))
        keep = [i for i in range(self.column_count) if i not in drop]
        out = self.project(keep)
        if inplace:
            self._t = out._t
            return None
        out._index = self.index
        return out

    def fillna(self, fill_value):
        return compute.fill_null(self, fill_value)

    def where(self, condition, other=None):
        return compute.where(self, condition, other)

    def isnull(self):
        return compute.is_null(self)

    def isna(self):
        return compute.is_null(self)

    def notnull(self):
        return compute.is_null(self, invert=True)

    def notna(self):
        return compute.is_null(self, invert=True)

    def rename(self, column_names: Union[List[str], Dict[str, str]]):
        cols = list(self._t.columns())
        if isinstance(column_names, dict):
            cols = [c.with_name(column_names.get(c.name, c.name)) for c in cols]
        else:
            if len(column_names) != len(cols):
                raise ValueError("number of names must match the number of columns")
            cols = [c.with_name(n) for c, n in zip(cols, column_names)]
        self._t = C.Table(self._t.context(), cols)
        return self

    def add_prefix(self, prefix: str):
        out = self._wrap(C.Table(self._t.context(), [c.with_name(prefix + c.name) for c in self._t.columns()]))
        out._index = self.index
        return out

    def add_suffix(self, suffix: str):
        out = self._wrap(C.Table(self._t.context(), [c.with_name(c.name + suffix) for c in self._t.columns()]))
        out._index = self.index
        return out

    def dropna(self, axis=0, how="any", inplace=False):
        nulls = compute.is_null(self)
        masks = [compute.col_values(c) for c in nulls.native.columns()]
        if axis == 0:
            if not masks:
                return self
            stacked = torch.stack(masks)
            bad = stacked.any(0) if how == "any" else stacked.all(0)
            out = self.filter_mask((~bad).to(torch.uint8))
        else:
            keep = [i for i, m in enumerate(masks) if not (m.any() if how == "any" else m.all())]
            out = self.project(keep)
        if inplace:
            self._t = out._t
            return None
        return out

    def isin(self, value, skip_null=True):
        return compute.is_in(self, value, skip_null)

    def applymap(self, func: Callable):
        return compute.apply_map(self, func)

    def astype(self, dtype, safe=True):
        return compute.cast(self, dtype, safe)

    def iterrows(self):
        at = self.to_arrow()
        idx = self.index.index_values
        for i, row in enumerate(at.to_pylist()):
            yield idx[i], list(row.values())

    def filter(self, statement):
        """Row filter by a boolean Table / mask tensor / per-row predicate (reference: Select)."""
        from .table import Table
        if isinstance(statement, Table):
            return self[statement]
        if callable(statement):
            return self.select(statement)
        return self.filter_mask(statement)

    def select(self, predicate: Callable):
        """Reference cylon::Select: keep rows for which predicate(row_dict) is true (host evaluation)."""
        rows = self.to_arrow().to_pylist()
        mask = torch.tensor([bool(predicate(r)) for r in rows], dtype=torch.uint8)
        return self.filter_mask(mask)

    @staticmethod
    def concat(tables: List, axis: int = 0, join: str = "inner", algorithm: str = "sort", distributed=False):
        """axis=0: vertical merge; axis=1: join on the row index (reference table.pyx:2334-2400)."""
        from .table import Table
        if not tables:
            raise ValueError("concat needs at least one table")
        if axis == 0:
            return Table.merge(tables)
        res = tables[0]
        for i, t in enumerate(tables[1:]):
            left = res.copy_with_index_column("__idx_l")
            right = t.copy_with_index_column("__idx_r")
            fn = left.distributed_join if distributed else left.join
            j = fn(right, join, algorithm, left_on=["__idx_l"], right_on=["__idx_r"])
            idxcol = j.to_arrow().column("__idx_l")
            res = j.drop(["__idx_l", "__idx_r"])
            res._index = build_index(idxcol, IndexingSchema.LINEAR, res.device)
        return res

    def copy_with_index_column(self, name: str):
        arr = self.index.get_index_array()
        out = self._wrap(self._t)
        t = type(self)(pa.table({name: arr}), self.context)
        out._t = C.Table(self._t.context(), [t.native.column(0)] + list(self._t.columns()))
        return out

    def equals(self, other, ordered: bool = True) -> bool:
        a, b = self.to_arrow(), other.to_arrow()
        if not ordered:
            a = a.sort_by([(n, "ascending") for n in a.column_names])
            b = b.sort_by([(n, "ascending") for n in b.column_names])
        return a.equals(b)
