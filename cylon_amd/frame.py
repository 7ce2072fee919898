"""pandas-like DataFrame / CylonEnv frontend (reference: python/pycylon/frame.py:31-1808).

Every DataFrame method runs locally when `env` is None and as the distributed
operator (shuffle over RCCL + device kernel) when an env is given, like the
reference.  `to_device` / `to_cpu`, stubs in the reference (frame.py:82-97),
really move the columns between host memory and the MI355X here.
"""
from typing import Dict, Hashable, List, Optional, Sequence, Union

import numpy as np
import pandas as pd
import pyarrow as pa
import torch

from ._lib import C
from .ctx.context import CylonContext
from .data.table import Table, default_context
from .net import CommConfig

DEVICE_CPU = "cpu"


class CylonEnv(object):
    """Owns a (distributed) context and finalizes it on deletion (reference frame.py:34-65)."""

    def __init__(self, config=None, distributed=True, device: Optional[str] = None) -> None:
        self._context = CylonContext(config=config if config is not None else (CommConfig() if distributed else None),
                                     distributed=distributed, device=device)
        self._distributed = distributed
        self._finalized = False

    @property
    def context(self) -> CylonContext:
        return self._context

    @property
    def rank(self) -> int:
        return self._context.get_rank()

    @property
    def world_size(self) -> int:
        return self._context.get_world_size()

    @property
    def is_distributed(self) -> bool:
        return self._distributed

    def finalize(self):
        if not self._finalized:
            self._finalized = True
            self._context.finalize()

    def barrier(self):
        self._context.barrier()

    def __del__(self):
        try:
            self.finalize()
        except Exception:
            pass


def _to_table(data, columns, ctx) -> Table:
    if isinstance(data, Table):
        return data
    if isinstance(data, pa.Table):
        return Table(data, ctx)
    if isinstance(data, pd.DataFrame):
        return Table.from_pandas(ctx, data)
    if isinstance(data, dict):
        return Table(pa.Table.from_pydict({str(k): v for k, v in data.items()}), ctx)
    if isinstance(data, np.ndarray):
        arr = data if data.ndim == 2 else data.reshape(-1, 1)
        names = columns or [str(i) for i in range(arr.shape[1])]
        return Table(pa.Table.from_arrays([pa.array(arr[:, i]) for i in range(arr.shape[1])], names=names), ctx)
    if isinstance(data, (list, tuple)):
        if data and isinstance(data[0], (list, tuple, np.ndarray)):
            names = columns or [str(i) for i in range(len(data))]
            return Table(pa.Table.from_arrays([pa.array(c) for c in data], names=names), ctx)
        names = columns or ["0"]
        return Table(pa.Table.from_arrays([pa.array(data)], names=names), ctx)
    if data is None:
        return Table(pa.table({}), ctx)
    raise ValueError(f"Invalid data structure, {type(data)}")


class DataFrame(object):
    def __init__(self, data=None, index=None, columns=None, copy=False, context: CylonContext = None):
        ctx = context or (data.context if isinstance(data, Table) else default_context())
        self._table = _to_table(data, columns, ctx)
        if columns is not None and not isinstance(data, (np.ndarray, list, tuple)) and \
                len(columns) == self._table.column_count:
            self._table.rename(list(columns))
        if index is not None:
            self._table.set_index(index)
        self._index_columns: List[str] = []

    # ------------------------------------------------------------- devices
    def to_cpu(self) -> "DataFrame":
        return DataFrame(self._table.to_device("cpu"))

    def to_device(self, device=None) -> "DataFrame":
        dev = device or ("cuda:0" if torch.cuda.is_available() else "cpu")
        return DataFrame(self._table.to_device(dev))

    def is_cpu(self) -> bool:
        return self._table.device == DEVICE_CPU

    def is_device(self, device) -> bool:
        return self._table.device == str(device)

    @property
    def device(self) -> str:
        return self._table.device

    def _change_context(self, env: CylonEnv) -> "DataFrame":
        ctx = env.context
        if self._table.context is not ctx:
            t = self._table
            if t.device != ctx.device:
                t = t.to_device(ctx.device)
            self._table = Table(context=ctx, _native=C.Table(ctx._ctx, list(t.native.columns())))
        return self

    # ------------------------------------------------------------ properties
    @property
    def shape(self):
        return self._table.shape

    @property
    def columns(self) -> List[str]:
        return self._table.column_names

    @property
    def index(self):
        return self._table.index

    def __len__(self):
        return self._table.row_count

    def to_pandas(self) -> pd.DataFrame:
        return self._table.to_pandas()

    def to_numpy(self, order: str = "F", zero_copy_only: bool = True, writable: bool = False) -> np.ndarray:
        return self._table.to_numpy(order, zero_copy_only, writable)

    def to_arrow(self) -> pa.Table:
        return self._table.to_arrow()

    def to_dict(self) -> Dict:
        return self._table.to_pydict()

    def to_table(self) -> Table:
        return self._table

    def to_torch(self) -> Dict[str, torch.Tensor]:
        return self._table.to_torch()

    def to_csv(self, path, csv_write_options=None):
        self._table.to_csv(path, csv_write_options)

    # ------------------------------------------------------------ indexing
    def __getitem__(self, item) -> "DataFrame":
        if isinstance(item, DataFrame):
            item = item._table
        return DataFrame(self._table[item])

    def __setitem__(self, key, value):
        if isinstance(value, DataFrame):
            value = value._table
        self._table[key] = value

    @property
    def loc(self):
        return _FrameIndexer(self._table.loc)

    @property
    def iloc(self):
        return _FrameIndexer(self._table.iloc)

    def __repr__(self):
        return self._table.to_string(row_limit=10)

    # ------------------------------------------------------------ operators
    def _bin(self, other, fn):
        o = other._table if isinstance(other, DataFrame) else other
        return DataFrame(fn(self._table, o))

    def __eq__(self, other):
        return self._bin(other, lambda a, b: a == b)

    def __ne__(self, other):
        return self._bin(other, lambda a, b: a != b)

    def __lt__(self, other):
        return self._bin(other, lambda a, b: a < b)

    def __gt__(self, other):
        return self._bin(other, lambda a, b: a > b)

    def __le__(self, other):
        return self._bin(other, lambda a, b: a <= b)

    def __ge__(self, other):
        return self._bin(other, lambda a, b: a >= b)

    def __or__(self, other):
        return self._bin(other, lambda a, b: a | b)

    def __and__(self, other):
        return self._bin(other, lambda a, b: a & b)

    def __invert__(self):
        return DataFrame(~self._table)

    def __neg__(self):
        return DataFrame(-self._table)

    def __add__(self, other):
        return self._bin(other, lambda a, b: a + b)

    def __sub__(self, other):
        return self._bin(other, lambda a, b: a - b)

    def __mul__(self, other):
        return self._bin(other, lambda a, b: a * b)

    def __truediv__(self, other):
        return self._bin(other, lambda a, b: a / b)

    __hash__ = object.__hash__

    # ------------------------------------------------------------ transforms
    def drop(self, column_names: List[str]) -> "DataFrame":
        return DataFrame(self._table.drop(column_names))

    def fillna(self, fill_value) -> "DataFrame":
        return DataFrame(self._table.fillna(fill_value))

    def where(self, condition: "DataFrame" = None, other=None) -> "DataFrame":
        if condition is None:
            raise ValueError("Condition must be provided")
        return DataFrame(self._table.where(condition._table, other._table if isinstance(other, DataFrame) else other))

    def isnull(self) -> "DataFrame":
        return DataFrame(self._table.isnull())

    isna = isnull

    def notnull(self) -> "DataFrame":
        return DataFrame(self._table.notnull())

    notna = notnull

    def rename(self, column_names) -> "DataFrame":
        self._table.rename(column_names)
        return self

    def add_prefix(self, prefix: str) -> "DataFrame":
        return DataFrame(self._table.add_prefix(prefix))

    def add_suffix(self, suffix: str) -> "DataFrame":
        return DataFrame(self._table.add_suffix(suffix))

    def dropna(self, axis=0, how="any") -> "DataFrame":
        return DataFrame(self._table.dropna(axis=axis, how=how))

    def isin(self, values) -> "DataFrame":
        return DataFrame(self._table.isin(values))

    def applymap(self, func) -> "DataFrame":
        return DataFrame(self._table.applymap(func))

    def astype(self, dtype, safe=True) -> "DataFrame":
        return DataFrame(self._table.astype(dtype, safe))

    def set_index(self, keys, drop: bool = True, append: bool = False, inplace: bool = False,
                  verify_integrity: bool = False):
        from .indexing.index import IndexingSchema
        keys_l = keys if isinstance(keys, list) else [keys]
        target = self if inplace else DataFrame(self._table.project(list(range(self._table.column_count))))
        key0 = keys_l[0]
        if isinstance(key0, str) and key0 in target.columns:
            target._table.set_index(key0, IndexingSchema.LINEAR, drop=drop)
            target._index_columns = [key0]
        else:
            target._table.set_index(keys_l, IndexingSchema.LINEAR)
        return None if inplace else target

    def reset_index(self, level=None, drop: bool = False, inplace: bool = False, col_level=0, col_fill=""):
        target = self if inplace else DataFrame(self._table.project(list(range(self._table.column_count))))
        names = list(self._index_columns)
        target._table._index = self._table.index
        had_index = "index" in target.columns
        target._table.reset_index(drop_index=drop)
        if not drop and not had_index and len(names) == 1 and isinstance(names[0], str) and \
                names[0] not in target.columns and "index" in target.columns:
            target._table.rename({"index": names[0]})  # pandas names the column after the index
        target._index_columns = []
        return None if inplace else target

    def _with_index_columns(self) -> "DataFrame":
        """This frame with its index columns present as ordinary columns (set_index(drop=True)
        moved them into the index)."""
        if all(isinstance(c, str) and c in self.columns for c in self._index_columns):
            return self
        out = self.reset_index()
        out._index_columns = list(self._index_columns)
        return out

    # ------------------------------------------------------------ relational
    def join(self, other: "DataFrame", on=None, how="left", lsuffix="l", rsuffix="r", sort=False,
             algorithm="sort", env: CylonEnv = None) -> "DataFrame":
        """Join on a key column of the caller against the other frame's index columns (reference frame.py:1115)."""
        left_on = on if on is not None else self._index_columns
        right_on = other._index_columns
        if not left_on or not right_on:
            return self._join_on_index(other, how, algorithm, env)
        left_on = left_on if isinstance(left_on, list) else [left_on]
        left = self._with_index_columns() if on is None else self
        return left._do_join(other._with_index_columns(), how, algorithm, left_on, right_on, lsuffix, rsuffix, env,
                             sort)

    def _join_on_index(self, other, how, algorithm, env):
        tables = [self._change_context(env)._table if env else self._table,
                  other._change_context(env)._table if env else other._table]
        return DataFrame(Table.concat(tables, axis=1, join=how, algorithm=algorithm, distributed=env is not None))

    def _do_join(self, other, how, algorithm, left_on, right_on, lp, rp, env, sort=False):
        if env is None:
            t = self._table.join(other._table, how, algorithm, left_on=left_on, right_on=right_on, left_prefix=lp,
                                 right_prefix=rp)
        else:
            self._change_context(env)
            other._change_context(env)
            t = self._table.distributed_join(other._table, how, algorithm, left_on=left_on, right_on=right_on,
                                             left_prefix=lp, right_prefix=rp)
        out = DataFrame(t)
        if sort:
            out = out.sort_values(by=[lp + left_on[0] if isinstance(left_on[0], str) else 0])
        return out

    def merge(self, right: "DataFrame", how="inner", algorithm="sort", on=None, left_on=None, right_on=None,
              left_index=False, right_index=False, sort=False, suffixes=("_x", "_y"), copy=True, indicator=False,
              validate=None, env: CylonEnv = None) -> "DataFrame":
        if on is not None:
            left_on = right_on = on
        if left_index:
            left_on = self._index_columns
        if right_index:
            right_on = right._index_columns
        if left_on is None or right_on is None:
            raise ValueError("merge needs join keys: pass on=, left_on=/right_on=, or left_index/right_index "
                             "on frames that have index columns set")
        left_on = left_on if isinstance(left_on, list) else [left_on]
        right_on = right_on if isinstance(right_on, list) else [right_on]
        return self._do_join(right, how, algorithm, left_on, right_on, suffixes[0], suffixes[1], env, sort)

    @staticmethod
    def concat(objs: List["DataFrame"], axis=0, join="outer", ignore_index: bool = False, keys=None, levels=None,
               names=None, verify_integrity: bool = False, sort: bool = False, copy: bool = True,
               env: CylonEnv = None) -> "DataFrame":
        """axis=0: set union of the frames (reference semantics, frame.py:1610-1634); axis=1: join on index."""
        if len(objs) == 0:
            raise ValueError("objs can't be empty")
        if axis == 0:
            cur = objs[0]._change_context(env)._table if env else objs[0]._table
            for o in objs[1:]:
                t = o._change_context(env)._table if env else o._table
                cur = cur.distributed_union(t) if env else cur.union(t)
            return DataFrame(cur)
        tables = [o._change_context(env)._table if env else o._table for o in objs]
        return DataFrame(Table.concat(tables, axis=1, join="inner" if join == "inner" else "outer",
                                      distributed=env is not None))

    def drop_duplicates(self, subset: Optional[Union[Hashable, Sequence[Hashable]]] = None,
                        keep: Union[str, bool] = "first", inplace: bool = False, ignore_index: bool = False,
                        env: CylonEnv = None) -> "DataFrame":
        cols = [subset] if isinstance(subset, (str, int)) else subset
        if env is None:
            return DataFrame(self._table.unique(columns=cols, keep=keep))
        return DataFrame(self._change_context(env)._table.distributed_unique(columns=cols, keep=keep))

    def sort_values(self, by, axis=0, ascending=True, inplace=False, kind="quicksort", na_position="last",
                    ignore_index=False, key=None, env: CylonEnv = None) -> "DataFrame":
        if env is None:
            return DataFrame(self._table.sort(order_by=by, ascending=ascending))
        return DataFrame(self._change_context(env)._table.distributed_sort(order_by=by, ascending=ascending))

    def groupby(self, by, agg: dict, algorithm: str = "hash", env: CylonEnv = None) -> "DataFrame":
        if env is None:
            return DataFrame(self._table.local_groupby(by, agg, algorithm))
        return DataFrame(self._change_context(env)._table.groupby(by, agg, algorithm))

    def shuffle(self, on, env: CylonEnv) -> "DataFrame":
        return DataFrame(self._change_context(env)._table.shuffle(on))


class _FrameIndexer:
    def __init__(self, indexer):
        self._ix = indexer

    def __getitem__(self, key):
        return DataFrame(self._ix[key])


__all__ = ["CylonEnv", "DataFrame", "DEVICE_CPU"]
