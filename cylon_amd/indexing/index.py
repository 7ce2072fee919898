"""Table indexing (reference: cpp/src/cylon/indexing/index.hpp:22-700,
indexer.hpp:76-260, python/pycylon/indexing/index.pyx, python/pycylon/index.py).

Index values live on the table's device as a tensor (numeric) or as an Arrow
array (strings).  Hash, BinaryTree and BTree indexes build their native structure
once (cylon/indexing/index.hpp: sorted order images, plus a device hash table for
Hash) and every lookup is a probe / binary search per label; Linear keeps the
reference's per-lookup semantics (one device join of the labels against the
column, C.index_lookup); Range indexes are arithmetic.  Range-of-values `loc` selects from the first position of the start
value to the last position of the end value, as the reference's LocIndexer does.
"""
from enum import IntEnum
from typing import Any, List, Sequence

import numpy as np
import pyarrow as pa
import torch

from .._lib import C
from ..data import arrow_bridge as ab

_CTXS = {}


def _native_ctx(device: str):
    if device not in _CTXS:
        _CTXS[device] = C.Context.init_local(device)
    return _CTXS[device]


class IndexingSchema(IntEnum):
    RANGE = 0
    LINEAR = 1
    HASH = 2
    BINARYTREE = 3
    BTREE = 4


class BaseIndex:
    schema = IndexingSchema.LINEAR

    def __init__(self, values, device: str = "cpu"):
        if isinstance(values, (pa.Array, pa.ChunkedArray)):
            arr = values.combine_chunks() if isinstance(values, pa.ChunkedArray) else values
            if (pa.types.is_integer(arr.type) or pa.types.is_floating(arr.type)) and arr.null_count == 0:
                self._values = torch.from_numpy(arr.to_numpy(zero_copy_only=False).copy()).to(device)
                self._arrow = None
            else:
                self._values = None
                self._arrow = arr
        elif torch.is_tensor(values):
            self._values = values.to(device)
            self._arrow = None
        else:
            arr = pa.array(list(values))
            self.__init__(arr, device)
            return
        self.device = device
        self._col = None

    def __len__(self):
        return len(self._values) if self._values is not None else len(self._arrow)

    # ---- reference API ----------------------------------------------------
    def get_index_array(self) -> pa.Array:
        if self._values is not None:
            return pa.array(self._values.cpu().numpy())
        return self._arrow

    def get_schema(self) -> IndexingSchema:
        return self.schema

    @property
    def index_values(self) -> List[Any]:
        return self.get_index_array().to_pylist()

    @property
    def values(self) -> np.ndarray:
        return self.get_index_array().to_numpy(zero_copy_only=False)

    def isin(self, values, skip_null: bool = True, zero_copy_only: bool = False) -> np.ndarray:
        """Per label: is it one of `values` (reference index.pyx:81, Arrow is_in semantics: a null
        label matches a null value only when skip_null is False).  Numeric labels are tested on the
        index's device (torch.isin against the exactly representable values); others via Arrow."""
        if not isinstance(values, (list, np.ndarray)):
            raise ValueError("values must be List or np.ndarray")
        vals = values.tolist() if isinstance(values, np.ndarray) else list(values)
        labels = getattr(self, "_values", None)
        if labels is None and getattr(self, "_arrow", None) is None:  # (a RangeIndex: its labels)
            labels = torch.from_numpy(self.get_index_array().to_numpy(zero_copy_only=False).copy())
        if labels is not None:
            dt = labels.dtype
            keep = []
            for v in vals:
                if v is None or isinstance(v, (str, bytes)):
                    continue
                try:
                    c = torch.tensor([v], dtype=dt)
                except (TypeError, RuntimeError, OverflowError):
                    continue
                if c.item() == v or (v != v and c.item() != c.item()):  # exactly representable (NaN too)
                    keep.append(c)
            vs = torch.cat(keep).to(labels.device) if keep else torch.empty(0, dtype=dt, device=labels.device)
            res = torch.isin(labels, vs)
            if dt.is_floating_point and any(v != v for v in vals if isinstance(v, float)):
                res |= torch.isnan(labels)
            return res.cpu().numpy()
        import pyarrow.compute as pc
        arr = self._arrow
        try:
            vset = pa.array(vals, type=arr.type)
        except (pa.ArrowInvalid, pa.ArrowTypeError, TypeError, OverflowError):
            vset = pa.array([v for v in vals if v is None or isinstance(v, (str, bytes)) == pa.types.is_string(arr.type)])
        out = pc.is_in(arr, options=pc.SetLookupOptions(value_set=vset, skip_nulls=skip_null))
        return out.to_numpy(zero_copy_only=zero_copy_only)

    def to(self, device: str) -> "BaseIndex":
        return type(self)(self._values if self._values is not None else self._arrow, device)

    def take(self, positions: torch.Tensor) -> "BaseIndex":
        if self._values is not None:
            return type(self)(self._values[positions.to(self._values.device)], self.device)
        return type(self)(self._arrow.take(pa.array(positions.cpu().numpy())), self.device)

    # ---- lookups ------------------------------------------------------------
    def _native_column(self):
        if getattr(self, "_col", None) is None:
            if self._values is not None:
                self._col = ab.column_from_tensor("i", self._values.contiguous())
            else:
                self._col = ab.column_from_arrow("i", self._arrow, self.device)
        return self._col

    def positions_of(self, value) -> torch.Tensor:
        return self.positions_of_list([value])

    def _persistent(self):
        """The native index structure (hash / sorted schemas), built once per index."""
        return None

    def positions_of_list(self, values: Sequence) -> torch.Tensor:
        values = list(values)
        if not values or len(self) == 0:
            return torch.empty(0, dtype=torch.int64)
        try:
            labels = pa.array(values, type=self.get_index_array().type)
        except (pa.ArrowInvalid, pa.ArrowTypeError, TypeError, OverflowError):
            return self._positions_slow(values)
        # a label the index type does not carry exactly (2.5 for an int index) matches nothing
        conv = labels.to_pylist()
        exact = [a == b or (a != a and b != b) for a, b in zip(conv, values)]
        if not all(exact):
            labels = pa.array([c if ok else None for c, ok in zip(conv, exact)], type=labels.type)
        col = ab.column_from_arrow("l", labels, self.device)
        nidx = self._persistent()
        if nidx is not None:
            return nidx.locations_of(col).cpu()
        return C.index_lookup(_native_ctx(self.device), self._native_column(), col).cpu()

    def _positions_slow(self, values) -> torch.Tensor:
        vals = self.index_values
        return torch.tensor([i for v in values for i, x in enumerate(vals) if x == v], dtype=torch.int64)

    def range_positions(self, start, end) -> torch.Tensor:
        s = self.positions_of(start)
        e = self.positions_of(end)
        if s.numel() == 0 or e.numel() == 0:
            raise KeyError(f"index values {start!r}..{end!r} not found")
        lo, hi = int(s.min()), int(e.max())
        return torch.arange(lo, hi + 1, dtype=torch.int64)


class LinearIndex(BaseIndex):
    schema = IndexingSchema.LINEAR


class _PersistentIndex(BaseIndex):
    """An index whose native structure (cylon/indexing/index.hpp) is built once, at
    construction (``set_index``), and reused by every lookup: Hash = sorted order images
    + an open-addressing table of the distinct values (one probe per label);
    BinaryTree / BTree = the sorted images (binary search per label).  A string / binary
    Hash index is persistent too (runs keyed by 64-bit hashes of the bytes, every candidate's
    bytes verified against its label); string BinaryTree / BTree indexes use the per-lookup
    join inside the native index."""

    def __init__(self, values, device: str = "cpu"):
        super().__init__(values, device)
        self._nidx = C.index_from_column(_native_ctx(self.device), self._native_column(),
                                         getattr(C.IndexingSchema, self.schema.name))

    def _persistent(self):
        return self._nidx

    @property
    def persistent_rows(self) -> int:
        """Rows held by the built structure (0 when the column type uses the join fallback)."""
        return self._nidx.persistent_rows()


class HashIndex(_PersistentIndex):
    schema = IndexingSchema.HASH


class BinaryTreeIndex(_PersistentIndex):
    schema = IndexingSchema.BINARYTREE


class BTreeIndex(_PersistentIndex):
    schema = IndexingSchema.BTREE


class RangeIndex(BaseIndex):
    schema = IndexingSchema.RANGE

    def __init__(self, start: int = 0, stop: int = 0, step: int = 1, device: str = "cpu"):
        self.start, self.stop, self.step = int(start), int(stop), int(step)
        self.device = device
        self._values = None
        self._arrow = None

    @classmethod
    def of_length(cls, n: int, device: str = "cpu"):
        return cls(0, n, 1, device)

    def __len__(self):
        return max(0, (self.stop - self.start + self.step - 1) // self.step)

    def get_index_array(self) -> pa.Array:
        return pa.array(np.arange(self.start, self.stop, self.step, dtype=np.int64))

    def to(self, device):
        return RangeIndex(self.start, self.stop, self.step, device)

    def take(self, positions: torch.Tensor) -> "BaseIndex":
        vals = torch.arange(self.start, self.stop, self.step, dtype=torch.int64)[positions.cpu()]
        return LinearIndex(vals, self.device)

    def positions_of_list(self, values: Sequence) -> torch.Tensor:
        parts = [self.positions_of(v) for v in values]
        return torch.cat(parts) if parts else torch.empty(0, dtype=torch.int64)

    def positions_of(self, value) -> torch.Tensor:
        v = int(value)
        if v < self.start or v >= self.stop or (v - self.start) % self.step:
            return torch.empty(0, dtype=torch.int64)
        return torch.tensor([(v - self.start) // self.step], dtype=torch.int64)


def build_index(values, schema: IndexingSchema, device: str = "cpu") -> BaseIndex:
    if schema == IndexingSchema.RANGE:
        return RangeIndex.of_length(len(values), device)
    if schema == IndexingSchema.HASH:
        return HashIndex(values, device)
    if schema == IndexingSchema.BINARYTREE:
        return BinaryTreeIndex(values, device)
    if schema == IndexingSchema.BTREE:
        return BTreeIndex(values, device)
    if schema == IndexingSchema.LINEAR:
        return LinearIndex(values, device)
    raise ValueError(f"unsupported indexing schema {schema}")


class _Indexer:
    """Row/column selector bound to a table.  Constructed with a table (``table.loc``) or,
    like the reference's ``LocIndexer(indexing_schema)``, with a schema, in which case the
    ``loc_with_*`` calls name the table explicitly."""

    def __init__(self, table=None):
        self._t = table if not isinstance(table, (IndexingSchema, int)) else None

    def _on(self, table):
        return type(self)(table) if table is not None else self

    # reference API (python/pycylon/indexing/index.pyx LocIndexer / ILocIndexer)
    def loc_with_single_column(self, indices, column_index, table=None):
        return self._on(table)[indices, column_index]

    def loc_with_multi_column(self, indices, column_list, table=None):
        return self._on(table)[indices, list(column_list)]

    def loc_with_range_column(self, indices, column_range, table=None):
        return self._on(table)[indices, column_range]

    def _cols(self, cols) -> List[int]:
        t = self._t
        if cols is None or (isinstance(cols, slice) and cols == slice(None)):
            return list(range(t.column_count))
        if isinstance(cols, slice):
            a = 0 if cols.start is None else t._resolve_column(cols.start)
            b = t.column_count - 1 if cols.stop is None else t._resolve_column(cols.stop)
            return list(range(a, b + 1))
        if isinstance(cols, (list, tuple)):
            return [t._resolve_column(c) for c in cols]
        return [t._resolve_column(cols)]

    def _select(self, rows: torch.Tensor, cols):
        t = self._t
        sub = t.project(self._cols(cols))
        out = sub.take(rows)
        out._index = t.index.take(rows)
        return out


class LocIndexer(_Indexer):
    """table.loc[rows, cols]: rows by index value / list of values / value range (inclusive)."""

    def __getitem__(self, key):
        rows, cols = (key if isinstance(key, tuple) else (key, None))
        idx = self._t.index
        if isinstance(rows, slice):
            if rows.start is None and rows.stop is None:
                pos = torch.arange(len(idx), dtype=torch.int64)
            else:
                start = rows.start if rows.start is not None else idx.index_values[0]
                stop = rows.stop if rows.stop is not None else idx.index_values[-1]
                pos = idx.range_positions(start, stop)
        elif isinstance(rows, (list, tuple)):
            pos = idx.positions_of_list(rows)
        else:
            pos = idx.positions_of(rows).cpu()
        return self._select(pos, cols)


class ILocIndexer(_Indexer):
    """table.iloc[rows, cols]: positional rows (int / list / slice, exclusive stop) and columns."""

    def __getitem__(self, key):
        rows, cols = (key if isinstance(key, tuple) else (key, None))
        n = self._t.row_count
        if isinstance(rows, slice):
            pos = torch.arange(n, dtype=torch.int64)[rows]
        elif isinstance(rows, (list, tuple)):
            pos = torch.tensor([r if r >= 0 else n + r for r in rows], dtype=torch.int64)
        else:
            r = int(rows)
            pos = torch.tensor([r if r >= 0 else n + r], dtype=torch.int64)
        if isinstance(cols, slice) and (cols.start is None or isinstance(cols.start, int)) and \
                (cols.stop is None or isinstance(cols.stop, int)):
            cols = list(range(self._t.column_count))[cols]
        return self._select(pos, cols)


class PyLocIndexer:
    """Reference python/pycylon/indexing/index.pyx PyLocIndexer: ``PyLocIndexer(table, "loc" | "iloc")[rows, cols]``."""

    def __init__(self, cn_table, mode):
        if mode not in ("loc", "iloc"):
            raise ValueError(f"unsupported indexing mode {mode}")
        self._indexer = (LocIndexer if mode == "loc" else ILocIndexer)(cn_table)

    def __getitem__(self, item):
        return self._indexer[item]


__all__ = ["IndexingSchema", "BaseIndex", "LinearIndex", "HashIndex", "RangeIndex", "build_index", "LocIndexer",
           "ILocIndexer", "PyLocIndexer"]
