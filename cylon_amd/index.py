"""pandas-style index descriptors (reference: python/pycylon/index.py).

These are light metadata objects the DataFrame layer uses to describe an index
before it is materialised; the materialised, device-backed indexes (Range /
Linear / Hash with loc / iloc lookups) live in ``cylon_amd.indexing``.
"""
import warnings
from typing import List

import numpy as np

from .indexing.index import IndexingSchema
from .indexing.index_utils import IndexUtil
from .utils import resolve_column_index_from_column_name


class Index:
    def __init__(self, data=None):
        self._index_values = data

    def initialize(self):
        pass

    @property
    def index(self):
        return self

    @property
    def index_values(self):
        return self._index_values

    @index_values.setter
    def index_values(self, data):
        self._index_values = data


class NumericIndex(Index):
    def __init__(self, data):
        super().__init__(data)
        self.initialize()


class IntegerIndex(NumericIndex):
    pass


class RangeIndex(IntegerIndex):
    """range(start, stop, step) index; built from a ``range`` or from explicit bounds."""

    def __init__(self, data=None, start: int = 0, stop: int = 0, step: int = 0):
        self.start, self.stop, self.step = start, stop, step
        super().__init__(data)

    def initialize(self):
        if self.stop != 0:
            self._index_values = range(self.start, self.stop, self.step or 1)
        elif isinstance(self._index_values, range):
            r = self._index_values
            self.start, self.stop, self.step = r.start, r.stop, r.step
        else:
            warnings.warn("Empty Range!. Range data or range criteria must be passed")


class CategoricalIndex(Index):
    pass


class ColumnIndex(Index):
    pass


def range_calculator(rg: range) -> int:
    """Number of elements of a range (ceil((stop - start) / step))."""
    return len(rg)


def _is_index_and_range_validity(table, index_range) -> bool:
    return isinstance(index_range, range) and len(index_range) == table.row_count


def _is_index_list_and_valid(table, index) -> bool:
    return isinstance(index, list) and len(index) == table.row_count


def _is_index_list_of_columns(table, index) -> bool:
    return isinstance(index, list) and all(i in table.column_names for i in index)


def _get_index_list_from_columns(table, index):
    at = table.to_arrow()
    return [at.column(i) for i in (index if isinstance(index, list) else [index])]


def _is_index_str_and_valid(table, index) -> bool:
    return isinstance(index, str) and index in table.column_names


def _get_column_by_name(table, column_name):
    return table.to_arrow().column(column_name)


def process_index_by_value(key, table, index_schema=IndexingSchema.LINEAR, drop_index=False):
    """A table indexed by column `key` (name or position) or by the value list `key`."""
    if np.isscalar(key):
        col = resolve_column_index_from_column_name(key, table) if isinstance(key, str) else int(key)
        return IndexUtil.build_index(index_schema, table, col, drop_index)
    if isinstance(key, List):
        return IndexUtil.build_index_from_list(index_schema, table, key)
    raise ValueError("Unexpected value")


def _process_index_by_value(key, table):
    """Index descriptor for `key` (value list, column list, range, descriptor or column name)."""
    if _is_index_list_and_valid(table, key):
        return CategoricalIndex(key)
    if _is_index_list_of_columns(table, key):
        return ColumnIndex(_get_index_list_from_columns(table, key))
    if isinstance(key, range):
        if _is_index_and_range_validity(table, key):
            return RangeIndex(key)
        raise ValueError(f"Index type {key} not supported or invalid!")
    if isinstance(key, CategoricalIndex):
        if _is_index_list_and_valid(table, list(key.index_values)):
            return key
        raise ValueError(f"Index type {key.index_values} not supported or invalid!")
    if isinstance(key, NumericIndex):
        if _is_index_list_and_valid(table, key.index_values):
            return CategoricalIndex(key.index_values)
        if _is_index_and_range_validity(table, key.index_values):
            return RangeIndex(key.index_values)
        raise ValueError(f"Index type {key.index_values} not supported or invalid!")
    if _is_index_str_and_valid(table, key):
        return ColumnIndex(_get_column_by_name(table, key))
    raise ValueError(f"Index type {key} not supported or invalid!")
