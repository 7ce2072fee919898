"""Index construction helpers (reference: python/pycylon/indexing/index_utils.pyx,
cpp/src/cylon/indexing/index_utils.cpp)."""
from typing import List

import pyarrow as pa

from .index import IndexingSchema, build_index


class IndexUtil:
    @staticmethod
    def build_index(indexing_schema: IndexingSchema, table, column: int, drop: bool):
        """A copy of `table` indexed by column `column` (removed from the columns when drop)."""
        out = table.project(list(range(table.column_count)))
        return out.set_index(column, indexing_schema, drop)

    @staticmethod
    def build_index_from_list(indexing_schema: IndexingSchema, table, index_arr: List):
        if len(index_arr) != table.row_count:
            raise ValueError(f"index of length {len(index_arr)} for a table of {table.row_count} rows")
        out = table.project(list(range(table.column_count)))
        out.set_index(build_index(pa.array(index_arr), indexing_schema, table.device))
        return out
