"""cylon_amd.ops: functional operator API over Tables (mirrors the C++ `cylon::ops` /
reference `cylon/table.hpp` free functions: Join, DistributedJoin, Union, ..., Sort,
DistributedSort, Shuffle, HashPartition, Unique, GroupBy, aggregates).

Every function is a thin call into the native extension; the Table methods of
`cylon_amd.Table` are the object-style spelling of the same operators.
"""
from typing import Dict, List, Sequence, Union

from ..data.table import SortOptions, Table


def join(left: Table, right: Table, join_type: str = "inner", algorithm: str = "sort", **kw) -> Table:
    return left.join(right, join_type, algorithm, **kw)


def distributed_join(left: Table, right: Table, join_type: str = "inner", algorithm: str = "sort", **kw) -> Table:
    return left.distributed_join(right, join_type, algorithm, **kw)


def union(a: Table, b: Table) -> Table:
    return a.union(b)


def subtract(a: Table, b: Table) -> Table:
    return a.subtract(b)


def intersect(a: Table, b: Table) -> Table:
    return a.intersect(b)


def distributed_union(a: Table, b: Table) -> Table:
    return a.distributed_union(b)


def distributed_subtract(a: Table, b: Table) -> Table:
    return a.distributed_subtract(b)


def distributed_intersect(a: Table, b: Table) -> Table:
    return a.distributed_intersect(b)


def sort(t: Table, order_by=None, ascending: Union[bool, List[bool]] = True) -> Table:
    return t.sort(order_by, ascending)


def distributed_sort(t: Table, order_by=None, ascending: Union[bool, List[bool]] = True,
                     sort_options: SortOptions = None) -> Table:
    return t.distributed_sort(order_by, ascending, sort_options)


def shuffle(t: Table, hash_columns: List = None) -> Table:
    return t.shuffle(hash_columns)


def hash_partition(t: Table, hash_columns: List, num_partitions: int) -> List[Table]:
    return t.hash_partition(hash_columns, num_partitions)


def unique(t: Table, columns: Sequence = None, keep: str = "first") -> Table:
    return t.unique(columns, keep)


def distributed_unique(t: Table, columns: Sequence = None) -> Table:
    return t.distributed_unique(columns)


def groupby(t: Table, index, agg: Dict, algorithm: str = "hash") -> Table:
    """Distributed (two-phase) group-by; equals local_groupby on a single rank."""
    return t.groupby(index, agg, algorithm)


def local_groupby(t: Table, index, agg: Dict, algorithm: str = "hash") -> Table:
    return t.local_groupby(index, agg, algorithm)


def project(t: Table, columns: Sequence) -> Table:
    return t.project(columns)


def merge(tables: Sequence[Table]) -> Table:
    return Table.merge(list(tables))


__all__ = ["join", "distributed_join", "union", "subtract", "intersect", "distributed_union",
           "distributed_subtract", "distributed_intersect", "sort", "distributed_sort", "shuffle",
           "hash_partition", "unique", "distributed_unique", "groupby", "local_groupby", "project", "merge"]
