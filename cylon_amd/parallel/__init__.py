"""Distributed building blocks (L1/L4): streaming op graphs, table all-to-all,
task-level all-to-all and the string-ID table registry.

Reference: cpp/src/cylon/ops/** (DisJoinOP, DisUnionOp), arrow/arrow_all_to_all.*,
arrow/arrow_task_all_to_all.*, table_api.hpp.  All of these are native (C++)
here; this module is the thin Python surface.
"""
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .._lib import C
from ..ctx.context import CylonContext
from ..data.table import Table


class DisJoinOp:
    """Streaming distributed join: insert left (tag 100) / right (tag 200) batches, then execute.

    Graph: Partition -> AllToAll (RCCL) -> Split(num_splits) per side -> JoinOp, scheduled
    left-subtree, right-subtree, join (JoinExecution) so every rank issues the same collectives.
    """
    LEFT = 100
    RIGHT = 200

    def __init__(self, ctx: CylonContext, join_type: str = "inner", algorithm: str = "hash", left_on=(0,),
                 right_on=(0,), left_prefix: str = "", right_prefix: str = "", num_splits: int = 16):
        self._ctx = ctx
        self._cfg = (join_type, algorithm, list(left_on), list(right_on), left_prefix, right_prefix)
        self._splits = num_splits
        self._left: List[Table] = []
        self._right: List[Table] = []

    def insert_table(self, tag: int, table: Table):
        (self._left if tag == self.LEFT else self._right).append(table)

    def execute(self) -> List[Table]:
        jt, alg, lc, rc, lp, rp = self._cfg
        out = C.dis_join_op(self._ctx._ctx, [t.native for t in self._left], [t.native for t in self._right], jt, alg,
                            lc, rc, lp, rp, self._splits)
        return [Table(context=self._ctx, _native=t) for t in out]


class DisUnionOp:
    """Streaming distributed union (Partition on all columns -> AllToAll -> Union)."""

    def __init__(self, ctx: CylonContext):
        self._ctx = ctx
        self._tables: List[Table] = []

    def insert_table(self, tag: int, table: Table):
        self._tables.append(table)

    def execute(self) -> List[Table]:
        out = C.dis_union_op(self._ctx._ctx, [t.native for t in self._tables])
        return [Table(context=self._ctx, _native=t) for t in out]


class TableAllToAll:
    """insert(table, target[, reference]) / finish() / is_complete() protocol of the reference's
    ArrowAllToAll; received tables are delivered to `callback(source, table, reference)`."""

    def __init__(self, ctx: CylonContext, callback: Optional[Callable[[int, Table, int], bool]] = None):
        self._ctx = ctx
        self._h = C.TableAllToAll(ctx._ctx)
        self._cb = callback
        self._delivered = False

    def insert(self, table: Table, target: int, reference: int = 0) -> int:
        return self._h.insert(table.native, int(target), int(reference))

    def finish(self):
        self._h.finish()

    def is_complete(self) -> bool:
        done = self._h.is_complete()
        if done and not self._delivered:
            self._delivered = True
            if self._cb is not None:
                for src, t, ref in self._h.received():
                    self._cb(src, Table(context=self._ctx, _native=t), ref)
        return done

    def received(self) -> List[Tuple[int, Table, int]]:
        return [(s, Table(context=self._ctx, _native=t), r) for s, t, r in self._h.received()]

    def close(self):
        self._h.close()


class TaskAllToAll:
    """Logical tasks mapped to workers (reference LogicalTaskPlan / ArrowTaskAllToAll)."""

    def __init__(self, ctx: CylonContext, task_to_worker: Sequence[int], callback=None):
        self._plan = list(task_to_worker)
        self._inner = TableAllToAll(ctx, callback)

    def insert(self, table: Table, target_task: int) -> int:
        return self._inner.insert(table, self._plan[target_task], target_task)

    def wait_for_completion(self):
        self._inner.finish()
        while not self._inner.is_complete():
            pass
        return self._inner.received()


class TableRegistry:
    """String-ID table registry + ID-based operators (reference table_api.hpp:38-195)."""

    def __init__(self, ctx: CylonContext):
        self._ctx = ctx

    def put(self, table_id: str, table: Table):
        C.registry_put(table_id, table.native)

    def get(self, table_id: str) -> Table:
        return Table(context=self._ctx, _native=C.registry_get(table_id))

    def remove(self, table_id: str):
        C.registry_remove(table_id)

    def ids(self) -> List[str]:
        return C.registry_list()

    def row_count(self, table_id: str) -> int:
        return C.registry_row_count(table_id)

    def column_count(self, table_id: str) -> int:
        return C.registry_column_count(table_id)

    def join(self, left_id, right_id, dest_id, join_type="inner", algorithm="sort", left_on=(0,), right_on=(0,),
             distributed=False):
        code, msg = C.registry_join(left_id, right_id, join_type, algorithm, list(left_on), list(right_on), dest_id,
                                    distributed)
        if code != 0:
            raise RuntimeError(msg)

    def union(self, a, b, dest_id, distributed=False):
        code, msg = C.registry_union(a, b, dest_id, distributed)
        if code != 0:
            raise RuntimeError(msg)


__all__ = ["DisJoinOp", "DisUnionOp", "TableAllToAll", "TaskAllToAll", "TableRegistry"]
