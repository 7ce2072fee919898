"""Common API objects (reference: python/pycylon/common/join_config.pyx:20-115,
common/status.pyx, common/code.pyx; cpp/src/cylon/code.cpp, status.hpp)."""
from enum import IntEnum
from typing import List, Union


class Code(IntEnum):
    OK = 0
    OutOfMemory = 1
    KeyError = 2
    TypeError = 3
    Invalid = 4
    IOError = 5
    CapacityError = 6
    IndexError = 7
    UnknownError = 9
    NotImplemented = 10
    SerializationError = 11
    GpuMemoryError = 12
    RError = 13
    CodeGenError = 40
    ExpressionValidationError = 41
    ExecutionError = 42
    AlreadyExists = 45


class Status:
    def __init__(self, code: Union[int, Code] = Code.OK, msg: str = ""):
        self._code = int(code)
        self._msg = msg

    def get_code(self) -> int:
        return self._code

    def get_msg(self) -> str:
        return self._msg

    def is_ok(self) -> bool:
        return self._code == Code.OK

    @staticmethod
    def OK() -> "Status":
        return Status(Code.OK)

    @staticmethod
    def from_exception(e: Exception) -> "Status":
        code = e.args[1] if len(e.args) > 1 and isinstance(e.args[1], int) else Code.UnknownError
        return Status(code, str(e.args[0]) if e.args else str(e))

    def __repr__(self):
        return f"Status({Code(self._code).name}, {self._msg!r})"


class JoinType(IntEnum):
    INNER = 0
    LEFT = 1
    RIGHT = 2
    FULL_OUTER = 3


class JoinAlgorithm(IntEnum):
    SORT = 0
    HASH = 1


_JT = {"inner": JoinType.INNER, "left": JoinType.LEFT, "right": JoinType.RIGHT, "outer": JoinType.FULL_OUTER,
       "full_outer": JoinType.FULL_OUTER, "fullouter": JoinType.FULL_OUTER}
_JA = {"sort": JoinAlgorithm.SORT, "hash": JoinAlgorithm.HASH}
_JT_STR = {JoinType.INNER: "inner", JoinType.LEFT: "left", JoinType.RIGHT: "right", JoinType.FULL_OUTER: "outer"}


class JoinConfig:
    """JoinConfig(join_type, join_algorithm, left_column_index, right_column_index, left_prefix, right_prefix)"""

    def __init__(self, join_type: Union[str, JoinType] = "inner", join_algorithm: Union[str, JoinAlgorithm] = "sort",
                 left_column_index: Union[int, List[int]] = 0, right_column_index: Union[int, List[int]] = 0,
                 left_prefix: str = "", right_prefix: str = ""):
        self.join_type = _JT[join_type.lower()] if isinstance(join_type, str) else JoinType(join_type)
        self.join_algorithm = _JA[join_algorithm.lower()] if isinstance(join_algorithm, str) else \
            JoinAlgorithm(join_algorithm)
        self.left_columns = [left_column_index] if isinstance(left_column_index, int) else list(left_column_index)
        self.right_columns = [right_column_index] if isinstance(right_column_index, int) else list(right_column_index)
        if len(self.left_columns) != len(self.right_columns):
            raise ValueError("left and right column indices sizes are not equal")
        self.left_prefix = left_prefix
        self.right_prefix = right_prefix

    @property
    def left_column_idx(self):
        return self.left_columns

    @property
    def right_column_idx(self):
        return self.right_columns

    @property
    def join_type_str(self) -> str:
        return _JT_STR[self.join_type]

    @property
    def join_algorithm_str(self) -> str:
        return "hash" if self.join_algorithm == JoinAlgorithm.HASH else "sort"

    def apply(self, left, right, distributed: bool = False):
        fn = left.distributed_join if distributed else left.join
        return fn(right, self.join_type_str, self.join_algorithm_str, left_on=self.left_columns,
                  right_on=self.right_columns, left_prefix=self.left_prefix, right_prefix=self.right_prefix)


__all__ = ["Code", "Status", "JoinType", "JoinAlgorithm", "JoinConfig"]
