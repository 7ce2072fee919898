"""Type factories (reference: python/pycylon/types.py:21-126, cpp/src/cylon/data_types.hpp)."""
import pyarrow as pa

from ._lib import C

Type = C.Type
Layout = C.Layout
DataType = C.DataType


def _dt(t, w=0):
    return C.DataType(t, w) if w else C.DataType(t)


def int8(): return _dt(Type.INT8)
def int16(): return _dt(Type.INT16)
def int32(): return _dt(Type.INT32)
def int64(): return _dt(Type.INT64)
def uint8(): return _dt(Type.UINT8)
def uint16(): return _dt(Type.UINT16)
def uint32(): return _dt(Type.UINT32)
def uint64(): return _dt(Type.UINT64)
def half_float(): return _dt(Type.HALF_FLOAT)
def float(): return _dt(Type.FLOAT)  # noqa: A001 (pycylon name)
def double(): return _dt(Type.DOUBLE)
def string(): return _dt(Type.STRING)
def binary(): return _dt(Type.BINARY)
def bool(): return _dt(Type.BOOL)  # noqa: A001 (pycylon name)
def fixed_sized_binary(width: int = 1): return _dt(Type.FIXED_SIZE_BINARY, width)
def date32(): return _dt(Type.DATE32)
def date64(): return _dt(Type.DATE64)
def timestamp(): return _dt(Type.TIMESTAMP)
def time32(): return _dt(Type.TIME32)
def time64(): return _dt(Type.TIME64)
def interval(): return _dt(Type.INTERVAL)
def decimal(): return _dt(Type.DECIMAL, 16)
def list(): return _dt(Type.LIST)  # noqa: A001
def fixed_sized_list(): return _dt(Type.FIXED_SIZE_LIST)
def extension(): return _dt(Type.EXTENSION)
def duration(): return _dt(Type.DURATION)


def to_arrow(t) -> pa.DataType:
    """Accepts a cylon DataType / Type, a numpy/pyarrow type or a type name."""
    from .data.arrow_bridge import to_arrow_type
    if isinstance(t, pa.DataType):
        return t
    if isinstance(t, C.DataType):
        return to_arrow_type(t)
    if isinstance(t, C.Type):
        return to_arrow_type(C.DataType(t))
    if isinstance(t, str):
        return pa.type_for_alias(t)
    return pa.from_numpy_dtype(t)
