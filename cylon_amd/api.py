"""C-API for native extensions (P8; reference python/pycylon/api/lib.pyx wrap/unwrap).

Tables and contexts cross into third-party C++ as PyCapsules holding a
`std::shared_ptr<cylon::Table>` ("cylon_amd.Table") or
`std::shared_ptr<cylon::CylonContext>` ("cylon_amd.Context"); a pybind11 module
built against `cylon_amd/csrc` headers unwraps them with
`*static_cast<std::shared_ptr<cylon::Table>*>(PyCapsule_GetPointer(obj, "cylon_amd.Table"))`.
Plain C / JNI callers use the C ABI in `cylon_amd/include/cylon_capi.h`
(exported from the same shared object; `capi_library()` loads it via ctypes).
"""
import ctypes

from ._lib import C
from .ctx.context import CylonContext
from .data.table import Table


def unwrap_table(table: Table):
    return C.table_to_capsule(table.native)


def wrap_table(capsule, context: CylonContext) -> Table:
    return Table(context=context, _native=C.table_from_capsule(capsule))


def unwrap_context(context: CylonContext):
    return C.context_to_capsule(context._ctx)


def wrap_context_native(capsule):
    """The native context inside a capsule (for CylonContext-level plumbing)."""
    return C.context_from_capsule(capsule)


ROW_PREDICATE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)


def capi_library() -> ctypes.CDLL:
    """ctypes handle on the C ABI (cylon_capi.h), with argument types declared."""
    lib = ctypes.CDLL(C.__file__)
    s, i, i64 = ctypes.c_char_p, ctypes.c_int, ctypes.c_int64
    sig = {
        "cylon_capi_version": ([], i), "cylon_last_error": ([], s), "cylon_init": ([s], i),
        "cylon_get_rank": ([], i), "cylon_get_world_size": ([], i), "cylon_barrier": ([], i),
        "cylon_finalize": ([], i), "cylon_read_csv": ([s, s], i), "cylon_write_csv": ([s, s], i),
        "cylon_row_count": ([s], i64), "cylon_column_count": ([s], ctypes.c_int32),
        "cylon_remove_table": ([s], i), "cylon_join": ([s, s, i, i, i, i, s], i),
        "cylon_distributed_join": ([s, s, i, i, i, i, s], i), "cylon_set_op": ([s, s, i, i, s], i),
        "cylon_sort": ([s, i, i, s], i), "cylon_project": ([s, ctypes.POINTER(ctypes.c_int32), i, s], i),
    }
    pp = ctypes.POINTER
    sig.update({
        "cylon_merge": ([pp(s), i, s], i), "cylon_print": ([s, i64, i64], i),
        "cylon_table_from_buffers": ([s, i, pp(s), pp(ctypes.c_int32), i64, pp(ctypes.c_void_p),
                                      pp(ctypes.c_void_p), pp(ctypes.c_void_p)], i),
        "cylon_select": ([s, ROW_PREDICATE, ctypes.c_void_p, s], i),
        "cylon_row_index": ([ctypes.c_void_p], i64), "cylon_row_is_null": ([ctypes.c_void_p, i], i),
        "cylon_row_get_int64": ([ctypes.c_void_p, i], i64),
        "cylon_row_get_double": ([ctypes.c_void_p, i], ctypes.c_double),
        "cylon_row_get_string": ([ctypes.c_void_p, i, ctypes.c_char_p, i64], i64),
    })
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes, f.restype = args, res
    return lib
