"""Arrow <-> device column bridge (reference: cpp/src/cylon/arrow/arrow_types.cpp,
arrow_builder.cpp; python/pycylon/data/table.pyx from_arrow/to_arrow).

Host Arrow buffers are viewed zero-copy through numpy, moved to the context
device in one H2D copy per buffer, and kept in the engine's layout:
fixed width values, int64 string offsets, uint8 validity byte-mask.
"""
import os
from typing import Optional

import numpy as np
import pyarrow as pa
import torch

from .._lib import C

T = C.Type

_UNIT = {"s": 0, "ms": 1, "us": 2, "ns": 3}
_UNIT_INV = {v: k for k, v in _UNIT.items()}

_SIMPLE = {
    pa.bool_(): T.BOOL, pa.uint8(): T.UINT8, pa.int8(): T.INT8, pa.uint16(): T.UINT16, pa.int16(): T.INT16,
    pa.uint32(): T.UINT32, pa.int32(): T.INT32, pa.uint64(): T.UINT64, pa.int64(): T.INT64,
    pa.float16(): T.HALF_FLOAT, pa.float32(): T.FLOAT, pa.float64(): T.DOUBLE, pa.date32(): T.DATE32,
    pa.date64(): T.DATE64,
}

_NP = {
    T.BOOL: np.uint8, T.UINT8: np.uint8, T.INT8: np.int8, T.UINT16: np.uint16, T.INT16: np.int16,
    T.UINT32: np.uint32, T.INT32: np.int32, T.UINT64: np.uint64, T.INT64: np.int64, T.HALF_FLOAT: np.float16,
    T.FLOAT: np.float32, T.DOUBLE: np.float64, T.DATE32: np.int32, T.DATE64: np.int64, T.TIMESTAMP: np.int64,
    T.TIME32: np.int32, T.TIME64: np.int64, T.DURATION: np.int64,
}

_TORCH = {
    T.BOOL: torch.uint8, T.UINT8: torch.uint8, T.INT8: torch.int8, T.UINT16: torch.uint16, T.INT16: torch.int16,
    T.UINT32: torch.uint32, T.INT32: torch.int32, T.UINT64: torch.uint64, T.INT64: torch.int64,
    T.HALF_FLOAT: torch.float16, T.FLOAT: torch.float32, T.DOUBLE: torch.float64, T.DATE32: torch.int32,
    T.DATE64: torch.int64, T.TIMESTAMP: torch.int64, T.TIME32: torch.int32, T.TIME64: torch.int64,
    T.DURATION: torch.int64,
}


def to_cylon_type(at: pa.DataType) -> "C.DataType":
    if at in _SIMPLE:
        return C.DataType(_SIMPLE[at])
    if pa.types.is_string(at) or pa.types.is_large_string(at):
        return C.DataType(T.STRING)
    if pa.types.is_binary(at) or pa.types.is_large_binary(at):
        return C.DataType(T.BINARY)
    if pa.types.is_fixed_size_binary(at):
        return C.DataType(T.FIXED_SIZE_BINARY, at.byte_width)
    if pa.types.is_decimal(at):
        d = C.DataType(T.DECIMAL, at.byte_width)
        d.precision, d.scale = at.precision, at.scale
        return d
    if pa.types.is_timestamp(at):
        d = C.DataType(T.TIMESTAMP)
        d.unit = _UNIT[at.unit]
        d.timezone = at.tz or ""
        return d
    if pa.types.is_time32(at) or pa.types.is_time64(at):
        d = C.DataType(T.TIME32 if pa.types.is_time32(at) else T.TIME64)
        d.unit = _UNIT[at.unit]
        return d
    if pa.types.is_duration(at):
        d = C.DataType(T.DURATION)
        d.unit = _UNIT[at.unit]
        return d
    if pa.types.is_dictionary(at):
        return to_cylon_type(at.value_type)
    if pa.types.is_list(at) or pa.types.is_large_list(at) or pa.types.is_fixed_size_list(at):
        vt = at.value_type
        if vt not in _SIMPLE or vt == pa.bool_() or not (pa.types.is_integer(vt) or pa.types.is_floating(vt)):
            raise TypeError(f"arrow type {at} is not supported by cylon_amd (list elements must be numeric)")
        if pa.types.is_fixed_size_list(at):
            return C.DataType.fixed_size_list_of(_SIMPLE[vt], at.list_size)
        return C.DataType.list_of(_SIMPLE[vt])
    raise TypeError(f"arrow type {at} is not supported by cylon_amd")


def to_arrow_type(dt: "C.DataType") -> pa.DataType:
    t = dt.type
    inv = {v: k for k, v in _SIMPLE.items()}
    if t in inv:
        return inv[t]
    if t == T.STRING:
        return pa.string()
    if t == T.BINARY:
        return pa.binary()
    if t == T.FIXED_SIZE_BINARY:
        return pa.binary(dt.byte_width)
    if t == T.DECIMAL:
        if dt.byte_width == 32:
            return pa.decimal256(dt.precision or 76, dt.scale)
        return pa.decimal128(dt.precision or 38, dt.scale)
    if t == T.TIMESTAMP:
        return pa.timestamp(_UNIT_INV[dt.unit], tz=dt.timezone or None)
    if t == T.TIME32:
        return pa.time32(_UNIT_INV[dt.unit])
    if t == T.TIME64:
        return pa.time64(_UNIT_INV[dt.unit])
    if t == T.DURATION:
        return pa.duration(_UNIT_INV[dt.unit])
    if t == T.LIST:
        return pa.list_(inv[dt.value_type])
    if t == T.FIXED_SIZE_LIST:
        return pa.list_(inv[dt.value_type], dt.list_size)
    raise TypeError(f"cylon type {dt} has no arrow mapping")


def torch_dtype(dt: "C.DataType"):
    return _TORCH.get(dt.type, torch.uint8)


_STAGED_MIN_BYTES = 1 << 20


def _staged_ingest() -> bool:
    """CYLON_STAGED_INGEST=0 falls back to torch's pageable copy (A/B knob, tools/ingest_bench.py)."""
    return os.environ.get("CYLON_STAGED_INGEST", "1") != "0"


def _to_dev(a: np.ndarray, device: str) -> torch.Tensor:
    """Host array -> tensor on `device`.  Device copies of >= 1 MiB go through the native pinned
    staging ring (io/h2d.cpp: worker threads fill pinned chunks while the DMA engine drains
    the previous ones; the device's current stream waits on the copy, the host does not)."""
    a = np.ascontiguousarray(a)
    if device != "cpu" and a.nbytes >= _STAGED_MIN_BYTES and _staged_ingest():
        out = torch.empty(a.shape, dtype=torch.from_numpy(np.empty(0, a.dtype)).dtype, device=device)
        C.h2d_copy(a.ctypes.data, a.nbytes, out)
        return out
    t = torch.from_numpy(a.copy() if not a.flags.writeable else a)
    return t.to(device, non_blocking=False) if device != "cpu" else t


def column_from_arrow(name: str, arr, device: str) -> "C.Column":
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
    if pa.types.is_dictionary(arr.type):
        arr = arr.dictionary_decode()
    dt = to_cylon_type(arr.type)
    n = len(arr)
    off = arr.offset
    bufs = arr.buffers()
    validity = None
    if arr.null_count > 0 and bufs[0] is not None:
        # the packed bitmap crosses to the device (1/8 of the bytes) and is unpacked there
        nb = (off + n + 7) // 8
        bits = _to_dev(np.frombuffer(bufs[0], dtype=np.uint8)[:nb], device)
        validity = C.unpack_validity(bits, off, n)
    t = dt.type
    if t in (T.STRING, T.BINARY):
        large = pa.types.is_large_string(arr.type) or pa.types.is_large_binary(arr.type)
        otype = np.int64 if large else np.int32
        offsets = np.frombuffer(bufs[1], dtype=otype)[off:off + n + 1].astype(np.int64) if n else np.zeros(1, np.int64)
        base = int(offsets[0]) if n else 0
        end = int(offsets[-1]) if n else 0
        data = np.frombuffer(bufs[2], dtype=np.uint8)[base:end] if (bufs[2] is not None and end > base) else \
            np.zeros(0, np.uint8)
        offsets = offsets - base
        return C.Column(name, dt, n, _to_dev(data, device), _to_dev(offsets, device), validity)
    if t in (T.LIST, T.FIXED_SIZE_LIST):  # numeric lists: child values' bytes (+ byte offsets)
        w = dt.value_width()
        npt = _NP[dt.value_type]
        if t == T.FIXED_SIZE_LIST:
            k = dt.list_size
            child = arr.values.slice(off * k, n * k)
        else:
            eoffs = np.asarray(arr.offsets).astype(np.int64) if n else np.zeros(1, np.int64)
            child = arr.values.slice(int(eoffs[0]), int(eoffs[-1] - eoffs[0]))
        if child.null_count:  # element nulls are only allowed under null rows (their values are unused)
            cvalid = np.asarray(child.is_valid())
            row_of = np.arange(len(child)) // k if t == T.FIXED_SIZE_LIST else \
                np.searchsorted(eoffs - eoffs[0], np.arange(len(child)), side="right") - 1
            rvalid = np.asarray(arr.is_valid())
            if np.any(~cvalid & rvalid[row_of]):
                raise NotImplementedError(f"column {name}: null list elements are not supported")
            child = child.fill_null(0)
        cb = child.buffers()
        vals = np.frombuffer(cb[1], dtype=npt)[child.offset:child.offset + len(child)] if len(child) else \
            np.zeros(0, npt)
        data = vals.view(np.uint8)
        if t == T.FIXED_SIZE_LIST:
            return C.Column(name, dt, n, _to_dev(data, device), None, validity)
        return C.Column(name, dt, n, _to_dev(data, device), _to_dev((eoffs - eoffs[0]) * w, device), validity)
    if t == T.BOOL:  # the packed values cross (1/8 of the bytes) and are unpacked where they land
        if not n:
            return C.Column(name, dt, n, _to_dev(np.zeros(0, np.uint8), device), None, validity)
        packed = _to_dev(np.frombuffer(bufs[1], dtype=np.uint8)[:(off + n + 7) // 8], device)
        return C.Column(name, dt, n, C.unpack_validity(packed, off, n), None, validity)
    if t in (T.FIXED_SIZE_BINARY, T.DECIMAL):
        w = dt.byte_width
        data = np.frombuffer(bufs[1], dtype=np.uint8)[off * w:(off + n) * w]
        return C.Column(name, dt, n, _to_dev(data, device), None, validity)
    npt = _NP[t]
    data = np.frombuffer(bufs[1], dtype=npt)[off:off + n] if n else np.zeros(0, npt)
    return C.Column(name, dt, n, _to_dev(data, device), None, validity)


def column_to_arrow(col: "C.Column") -> pa.Array:
    dt = col.type
    n = col.length
    at = to_arrow_type(dt)
    vbuf = None
    null_count = 0
    if col.validity is not None and n:
        # packed on the device by one ballot per 64 rows; only the bitmap crosses to the host
        words, null_count = C.pack_validity(col.validity)
        if null_count:
            vbuf = pa.py_buffer(words.cpu().numpy().tobytes())
    t = dt.type
    data = col.data.cpu()
    if t in (T.STRING, T.BINARY):
        offsets = col.offsets.cpu().numpy()
        nbytes = int(offsets[-1]) if n else 0
        if nbytes >= 2 ** 31 - 1:
            at = pa.large_string() if t == T.STRING else pa.large_binary()
            obuf = pa.py_buffer(offsets.astype(np.int64))
        else:
            obuf = pa.py_buffer(offsets.astype(np.int32))
        dbuf = pa.py_buffer(data.numpy().tobytes())
        return pa.Array.from_buffers(at, n, [vbuf, obuf, dbuf], null_count=null_count)
    if t in (T.LIST, T.FIXED_SIZE_LIST):
        et = to_arrow_type(C.DataType(dt.value_type))
        w = dt.value_width()
        raw = data.numpy().tobytes()
        child = pa.Array.from_buffers(et, len(raw) // w, [None, pa.py_buffer(raw)])
        if t == T.FIXED_SIZE_LIST:
            return pa.Array.from_buffers(at, n, [vbuf], null_count=null_count, children=[child])
        eoffs = col.offsets.cpu().numpy() // w
        if len(child) >= 2 ** 31 - 1:
            at = pa.large_list(et)
            obuf = pa.py_buffer(eoffs.astype(np.int64))
        else:
            obuf = pa.py_buffer(eoffs.astype(np.int32))
        return pa.Array.from_buffers(at, n, [vbuf, obuf], null_count=null_count, children=[child])
    if t == T.BOOL:
        bits = np.packbits(data.numpy().astype(np.uint8) != 0, bitorder="little")
        return pa.Array.from_buffers(at, n, [vbuf, pa.py_buffer(bits)], null_count=null_count)
    if t == T.DECIMAL:
        return pa.Array.from_buffers(at, n, [vbuf, pa.py_buffer(data.numpy().tobytes())], null_count=null_count)
    arr = data.numpy()
    return pa.Array.from_buffers(at, n, [vbuf, pa.py_buffer(arr.tobytes())], null_count=null_count)


def table_from_arrow(ctx_native, table: pa.Table, device: str) -> "C.Table":
    cols = [column_from_arrow(name, table.column(i), device) for i, name in enumerate(table.column_names)]
    return C.Table(ctx_native, cols)


def table_to_arrow(ctable: "C.Table") -> pa.Table:
    cols = ctable.columns()
    return pa.Table.from_arrays([column_to_arrow(c) for c in cols], names=[c.name for c in cols])


def column_from_tensor(name: str, t: torch.Tensor, validity: Optional[torch.Tensor] = None) -> "C.Column":
    """Zero-copy column over a 1-D torch tensor (device tensors stay on device)."""
    m = {torch.bool: T.BOOL, torch.uint8: T.UINT8, torch.int8: T.INT8, torch.int16: T.INT16, torch.int32: T.INT32,
         torch.int64: T.INT64, torch.float16: T.HALF_FLOAT, torch.float32: T.FLOAT, torch.float64: T.DOUBLE,
         torch.uint16: T.UINT16, torch.uint32: T.UINT32, torch.uint64: T.UINT64}
    if t.dtype not in m:
        raise TypeError(f"unsupported tensor dtype {t.dtype}")
    typ = m[t.dtype]
    if t.dtype == torch.bool:
        t = t.to(torch.uint8)
    t = t.contiguous().reshape(-1)
    if validity is not None:
        validity = validity.to(torch.uint8).contiguous().reshape(-1)
    return C.Column(name, C.DataType(typ), t.numel(), t, None, validity)
