"""Table I/O (reference: cpp/src/cylon/io/arrow_io.cpp:33-116, csv_read_config.hpp,
csv_write_config.hpp, parquet_config.hpp; python/pycylon/io/*.pyx, data/csv.pyx).

Parsing stays on the host in Arrow's multi-threaded C++ readers (as in the
reference); the parsed columns are then moved to the context's device in one
H2D copy per buffer.  Several files are read concurrently, one thread each
(reference table.cpp:799-829).
"""
import os
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence, Union

import pyarrow as pa
import pyarrow.csv as pacsv

from .._lib import C

Type = C.Type
from ..ctx.context import CylonContext
from ..data.table import Table, _ensure_ctx


def _arrow_type(t):
    if isinstance(t, pa.DataType):
        return t
    from .. import types as cytypes
    return cytypes.to_arrow(t)


class CSVReadOptions:
    """Builder with both pycylon (snake_case) and C++ (CamelCase) spellings."""

    def __init__(self):
        self._use_threads = True
        self._block_size = 1 << 20
        self._delimiter = ","
        self._ignore_empty_lines = True
        self._autogenerate_column_names = False
        self._column_names: Optional[List[str]] = None
        self._skip_rows = 0
        self._column_types: Dict[str, pa.DataType] = {}
        self._null_values: Optional[List[str]] = None
        self._true_values: Optional[List[str]] = None
        self._false_values: Optional[List[str]] = None
        self._strings_can_be_null = False
        self._include_columns: Optional[List[str]] = None
        self._include_missing_columns = False
        self._quoting = True
        self._quote_char = '"'
        self._double_quote = True
        self._escaping = False
        self._escape_char = "\\"
        self._newlines_in_values = False

    # pycylon spellings
    def use_threads(self, v: bool = True):
        self._use_threads = bool(v)
        return self

    def block_size(self, b: int):
        self._block_size = int(b)
        return self

    def with_delimiter(self, d: str):
        self._delimiter = d[0]
        return self

    def ignore_emptylines(self, v: bool = True):
        self._ignore_empty_lines = v
        return self

    def use_cols(self, cols: List):
        self._include_columns = [str(c) for c in cols]
        return self

    def skip_rows(self, rows: int = 0):
        self._skip_rows = int(rows)
        return self

    def na_values(self, vals: List[str]):
        self._null_values = list(vals)
        return self

    def with_column_types(self, types: Dict[str, object]):
        self._column_types = {str(k): _arrow_type(v) for k, v in types.items()}
        return self

    def column_names(self, names: List[str]):
        self._column_names = list(names)
        return self

    def autogenerate_column_names(self, v: bool = True):
        self._autogenerate_column_names = v
        return self

    def true_values(self, vals):
        self._true_values = list(vals)
        return self

    def false_values(self, vals):
        self._false_values = list(vals)
        return self

    def strings_can_be_null(self, v: bool = True):
        self._strings_can_be_null = v
        return self

    def include_missing_columns(self, v: bool = True):
        self._include_missing_columns = v
        return self

    def use_quoting(self, v: bool = True):
        self._quoting = v
        return self

    def with_quote_char(self, c: str):
        self._quote_char = c
        return self

    def double_quote(self, v: bool = True):
        self._double_quote = v
        return self

    def use_escaping(self, v: bool = True):
        self._escaping = v
        return self

    def escaping_character(self, c: str):
        self._escape_char = c
        self._escaping = True
        return self

    def has_new_lines_in_values(self, v: bool = True):
        self._newlines_in_values = v
        return self

    # C++ spellings (cylon/io/csv_read_config.hpp)
    UseThreads = use_threads
    BlockSize = block_size
    WithDelimiter = with_delimiter
    IgnoreEmptyLines = ignore_emptylines
    SkipRows = skip_rows
    NullValues = na_values
    WithColumnTypes = with_column_types
    ColumnNames = column_names
    AutoGenerateColumnNames = autogenerate_column_names
    TrueValues = true_values
    FalseValues = false_values
    StringsCanBeNull = strings_can_be_null
    IncludeColumns = use_cols
    IncludeMissingColumns = include_missing_columns
    UseQuoting = use_quoting
    WithQuoteChar = with_quote_char
    DoubleQuote = double_quote
    UseEscaping = use_escaping
    EscapingCharacter = escaping_character
    HasNewLinesInValues = has_new_lines_in_values

    def _arrow(self):
        ro = pacsv.ReadOptions(use_threads=self._use_threads, block_size=self._block_size,
                               skip_rows=self._skip_rows, column_names=self._column_names,
                               autogenerate_column_names=self._autogenerate_column_names)
        po = pacsv.ParseOptions(delimiter=self._delimiter, quote_char=self._quote_char if self._quoting else False,
                                double_quote=self._double_quote,
                                escape_char=self._escape_char if self._escaping else False,
                                newlines_in_values=self._newlines_in_values,
                                ignore_empty_lines=self._ignore_empty_lines)
        kw = dict(column_types=self._column_types or None, strings_can_be_null=self._strings_can_be_null,
                  include_columns=self._include_columns,
                  include_missing_columns=self._include_missing_columns)
        if self._null_values is not None:
            kw["null_values"] = self._null_values
        if self._true_values is not None:
            kw["true_values"] = self._true_values
        if self._false_values is not None:
            kw["false_values"] = self._false_values
        co = pacsv.ConvertOptions(**kw)
        return ro, po, co


class CSVWriteOptions:
    def __init__(self):
        self._delimiter = ","
        self._column_names: Optional[List[str]] = None

    def with_delimiter(self, d: str):
        self._delimiter = d
        return self

    def with_column_names(self, names=None):
        self._column_names = list(names or [])
        return self

    def delimiter(self) -> str:
        return self._delimiter

    def column_names(self) -> List[str]:
        return self._column_names or []

    WithDelimiter = with_delimiter
    ColumnNames = with_column_names


_NATIVE_COLUMN_TYPES = {
    pa.int8(): Type.INT8, pa.int16(): Type.INT16, pa.int32(): Type.INT32, pa.int64(): Type.INT64,
    pa.uint8(): Type.UINT8, pa.uint16(): Type.UINT16, pa.uint32(): Type.UINT32, pa.uint64(): Type.UINT64,
    pa.float16(): Type.HALF_FLOAT, pa.float32(): Type.FLOAT, pa.float64(): Type.DOUBLE, pa.bool_(): Type.BOOL,
    pa.string(): Type.STRING, pa.binary(): Type.BINARY,
}


def _native_ok(o: CSVReadOptions) -> bool:
    """Options the native C++ reader (cylon/io/csv.cpp) implements; explicit column types
    other than plain numeric / bool / string ones go through Arrow."""
    return all(t in _NATIVE_COLUMN_TYPES for t in o._column_types.values())


def _read_native(ctx: CylonContext, paths: Sequence[str], o: CSVReadOptions) -> List[Table]:
    nulls = o._null_values
    if nulls is not None and len(nulls) == 0:
        nulls = ["\x00"]  # explicit empty list: nothing is null
    tabs = C.read_csv(ctx._ctx, list(paths), delimiter=o._delimiter, header=True,
                      autogenerate_column_names=o._autogenerate_column_names,
                      column_names=o._column_names or [], skip_rows=o._skip_rows,
                      ignore_empty_lines=o._ignore_empty_lines, include_columns=o._include_columns or [],
                      null_values=nulls or [], true_values=o._true_values or [],
                      false_values=o._false_values or [], strings_can_be_null=o._strings_can_be_null,
                      quoting=o._quoting, quote_char=o._quote_char, double_quote=o._double_quote,
                      threads=0 if o._use_threads else 1, escaping=o._escaping, escape_char=o._escape_char,
                      newlines_in_values=o._newlines_in_values,
                      column_types={k: int(_NATIVE_COLUMN_TYPES[t]) for k, t in o._column_types.items()},
                      include_missing_columns=o._include_missing_columns, block_size=o._block_size)
    return [Table(context=ctx, _native=t) for t in tabs]


def _read_one_csv(path: str, options: CSVReadOptions) -> pa.Table:
    ro, po, co = options._arrow()
    try:
        small = os.path.getsize(path) <= max(ro.block_size, 1 << 20)
    except OSError:
        small = False
    if small:
        # one block: the streaming reader infers types from the whole file and skips
        # read_csv's per-call traceback-cycle sweep (a gc.get_referrers walk, ~6 ms)
        with pacsv.open_csv(path, read_options=ro, parse_options=po, convert_options=co) as r:
            return r.read_all()
    return pacsv.read_csv(path, read_options=ro, parse_options=po, convert_options=co)


def read_csv(context: CylonContext, path: Union[str, Sequence[str]], csv_read_options: CSVReadOptions = None):
    """Read one CSV file into a Table, or several concurrently into a list of Tables."""
    ctx = _ensure_ctx(context)
    opts = csv_read_options or CSVReadOptions()
    if _native_ok(opts) and os.environ.get("CYLON_CSV_READER", "native") == "native":
        tabs = _read_native(ctx, list(path) if isinstance(path, (list, tuple)) else [path], opts)
        return tabs if isinstance(path, (list, tuple)) else tabs[0]
    if isinstance(path, (list, tuple)):
        with ThreadPoolExecutor(max_workers=max(1, len(path))) as ex:
            tabs = list(ex.map(lambda p: _read_one_csv(p, opts), path))
        return [Table(t, ctx) for t in tabs]
    return Table(_read_one_csv(path, opts), ctx)


def write_csv(table: Table, path: str, csv_write_options: CSVWriteOptions = None):
    opts = csv_write_options or CSVWriteOptions()
    at = table.to_arrow()
    if opts.column_names():
        at = at.rename_columns(opts.column_names())
    pacsv.write_csv(at, path, write_options=pacsv.WriteOptions(delimiter=opts.delimiter()))


class ParquetOptions:
    """reference: cpp/src/cylon/io/parquet_config.hpp:24-53 (concurrent file reads, chunk size,
    writer properties -> compression here); `columns` selects / orders the columns to read."""

    def __init__(self, concurrent_file_reads: bool = True, chunk_size: int = 1 << 20,
                 compression: str = "snappy", columns: Sequence[str] = (), use_threads: bool = True):
        self.concurrent_file_reads = concurrent_file_reads
        self.chunk_size = chunk_size
        self.compression = compression
        self.columns = list(columns)
        self.use_threads = use_threads

    def ConcurrentFileReads(self, v: bool) -> "ParquetOptions":
        self.concurrent_file_reads = v
        return self

    def ChunkSize(self, rows: int) -> "ParquetOptions":
        self.chunk_size = rows
        return self


def read_parquet(context: CylonContext, path: Union[str, Sequence[str]], options: ParquetOptions = None):
    """Native Parquet reader (io/arrow_io.cpp, Arrow / Parquet C++): a Table, or a list of Tables
    for a list of paths (read concurrently, one thread per file)."""
    ctx = _ensure_ctx(context)
    opts = options or ParquetOptions()
    paths = list(path) if isinstance(path, (list, tuple)) else [path]
    natives = C.read_parquet(ctx._ctx, [str(p) for p in paths], opts.columns, opts.use_threads,
                             opts.concurrent_file_reads)
    tables = [Table(None, ctx, _native=n) for n in natives]
    return tables if isinstance(path, (list, tuple)) else tables[0]


def write_parquet(table: Table, path: str, options: ParquetOptions = None):
    opts = options or ParquetOptions()
    C.write_parquet(table.native, str(path), opts.compression or "none", max(1, int(opts.chunk_size)))


def write_arrow_ipc(table: Table, path: str):
    """Arrow IPC (Feather v2) serialisation of a device table."""
    at = table.to_arrow()
    with pa.OSFile(path, "wb") as sink, pa.ipc.new_file(sink, at.schema) as writer:
        writer.write_table(at)


def read_arrow_ipc(context: CylonContext, path: str) -> Table:
    with pa.memory_map(path, "r") as src:
        at = pa.ipc.open_file(src).read_all()
    return Table(at, _ensure_ctx(context))


__all__ = ["CSVReadOptions", "CSVWriteOptions", "ParquetOptions", "read_csv", "write_csv", "read_parquet",
           "write_parquet", "write_arrow_ipc", "read_arrow_ipc"]
