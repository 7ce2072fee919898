"""Small pycylon utilities (reference: python/pycylon/util/FileUtils.py,
TableUtils.py, type_utils.py)."""
import os
from typing import List, Optional

import pyarrow as pa

# dtype names / Python types -> Arrow types, as pycylon's get_arrow_type resolves them
_STR_TYPES = {"int8": pa.int8(), "int16": pa.int16(), "int32": pa.int32(), "int64": pa.int64(),
              "uint8": pa.uint8(), "uint16": pa.uint16(), "uint32": pa.uint32(), "uint64": pa.uint64(),
              "half_float": pa.float16(), "float": pa.float32(), "float32": pa.float32(),
              "float64": pa.float64(), "double": pa.float64(), "string": pa.string(), "str": pa.string(),
              "binary": pa.binary(), "bool": pa.bool_(), "int": pa.int32()}
_PY_TYPES = {float: pa.float32(), int: pa.int32(), str: pa.string()}


def path_exists(path: Optional[str] = None) -> bool:
    if path is None:
        raise ValueError("Directory path is None")
    return os.path.exists(path)


def files_exist(dir_path: Optional[str] = None, files: Optional[List[str]] = None) -> bool:
    """True when dir_path exists and holds every file in `files` (ValueError names the first missing one)."""
    if not path_exists(dir_path):
        raise ValueError(f"Directory {dir_path} doesn't exist")
    for f in files or []:
        if not path_exists(os.path.join(dir_path, f)):
            raise ValueError(f"File {os.path.join(dir_path, f)} doesn't exist in the given fileset")
    return True


def resolve_column_index_from_column_name(column_name, table) -> int:
    for i, name in enumerate(table.column_names):
        if name == column_name:
            return i
    raise ValueError(f"Column {column_name} does not exist in the table")


def get_arrow_type(dtype):
    """Arrow type for a dtype name ('int64', 'double', ...) or a Python type (int, float, str)."""
    if isinstance(dtype, str):
        return _STR_TYPES.get(dtype)
    if isinstance(dtype, type):
        return _PY_TYPES.get(dtype)
    raise ValueError(f"Unsupported dtype {dtype}")
