"""Arrow object introspection (reference: python/pycylon/data/arrow_util.pyx)."""
import pyarrow as pa


class ArrowUtil:
    @staticmethod
    def get_array_length(obj) -> int:
        if not isinstance(obj, (pa.Array, pa.ChunkedArray)):
            raise ValueError(f"expected a pyarrow array, got {type(obj)}")
        return len(obj)

    @staticmethod
    def get_array_info(obj):
        """(length, null count, type) of an Arrow array."""
        if not isinstance(obj, (pa.Array, pa.ChunkedArray)):
            raise ValueError(f"expected a pyarrow array, got {type(obj)}")
        return len(obj), obj.null_count, obj.type

    @staticmethod
    def get_table_info(obj):
        """(rows, columns, schema) of an Arrow table."""
        if not isinstance(obj, pa.Table):
            raise ValueError(f"expected a pyarrow table, got {type(obj)}")
        return obj.num_rows, obj.num_columns, obj.schema
