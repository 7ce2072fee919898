"""cylon_amd: an MI355X-native distributed relational engine with Cylon's capabilities.

Layers (see SURVEY.md §1 for the reference's layer map):
  L0 ctx        CylonContext (torch.distributed / RCCL bootstrap, device ownership)
  L1 net        Communicator over a c10d ProcessGroup (RCCL over xGMI, gloo on CPU)
  L2 data       device-resident Arrow-layout tables (cylon_amd._C.Table)
  L3 kernels    hand-written HIP kernels for gfx950 (hash, partition, scatter, gather,
                radix sort, hash join, merge join, group-by, ...) + C++ CPU twins
  L4 ops        distributed operators (shuffle + local op), in C++
  L5/L6 API     pycylon-compatible Table / DataFrame / CylonEnv / Series
"""
from ._lib import C, CylonError
from .common import Code, JoinAlgorithm, JoinConfig, JoinType, Status
from .ctx.context import CylonContext
from .data.aggregates import AggregationOp
from .data.table import SortOptions, Table
from .frame import CylonEnv, DataFrame
from .indexing.index import IndexingSchema
from .io import CSVReadOptions, CSVWriteOptions, read_csv
from .net import CommConfig, GlooConfig, MPIConfig, RCCLConfig, TCPConfig
from .series import Series

Column = C.Column      # pycylon.data.column.Column
DataType = C.DataType  # pycylon.data.data_type.DataType
from .types import (binary, bool, date32, date64, decimal, double, duration, extension, fixed_sized_binary,  # noqa
                    fixed_sized_list, float, half_float, int8, int16, int32, int64, interval, list, string, time32,
                    time64, timestamp, uint8, uint16, uint32, uint64)

__version__ = "0.1.0"

__all__ = ["C", "CylonError", "CylonContext", "Table", "DataFrame", "CylonEnv", "Series", "SortOptions",
           "JoinConfig", "JoinType", "JoinAlgorithm", "Status", "Code", "AggregationOp", "IndexingSchema",
           "CommConfig", "GlooConfig", "MPIConfig", "RCCLConfig", "TCPConfig", "Column", "DataType", "read_csv",
           "CSVReadOptions", "CSVWriteOptions"]
