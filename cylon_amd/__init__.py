"""cylon_amd: an MI355X-native distributed relational engine with Cylon's capabilities.

Layers (see SURVEY.md §1 for the reference's layer map):
  L0 ctx        CylonContext (torch.distributed / RCCL bootstrap, device ownership)
  L1 net        Communicator over a c10d ProcessGroup (RCCL over xGMI, gloo on CPU)
  L2 data       device-resident Arrow-layout tables (cylon_amd._C.Table)
  L3 kernels    hand-written HIP kernels for gfx950 (hash, partition, scatter, gather,
                radix sort, hash join, merge join, group-by, ...) + C++ CPU twins
  L4 ops        distributed operators (shuffle + local op), in C++
  L5/L6 API     pycylon-compatible Table / DataFrame / CylonEnv
"""
from ._lib import C, CylonError
from .ctx.context import CylonContext
from .data.table import SortOptions, Table
from .net import CommConfig, GlooConfig, MPIConfig, RCCLConfig

__version__ = "0.1.0"

__all__ = ["C", "CylonError", "CylonContext", "Table", "SortOptions", "CommConfig", "GlooConfig", "MPIConfig",
           "RCCLConfig"]
