"""Utilities (reference: python/pycylon/util/*): benchmarking helpers, data loading and
mini-batching (zero-copy to torch on the device), synthetic data generation, tracing,
memory statistics, checkpointing and DLPack interop."""
from .benchutils import benchmark_with_repitions, benchmark_with_repetitions, time_conversion
from .data import DataLoader, DistributedDataLoader, LocalDataLoader, MiniBatcher, Partition
from .datagen import generate_numeric_csv, random_table
from .misc import files_exist, get_arrow_type, path_exists, resolve_column_index_from_column_name
from .trace import counters, enable_tracing, phases, report, reset_tracing, traced

__all__ = ["files_exist", "get_arrow_type", "path_exists", "resolve_column_index_from_column_name", "benchmark_with_repitions", "benchmark_with_repetitions", "time_conversion", "DataLoader",
           "LocalDataLoader", "DistributedDataLoader", "MiniBatcher", "Partition", "generate_numeric_csv",
           "random_table", "enable_tracing", "phases", "counters", "report", "reset_tracing", "traced"]
