"""CylonContext (reference: python/pycylon/ctx/context.pyx:29-149,
cpp/src/cylon/ctx/cylon_context.cpp).

One process per GPU: a distributed context initialises torch.distributed
(RCCL over xGMI for GPU ranks, gloo for CPU ranks) from the torchrun
environment and hands the ProcessGroup to the native communicator.  The
context also fixes the device its tables live on (cuda:<LOCAL_RANK>).

Config keys (add_config/get_config):
  compute_engine : "arrow" | "numpy" | "device"  (elementwise engine, pycylon parity)
  device         : overrides the table device
"""
import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

from .._lib import C
from ..net import CommConfig


def _default_device(distributed: bool) -> str:
    if torch.cuda.is_available():
        lr = int(os.environ.get("LOCAL_RANK", "0")) if distributed else torch.cuda.current_device()
        return f"cuda:{lr % max(torch.cuda.device_count(), 1)}"
    return "cpu"


def _rccl_options():
    """ProcessGroupNCCL options: RCCL's stream at high priority.  HIP maps streams onto a few
    hardware queues; a normal-priority comm stream can land on the compute stream's queue, and
    then every posted all-to-all runs serialised with the operator kernels instead of under them
    (forced world-1 shuffle trace: 0 of 50 ms overlapped by default, 68 of 74 ms at high
    priority; profiles/rccl_queue_r03.txt)."""
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return opts


class CylonContext:
    def __init__(self, config: Optional[object] = None, distributed: Optional[bool] = None,
                 device: Optional[str] = None):
        if distributed is None:
            distributed = config is not None
        self._owns_pg = False
        if isinstance(config, str):
            config = CommConfig(backend=config)
        if isinstance(config, dict):
            config = CommConfig(**config)
        if distributed:
            cfg = config if isinstance(config, CommConfig) else CommConfig()
            backend = cfg.resolved_backend()
            if backend == "tcp":  # native bootstrap + TCP mesh, no torch.distributed
                self._ctx = C.Context.init_native("tcp", -1 if cfg.rank is None else cfg.rank,
                                                  -1 if cfg.world_size is None else cfg.world_size,
                                                  device or cfg.device or "cpu", float(cfg.timeout_s))
                self._finalized = False
                return
            dev = device or cfg.device or (_default_device(True) if backend == "nccl" else "cpu")
            if dev.startswith("cuda"):
                torch.cuda.set_device(torch.device(dev))
            if not dist.is_initialized():
                kw = {}
                if cfg.rank is not None:
                    kw["rank"] = cfg.rank
                if cfg.world_size is not None:
                    kw["world_size"] = cfg.world_size
                if backend == "nccl" and dev.startswith("cuda"):
                    kw["device_id"] = torch.device(dev)
                    kw["pg_options"] = _rccl_options()
                dist.init_process_group(backend=backend, init_method=cfg.init_method or "env://",
                                        timeout=datetime.timedelta(seconds=cfg.timeout_s), **kw)
                self._owns_pg = True
            pg = dist.group.WORLD
            self._ctx = C.Context.init_distributed(pg, dist.get_backend(pg), dev)
        else:
            dev = device or _default_device(False)
            self._ctx = C.Context.init_local(dev)
        self._finalized = False

    @classmethod
    def _wrap(cls, native):
        obj = cls.__new__(cls)
        obj._ctx = native
        obj._owns_pg = False
        obj._finalized = False
        return obj

    # ---- pycylon API -----------------------------------------------------
    def get_rank(self) -> int:
        return self._ctx.get_rank()

    def get_world_size(self) -> int:
        return self._ctx.get_world_size()

    def get_neighbours(self, include_self: bool = False):
        return self._ctx.get_neighbours(include_self)

    def get_next_sequence(self) -> int:
        return self._ctx.get_next_sequence()

    def is_distributed(self) -> bool:
        return self._ctx.is_distributed()

    def get_comm_type(self):
        return self._ctx.get_comm_type()

    def barrier(self):
        self._ctx.barrier()

    def finalize(self):
        if self._finalized:
            return
        self._finalized = True
        self._ctx.finalize()
        if self._owns_pg and dist.is_initialized():
            dist.destroy_process_group()

    def add_config(self, key: str, value: str):
        self._ctx.add_config(key, str(value))

    def get_config(self, key: str, default: str = ""):
        return self._ctx.get_config(key, default)

    # ---- MI355X additions --------------------------------------------------
    @property
    def device(self) -> str:
        return self.get_config("device") or self._ctx.device()

    @property
    def on_gpu(self) -> bool:
        return self.device.startswith("cuda")

    def memory_stats(self) -> dict:
        pool = self.memory_pool()
        return {"bytes_allocated": self._ctx.bytes_allocated(), "max_memory": self._ctx.max_memory(),
                "pool_backend": pool.backend_name(), "pool_bytes_allocated": pool.bytes_allocated(),
                "pool_max_memory": pool.max_memory()}

    def memory_pool(self):
        """The context's MemoryPool (C2; reference ctx/memory_pool.hpp): HBM via the HIP caching
        allocator on a GPU context, aligned host memory otherwise."""
        return self._ctx.memory_pool()

    def set_memory_pool(self, pool) -> None:
        self._ctx.set_memory_pool(pool)

    def allreduce(self, tensor: torch.Tensor, op: str = "sum") -> torch.Tensor:
        ops = {"sum": 0, "min": 1, "max": 2, "prod": 3}
        return self._ctx.allreduce(tensor, ops[op])

    def allgather(self, tensor: torch.Tensor) -> torch.Tensor:
        return self._ctx.allgather(tensor)

    def __repr__(self):
        return (f"CylonContext(rank={self.get_rank()}, world={self.get_world_size()}, "
                f"device={self.device}, comm={self.get_comm_type()})")
