"""Communication configs (reference: python/pycylon/net/*.pyx).

`MPIConfig` is kept as a name for source compatibility with pycylon programs,
but on MI355X the transport is torch.distributed: RCCL (backend "nccl" on ROCm)
over xGMI when the ranks own GPUs, gloo on CPU.  Rendezvous uses the torchrun
environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT).
"""
from dataclasses import dataclass, field
from typing import Optional

from .._lib import C

CommType = C.CommType


@dataclass
class CommConfig:
    """Base distributed configuration."""
    backend: Optional[str] = None          # "nccl"(=RCCL) | "gloo" | None -> auto
    init_method: Optional[str] = None      # torch.distributed init_method (default env://)
    rank: Optional[int] = None
    world_size: Optional[int] = None
    device: Optional[str] = None           # "cuda:<i>" | "cpu" | None -> auto
    timeout_s: float = 600.0
    options: dict = field(default_factory=dict)

    def comm_type(self):
        return CommType.RCCL if self.resolved_backend() == "nccl" else CommType.GLOO

    def resolved_backend(self) -> str:
        if self.backend:
            return "nccl" if self.backend in ("nccl", "rccl") else self.backend
        import torch
        return "nccl" if torch.cuda.is_available() else "gloo"


@dataclass
class RCCLConfig(CommConfig):
    """RCCL over xGMI (one process per MI355X)."""
    backend: Optional[str] = "nccl"


@dataclass
class GlooConfig(CommConfig):
    """gloo over TCP (CPU tables / tests)."""
    backend: Optional[str] = "gloo"


@dataclass
class TCPConfig(CommConfig):
    """Native TCP mesh (CommType.TCP, no torch.distributed): the C++ bootstrap
    (CylonContext::InitDistributed) rendezvouses through a c10d TCPStore at
    MASTER_ADDR:MASTER_PORT and connects every rank pair by a socket.  Host tables;
    the reference declares this comm type but never implements it."""
    backend: Optional[str] = "tcp"

    def comm_type(self):
        return CommType.TCP

    def resolved_backend(self) -> str:
        return "tcp"


class MPIConfig(CommConfig):
    """pycylon compatibility alias: selects the default torch.distributed backend."""


__all__ = ["CommConfig", "RCCLConfig", "GlooConfig", "TCPConfig", "MPIConfig", "CommType"]


# ---- point-to-point channel (C4 / P6; reference net/channel.hpp, pycylon/net/txrequest.pyx)
TxRequest = C.TxRequest
ChannelReceiveCallback = C.ChannelReceiveCallback
ChannelSendCallback = C.ChannelSendCallback


class Channel:
    """Polled header+payload message channel between ranks over the context's
    communicator (c10d send/recv: RCCL p2p over xGMI, gloo on CPU).

    channel = Channel(ctx); channel.init(edge, receives, send_ids, rcv_cb, snd_cb)
    channel.send(TxRequest(target, tensor, [h0..h5])); channel.send_fin(TxRequest(target))
    while not channel.is_complete(): channel.progress_sends(); channel.progress_receives()
    """

    def __init__(self, ctx):
        self._ch = C.Channel(ctx._ctx if hasattr(ctx, "_ctx") else ctx)

    def init(self, edge: int, receives, send_ids, receive_callback, send_callback):
        self._ch.init(int(edge), list(receives), list(send_ids), receive_callback, send_callback)

    def send(self, req) -> int:
        return self._ch.send(req)

    def send_fin(self, req) -> int:
        return self._ch.send_fin(req)

    def progress_sends(self):
        self._ch.progress_sends()

    def progress_receives(self):
        self._ch.progress_receives()

    def is_complete(self) -> bool:
        return self._ch.is_complete()

    def close(self):
        self._ch.close()
