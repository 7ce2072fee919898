"""cylon_amd.ctx: runtime context and memory pools (reference cpp/src/cylon/ctx)."""
from .._lib import C


def host_memory_pool():
    """64-byte aligned host MemoryPool."""
    return C.host_memory_pool()


def device_memory_pool(device: str = "cuda:0"):
    """HBM MemoryPool over the HIP caching allocator of `device`."""
    return C.device_memory_pool(device)
