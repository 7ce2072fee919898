"""Multi-process test harness: N ranks as N local processes over gloo (the
analogue of the reference's `mpirun --oversubscribe -np N`, cpp/test/CMakeLists.txt:45-49)."""
import os
import socket
import sys
import traceback

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, fn, args, q, device="cpu", env=None):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    os.environ.update(env or {})
    try:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        if root not in sys.path:
            sys.path.insert(0, root)
        from cylon_amd import CylonContext, GlooConfig, RCCLConfig, TCPConfig
        # CYLON_TEST_COMM=tcp: the native bootstrap + TCP mesh instead of torch.distributed gloo;
        # CYLON_TEST_COMM=rccl: torch.distributed nccl (RCCL), one rank per GPU
        comm = os.environ.get("CYLON_TEST_COMM")
        cfg = TCPConfig() if comm == "tcp" else (RCCLConfig() if comm == "rccl" else GlooConfig())
        ctx = CylonContext(config=cfg, distributed=True, device=device)
        try:
            res = fn(ctx, *args)
        finally:
            ctx.finalize()
        q.put((rank, True, res))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, False, traceback.format_exc()))


def run_distributed(fn, world: int, *args, timeout: float = 240.0, device: str = "cpu", env=None):
    """Run fn(ctx, *args) on `world` gloo ranks; returns the list of per-rank results.

    device="cuda:0" puts every rank's tables on the (single) GPU of the box while the
    collectives go over gloo: the device kernels of the multi-rank paths run for real."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q, device, env)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, ok, res = q.get(timeout=timeout)
            if not ok:
                raise AssertionError(f"rank {rank} failed:\n{res}")
            results[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]
