"""Benchmark helpers (reference: python/pycylon/util/benchutils.py:19-45).

Device-aware: the timed region is closed by a device synchronise so GPU work
launched inside it is counted."""
import time


def time_conversion(time_ns: int, time_type: str = "ms") -> float:
    if time_type is None:
        raise ValueError("Time Type cannot be None")
    scale = {"ms": 1e6, "us": 1e3, "s": 1e9, "ns": 1.0}
    if time_type not in scale:
        raise ValueError(f"unknown time type {time_type}")
    return time_ns / scale[time_type]


def _sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:  # pragma: no cover
        pass


def benchmark_with_repetitions(repetitions: int = 10, time_type: str = "ms"):
    """Decorator: returns (average time per call, last return value)."""

    def wrap(f):
        def wrapped_f(*args, **kwargs):
            _sync()
            t1 = time.time_ns()
            rets = None
            for _ in range(repetitions):
                rets = f(*args, **kwargs)
            _sync()
            t2 = time.time_ns()
            return time_conversion(t2 - t1, time_type) / float(repetitions), rets

        return wrapped_f

    return wrap


# pycylon spelling
def benchmark_with_repitions(repititions: int = 10, time_type: str = "ms"):
    return benchmark_with_repetitions(repititions, time_type)
