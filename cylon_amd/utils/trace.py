"""Phase timers / counters front-end (native: cylon/trace.cpp).

Phases are ROCTx ranges (shown by `rocprofv3 --marker-trace`) plus HIP-event timings
per operator phase: join.build.*, join.probe.*, join.materialize, shuffle.partition,
shuffle.exchange, sort.indices, groupby.group_ids, groupby.aggregate."""
import contextlib
from typing import Dict, Tuple

from .._lib import C


def enable_tracing(on: bool = True):
    C.trace_enable(bool(on))


def phases() -> Dict[str, Tuple[float, int]]:
    """{phase: (total_ms, calls)} - resolves (synchronises) pending GPU events."""
    return dict(C.trace_phases())


def counters() -> Dict[str, int]:
    return dict(C.trace_counters())


def reset_tracing():
    C.trace_reset()


def report() -> str:
    rows = sorted(phases().items(), key=lambda kv: -kv[1][0])
    lines = [f"{'phase':28s} {'total_ms':>10s} {'calls':>6s}"]
    lines += [f"{k:28s} {v[0]:10.3f} {v[1]:6d}" for k, v in rows]
    for k, v in sorted(counters().items()):
        lines.append(f"{k:28s} {v:>17d}")
    return "\n".join(lines)


@contextlib.contextmanager
def traced():
    prev = C.trace_enabled()
    C.trace_enable(True)
    C.trace_reset()
    try:
        yield
    finally:
        C.trace_enable(prev)
