"""Shared helpers of the Python examples: device choice and result printing."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def device_from_argv(default: str = "auto") -> str:
    """`--device cpu|cuda:0|auto` (auto: the first GPU when one is visible)."""
    dev = default
    if "--device" in sys.argv:
        dev = sys.argv[sys.argv.index("--device") + 1]
    if dev == "auto":
        dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    return dev


def rows_from_argv(default: int) -> int:
    return int(sys.argv[sys.argv.index("--rows") + 1]) if "--rows" in sys.argv else default


def report(name: str, value) -> None:
    """One "name value" line per result (tests/test_python_examples.py parses them)."""
    # one write per line: ranks share the pipe, and print's separate end="\n" write could interleave
    sys.stdout.write(f"{name} {value}\n")
    sys.stdout.flush()
