"""Loader of the native engine (cylon_amd/_C*.so, built in-tree by _build.py).

The native module is mandatory: every operator runs in C++ (HIP kernels on
MI355X, C++ twins on CPU).  There is no Python fallback, so a missing build
fails loudly here.
"""
import torch  # noqa: F401  (loads libtorch / libc10 for the extension)

try:
    from . import _C as C  # type: ignore
except ImportError as e:  # pragma: no cover - exercised only without a build
    raise ImportError(
        "cylon_amd native extension is not built; run `python setup.py build_ext --inplace` "
        "(or cylon_amd._build.build())"
    ) from e

CylonError = C.CylonError

__all__ = ["C", "CylonError"]
