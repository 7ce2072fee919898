"""Build the cylon_amd native engine in-tree.

Two artefacts:
  1. cylon_amd/libcylon_amd.so - the native core library (C++ engine, C ABI,
     every HIP kernel compiled by hipcc for gfx950 / MI355X; links libtorch /
     c10, the HIP runtime and the Arrow / Parquet C++ libraries from pyarrow;
     no Python).  Built by cylon_amd/_build.py with hipcc + g++.  C++ programs
     link it directly (examples/cpp).
  2. cylon_amd/_C*.so - the pybind11 bindings (torch CppExtension) over the
     core library (rpath $ORIGIN).

Usage: python setup.py build_ext --inplace   (or cylon_amd._build.build())
"""
import importlib.util
import os

from setuptools import setup

_spec = importlib.util.spec_from_file_location(
    "cylon_amd_build", os.path.join(os.path.dirname(os.path.abspath(__file__)), "cylon_amd", "_build.py"))
_build = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_build)

core_lib = _build.build_core()

from torch.utils.cpp_extension import BuildExtension, CppExtension  # noqa: E402

ext = CppExtension(
    name="cylon_amd._C",
    sources=_build.binding_sources(),
    include_dirs=[_build.CSRC, _build.ROCM_INCLUDE, _build._arrow_paths()[0]],
    define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
    extra_compile_args=["-O3", "-std=c++17", "-Wno-unused-function"],
    extra_objects=[core_lib],
    library_dirs=[_build.ROCM_LIB],
    libraries=["amdhip64"],
    extra_link_args=["-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{_build.ROCM_LIB}"],
)

setup(
    name="cylon_amd",
    version="0.1.0",
    packages=["cylon_amd"],
    ext_modules=[ext],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
