"""Build the cylon_amd native engine in-tree.

Two stages:
  1. every HIP kernel file (cylon_amd/csrc/cylon/kernels/*.hip) is compiled by
     hipcc for gfx950 (MI355X) into an object file (no torch headers, no
     hipify: the sources are HIP);
  2. the host C++ core + pybind11 bindings are compiled as a torch
     CppExtension and linked with those objects and libamdhip64 into
     cylon_amd/_C*.so.

Usage: python setup.py build_ext --inplace   (or cylon_amd._build.build())
"""
import importlib.util
import os

from setuptools import setup

_spec = importlib.util.spec_from_file_location(
    "cylon_amd_build", os.path.join(os.path.dirname(os.path.abspath(__file__)), "cylon_amd", "_build.py"))
_build = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_build)

hip_objects = _build.compile_hip_objects()

from torch.utils.cpp_extension import BuildExtension, CppExtension  # noqa: E402

# Arrow / Parquet C++ (native Parquet I/O and the Arrow bridge, io/arrow_io.cpp):
# the libraries and headers that ship inside pyarrow, linked by path (the wheel
# has no unversioned .so symlinks) with an rpath to pyarrow's directory.
import pyarrow  # noqa: E402

_PA_DIR = pyarrow.get_library_dirs()[0]
_PA_LIBS = [os.path.join(_PA_DIR, f) for f in sorted(os.listdir(_PA_DIR))
            if f.startswith(("libarrow.so.", "libparquet.so.")) and f.count(".") == 2]

ext = CppExtension(
    name="cylon_amd._C",
    sources=_build.cpp_sources(),
    include_dirs=[_build.CSRC, _build.ROCM_INCLUDE],
    define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
    extra_compile_args=["-O3", "-std=c++17", "-Wno-unused-function"],
    extra_objects=hip_objects + _build.compile_cxx20_objects([pyarrow.get_include()]) + _PA_LIBS,
    library_dirs=[_build.ROCM_LIB],
    libraries=["amdhip64", "rocprofiler-sdk-roctx"],
    extra_link_args=[f"-Wl,-rpath,{_build.ROCM_LIB}", f"-Wl,-rpath,{_PA_DIR}"],
)

setup(
    name="cylon_amd",
    version="0.1.0",
    packages=["cylon_amd"],
    ext_modules=[ext],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
