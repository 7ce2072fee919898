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

ext = CppExtension(
    name="cylon_amd._C",
    sources=_build.cpp_sources(),
    include_dirs=[_build.CSRC, _build.ROCM_INCLUDE],
    define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
    extra_compile_args=["-O3", "-std=c++17", "-Wno-unused-function"],
    extra_objects=hip_objects,
    library_dirs=[_build.ROCM_LIB],
    libraries=["amdhip64", "rocprofiler-sdk-roctx"],
    extra_link_args=[f"-Wl,-rpath,{_build.ROCM_LIB}"],
)

setup(
    name="cylon_amd",
    version="0.1.0",
    packages=["cylon_amd"],
    ext_modules=[ext],
    cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
)
