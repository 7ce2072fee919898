"""In-tree build driver for the native engine (hipcc for gfx950 + torch CppExtension).

The built extension lands at cylon_amd/_C*.so so that it travels with the repo
snapshot to the GPU box (no JIT cache under ~/.cache).
"""
import glob
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
KERNELS = os.path.join(CSRC, "cylon", "kernels")
OBJ_DIR = os.path.join(ROOT, "build", "hip_objs")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ROCM_INCLUDE = os.path.join(ROCM, "include")
ROCM_LIB = os.path.join(ROCM, "lib")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
OFFLOAD_ARCH = os.environ.get("CYLON_OFFLOAD_ARCH", "gfx950")

HIP_FLAGS = [
    f"--offload-arch={OFFLOAD_ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
]


def hip_sources():
    return sorted(glob.glob(os.path.join(KERNELS, "*.hip")))


# sources that need C++20 (the Arrow 25 C++ headers)
CXX20_SOURCES = [os.path.join(CSRC, "cylon", "io", "arrow_io.cpp")]
# the Python extension (pybind11 bindings) - everything else is the native core library
BINDING_SOURCES = [os.path.join(CSRC, "bindings.cpp"), os.path.join(CSRC, "bindings_ops.cpp")]
CORE_LIB = os.path.join(PKG, "libcylon_amd.so")


def core_sources():
    srcs = [os.path.join(CSRC, "capi.cpp")]
    for sub in ("cylon", "cylon/net", "cylon/ops", "cylon/ctx", "cylon/io", "cylon/kernels", "cylon/indexing"):
        srcs += sorted(glob.glob(os.path.join(CSRC, sub, "*.cpp")))
    return srcs


def binding_sources():
    return [os.path.relpath(s, ROOT) for s in BINDING_SOURCES]


def _torch_flags():
    import torch
    from torch.utils.cpp_extension import include_paths, library_paths
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return include_paths(), library_paths()[0], [f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]


def _arrow_paths():
    import pyarrow
    d = pyarrow.get_library_dirs()[0]
    libs = [os.path.join(d, f) for f in sorted(os.listdir(d))
            if f.startswith(("libarrow.so.", "libparquet.so.")) and f.count(".") == 2]
    return pyarrow.get_include(), d, libs


def _compile_cxx(src, digest, incs, defs):
    std = "-std=c++20" if src in CXX20_SOURCES else "-std=c++17"
    flags = [std, "-O3", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-Wall", "-Wno-unused-function",
             "-Wno-sign-compare"] + defs
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    obj = os.path.join(OBJ_DIR, "core", os.path.splitext(rel)[0] + ".o")
    stamp = obj + ".stamp"
    with open(src, "rb") as f:
        key = hashlib.sha1(f.read() + digest.encode() + " ".join(flags + incs).encode()).hexdigest()
    if os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == key:
                return obj, False
    cmd = ["g++"] + flags + [x for i in incs for x in ("-I", i)] + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"g++ failed for {src}:\n{r.stderr[-6000:]}")
    with open(stamp, "w") as f:
        f.write(key)
    return obj, True


def build_core(jobs=None):
    """Native core library cylon_amd/libcylon_amd.so: C++ engine + C ABI + HIP kernels.

    Links libtorch / c10 (tensors, allocator, c10d process groups), the HIP
    runtime and the Arrow / Parquet C++ libraries shipped with pyarrow; no
    Python.  C++ programs (examples/cpp) and the Python extension link it."""
    hip_objs = compile_hip_objects(jobs)
    os.makedirs(os.path.join(OBJ_DIR, "core"), exist_ok=True)
    digest = _headers_digest()
    tinc, tlib, tdefs = _torch_flags()
    ainc, adir, alibs = _arrow_paths()
    incs = [CSRC, ROCM_INCLUDE] + tinc + [ainc]
    jobs = jobs or min(8, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        res = list(ex.map(lambda s: _compile_cxx(s, digest, incs, tdefs), core_sources()))
    objs = [o for o, _ in res]
    inputs = objs + hip_objs
    if os.path.exists(CORE_LIB) and not any(c for _, c in res) and \
            all(os.path.getmtime(o) <= os.path.getmtime(CORE_LIB) for o in inputs):
        return CORE_LIB
    cmd = (["g++", "-shared", "-o", CORE_LIB, "-Wl,-soname,libcylon_amd.so"] + inputs +
           ["-L", tlib, "-Wl,--no-as-needed", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lc10", "-lc10_hip",
            "-Wl,--as-needed", "-L", ROCM_LIB, "-lamdhip64", "-lrocprofiler-sdk-roctx"] + alibs +
           [f"-Wl,-rpath,{tlib}", f"-Wl,-rpath,{ROCM_LIB}", f"-Wl,-rpath,{adir}"])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"linking {CORE_LIB} failed:\n{r.stderr[-6000:]}")
    return CORE_LIB


def _headers_digest():
    h = hashlib.sha1()
    for p in sorted(glob.glob(os.path.join(CSRC, "**", "*.hpp"), recursive=True) +
                    glob.glob(os.path.join(CSRC, "**", "*.inc"), recursive=True)):
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _compile_one(src, digest):
    name = os.path.splitext(os.path.basename(src))[0]
    obj = os.path.join(OBJ_DIR, name + ".o")
    stamp = obj + ".stamp"
    with open(src, "rb") as f:
        key = hashlib.sha1(f.read() + digest.encode() + " ".join(HIP_FLAGS).encode()).hexdigest()
    if os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == key:
                return obj
    cmd = [HIPCC] + HIP_FLAGS + ["-I", CSRC, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    with open(stamp, "w") as f:
        f.write(key)
    return obj


def compile_hip_objects(jobs=None):
    os.makedirs(OBJ_DIR, exist_ok=True)
    digest = _headers_digest()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        return list(ex.map(lambda s: _compile_one(s, digest), hip_sources()))


def build(verbose=False):
    """Compile every HIP kernel for gfx950 and the extension, in-tree."""
    env = dict(os.environ)
    env.setdefault("MAX_JOBS", str(min(8, os.cpu_count() or 4)))
    env.setdefault("PYTORCH_ROCM_ARCH", OFFLOAD_ARCH)
    cmd = [sys.executable, "setup.py", "build_ext", "--inplace"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=not verbose, text=True)
    if r.returncode != 0:
        out = (r.stdout or "")[-4000:] + (r.stderr or "")[-8000:]
        raise RuntimeError(f"native build failed:\n{out}")


if __name__ == "__main__":
    build(verbose=True)
