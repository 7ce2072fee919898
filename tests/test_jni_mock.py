"""The JNI layer (java/src/main/native/cylon_jni.cpp, component J2) compiled and EXECUTED without a
JDK: java/src/test/native/mock_jni/jni.h declares the JNI surface the layer uses and
jni_mock_test.cpp implements JNIEnv over plain C++ objects, then calls every native method of
org.cylonamd.{CylonContext, Table, Row, ArrowTable} the way the Java classes do (predicate select
through Row handles, ArrowTable.fromBuffers, error codes + lastError).  Numbers are checked against
the Python API on the same CSV files.  (The Java classes themselves need javac: not in this image.)"""
import os
import subprocess

import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "tests", "data", "input")
SO = os.path.join(ROOT, "cylon_amd", "libcylon_amd.so")


def _build(tmp_path):
    import torch
    tdir = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    exe = str(tmp_path / "jni_mock_test")
    cmd = ["g++", "-std=c++17", "-O1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-I", os.path.join(ROOT, "java", "src", "test", "native", "mock_jni"),
           os.path.join(ROOT, "java", "src", "main", "native", "cylon_jni.cpp"),
           os.path.join(ROOT, "java", "src", "test", "native", "jni_mock_test.cpp"),
           "-o", exe, SO, "-L", os.path.join(tdir, "lib"), "-Wl,--no-as-needed", "-ltorch", "-ltorch_cpu", "-lc10",
           f"-Wl,-rpath,{os.path.dirname(SO)}", f"-Wl,-rpath,{os.path.join(tdir, 'lib')}"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


@pytest.mark.skipif(not os.path.exists(SO), reason="native core library not built")
@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "java", "src", "main", "native", "cylon_jni.cpp")),
                    reason="java sources not in this snapshot (.gpurunignore leaves ./java off the GPU box)")
def test_jni_layer_through_mock_jnienv(ctx, tmp_path):
    exe = _build(tmp_path)
    a, b = os.path.join(DATA, "csv1_0.csv"), os.path.join(DATA, "csv2_0.csv")
    r = subprocess.run([exe, a, b, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = dict((k, int(v)) for k, v in (line.split() for line in r.stdout.splitlines() if len(line.split()) == 2))
    from cylon_amd.io import read_csv
    ta, tb = read_csv(ctx, a), read_csv(ctx, b)
    da = ta.to_pandas()
    assert got["world"] == 1 and got["rank"] == 0 and got["failures"] == 0
    assert got["rows_a"] == ta.row_count and got["cols_a"] == ta.column_count
    j = ta.join(tb, "inner", "hash", on=[0])
    assert got["join_rows"] == j.row_count and got["join_cols"] == j.column_count
    assert got["outer_rows"] == ta.join(tb, "outer", "sort", on=[0]).row_count
    assert got["union_rows"] == ta.union(tb).row_count
    assert got["project_cols"] == 1
    assert got["merge_rows"] == ta.row_count + tb.row_count
    k0 = da.iloc[:, 0]
    assert got["select_even_rows"] == int((k0.notna() & (k0 % 2 == 0)).sum())
    assert got["select_visited"] == ta.row_count and got["local_refs_left"] == 0
    s = pd.read_csv(tmp_path / "jni_sorted.csv")
    assert s.iloc[:, 0].is_monotonic_increasing and len(s) == ta.row_count
    assert got["buffers_rows"] == 4 and got["buffers_cols"] == 3
    assert got["buffers_nulls"] == 1 and got["buffers_dsum_x10"] == 80 and got["buffers_selected"] == 3
