#!/usr/bin/env bash
# Host-code sanitizer run (SURVEY.md §5 "race detection / sanitizers"): every C++ source of
# the native core (operators, CPU kernel twins, CSV / Parquet I/O, registry, C ABI) is rebuilt
# with AddressSanitizer + UndefinedBehaviorSanitizer and linked with the C++ examples; the
# HIP kernel objects are linked unchanged (no GPU sanitizer on this pool).  The examples
# then run on the CPU engine.  Usage: bash tools/sanitize_host.sh [out_dir]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/cylon_asan}
mkdir -p "$OUT/obj"
TORCH=$(python -c "import torch, os; print(os.path.dirname(torch.__file__))")
ABI=$(python -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
PA_INC=$(python -c "import pyarrow; print(pyarrow.get_include())")
PA_DIR=$(python -c "import pyarrow; print(pyarrow.get_library_dirs()[0])")
SAN="-fsanitize=address,undefined -fno-sanitize=vptr -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
# (vptr checks off: they fire on shared_ptr code inlined into uninstrumented system libraries at exit)
INC="-I $ROOT/cylon_amd/csrc -I /opt/rocm/include -I $TORCH/include -I $TORCH/include/torch/csrc/api/include -I $PA_INC"
DEFS="-D_GLIBCXX_USE_CXX11_ABI=$ABI -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1"
SRCS=$(python - "$ROOT" <<'PY'
import importlib.util, os, sys
root = sys.argv[1]
spec = importlib.util.spec_from_file_location("b", os.path.join(root, "cylon_amd", "_build.py"))
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
print(" ".join(b.core_sources()))
PY
)
pids=()
for src in $SRCS; do
  std=-std=c++17; [[ "$src" == *arrow_io.cpp ]] && std=-std=c++20
  obj="$OUT/obj/$(echo "${src#$ROOT/}" | tr '/' '_').o"
  g++ $std -O1 -g -fPIC $SAN $DEFS $INC -c "$src" -o "$obj" &
  pids+=($!)
  if (( ${#pids[@]} >= 8 )); then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
done
wait
HIP_OBJS=$(ls "$ROOT"/build/hip_objs/*.o)
for ex in relational_example registry_example; do
  g++ -std=c++17 -O1 -g $SAN $DEFS $INC "$ROOT/examples/cpp/$ex.cpp" "$OUT"/obj/*.o $HIP_OBJS -o "$OUT/$ex" \
      -L "$TORCH/lib" -Wl,--no-as-needed -ltorch -ltorch_cpu -ltorch_hip -lc10 -lc10_hip -Wl,--as-needed \
      -L /opt/rocm/lib -lamdhip64 -lrocprofiler-sdk-roctx "$PA_DIR"/libarrow.so.2500 "$PA_DIR"/libparquet.so.2500 \
      -Wl,-rpath,"$TORCH/lib" -Wl,-rpath,/opt/rocm/lib -Wl,-rpath,"$PA_DIR"
done
mkdir -p "$OUT/run"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1
for ex in relational_example registry_example; do
  "$OUT/$ex" cpu "$ROOT/tests/data/input/csv1_0.csv" "$ROOT/tests/data/input/csv2_0.csv" "$OUT/run" > "$OUT/$ex.out"
  echo "$ex: clean ($(wc -l < "$OUT/$ex.out") result lines)"
done
