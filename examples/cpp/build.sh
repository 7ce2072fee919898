#!/usr/bin/env bash
# Build the C++ examples against the native core library (run `python setup.py build_ext --inplace` first).
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
TORCH=$(python -c "import torch, os; print(os.path.dirname(torch.__file__))")
ABI=$(python -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
# (not "build/": that name is excluded from the GPU-box snapshots)
OUT=${1:-$HERE/bin}
mkdir -p "$OUT"
for src in "$HERE"/*.cpp; do
  exe="$OUT/$(basename "${src%.cpp}")"
  g++ -std=c++17 -O2 -D_GLIBCXX_USE_CXX11_ABI=$ABI -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 \
      -I "$ROOT/cylon_amd/csrc" -I /opt/rocm/include -I "$TORCH/include" -I "$TORCH/include/torch/csrc/api/include" \
      "$src" -o "$exe" "$ROOT/cylon_amd/libcylon_amd.so" -L "$TORCH/lib" -Wl,--no-as-needed -ltorch -ltorch_cpu -lc10 \
      -Wl,-rpath,'$ORIGIN/../../../cylon_amd' -Wl,-rpath,"$ROOT/cylon_amd" -Wl,-rpath,"$TORCH/lib"
  echo "built $exe"
done
