#!/usr/bin/env bash
# Build the Java API (J1) and its JNI layer (J2).  Needs a JDK (javac, jni.h) and the built
# native core library cylon_amd/libcylon_amd.so (python setup.py build_ext --inplace); the JNI
# layer links only that library (C ABI), no Python.  Not part of the CI image (no JDK).
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/.." && pwd)
: "${JAVA_HOME:?set JAVA_HOME to a JDK}"
SO="$ROOT/cylon_amd/libcylon_amd.so"
mkdir -p "$HERE/build/classes"
javac -d "$HERE/build/classes" $(find "$HERE/src/main/java" -name '*.java')
g++ -O2 -shared -fPIC -std=c++17 -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" \
    "$HERE/src/main/native/cylon_jni.cpp" "$SO" -Wl,-rpath,"$(dirname "$SO")" -o "$HERE/build/libcylon_jni.so"
jar cf "$HERE/build/cylon_amd.jar" -C "$HERE/build/classes" .
echo "built $HERE/build/cylon_amd.jar and $HERE/build/libcylon_jni.so"
