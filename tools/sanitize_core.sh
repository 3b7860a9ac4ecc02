#!/bin/bash
# Host sanitizer run of the C++ codec core: csrc/core/*.cpp + the driver
# tools/native/sanitize_core.cpp under AddressSanitizer + UndefinedBehaviorSanitizer (CPU
# only; the GPU kernels are checked against this golden model instead).
#   tools/sanitize_core.sh [outdir]      -> builds <outdir>/sanitize_core and runs it
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$ROOT/build/sanitize}
mkdir -p "$OUT"
CXX=${CXX:-g++}
$CXX -O1 -g -std=c++17 -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -pthread -I"$ROOT/csrc/include" "$ROOT"/csrc/core/*.cpp "$ROOT/tools/native/sanitize_core.cpp" -o "$OUT/sanitize_core"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 "$OUT/sanitize_core"
