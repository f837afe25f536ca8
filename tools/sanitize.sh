#!/bin/bash
# Build and run the native runtime self-test under ASan+UBSan and under TSan (host code only).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$ROOT/build/sanitize}
mkdir -p "$OUT"
SRC="$ROOT/csrc/tests/runtime_selftest.cpp $ROOT/csrc/runtime/store.cpp $ROOT/csrc/runtime/reducer.cpp $ROOT/csrc/runtime/host_ring.cpp $ROOT/csrc/runtime/watchdog.cpp"
CXX=${CXX:-g++}
$CXX -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -I"$ROOT/csrc/runtime" $SRC -o "$OUT/selftest_asan" -lpthread
$CXX -std=c++17 -O1 -g -fsanitize=thread -I"$ROOT/csrc/runtime" $SRC -o "$OUT/selftest_tsan" -lpthread
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/selftest_asan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/selftest_tsan"
echo "sanitizers clean"
