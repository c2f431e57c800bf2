#!/bin/bash
# Builds the native host runtime (log, offsets, ingest) with the stress driver under
# AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer, and runs both
# (host code only: GPU sanitizers are not available on the MI355X pool).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-/tmp/oryx_sanitize}
mkdir -p "$OUT"
SRCS="csrc/runtime/oryx_log.cpp csrc/runtime/oryx_ingest.cpp csrc/runtime/tests/runtime_stress.cpp"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -pthread -fsanitize=address,undefined \
    -fno-sanitize-recover=undefined -o "$OUT/stress_asan" $SRCS -lz
g++ -std=c++17 -O1 -g -pthread -fsanitize=thread -o "$OUT/stress_tsan" $SRCS -lz
rm -rf "$OUT/log_asan" "$OUT/log_tsan"
ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 "$OUT/stress_asan" "$OUT/log_asan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/stress_tsan" "$OUT/log_tsan"
echo "sanitizers clean"
