#!/bin/bash
# Builds the native host runtime (log, offsets, ingest, HTTP front end) with the two stress
# drivers under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer, and
# runs them (host code only: GPU sanitizers are not available on the MI355X pool).
#   runtime_stress.cpp:  producers / partition readers / offsets / ingest parser
#   runtime_stress2.cpp: append_fill writers + frame and text readers across segment rolls,
#                        the HTTP server under concurrent, pipelined, chunked and abusive
#                        clients, oryx_topn_prep from several threads, the native thread pool,
#                        and the HTTPS server (OpenSSL) under concurrent and abusive TLS clients
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-/tmp/oryx_sanitize}
mkdir -p "$OUT"
RT="csrc/runtime/oryx_log.cpp csrc/runtime/oryx_ingest.cpp csrc/runtime/oryx_http.cpp csrc/runtime/oryx_hostbuf.cpp"
LIBS="-lz -lssl -lcrypto"
ASAN="-std=c++17 -O1 -g -fno-omit-frame-pointer -pthread -fsanitize=address,undefined -fno-sanitize-recover=undefined"
TSAN="-std=c++17 -O1 -g -pthread -fsanitize=thread"
for prog in runtime_stress runtime_stress2; do
  g++ $ASAN -o "$OUT/${prog}_asan" $RT csrc/runtime/tests/$prog.cpp $LIBS &
  g++ $TSAN -o "$OUT/${prog}_tsan" $RT csrc/runtime/tests/$prog.cpp $LIBS &
done
wait
# a throwaway certificate for the HTTPS part of runtime_stress2
TLS=""
if command -v openssl > /dev/null; then
  openssl req -x509 -newkey rsa:2048 -nodes -keyout "$OUT/key.pem" -out "$OUT/cert.pem" \
    -days 2 -subj /CN=127.0.0.1 > /dev/null 2>&1 && TLS="$OUT/cert.pem $OUT/key.pem"
fi
for prog in runtime_stress runtime_stress2; do
  rm -rf "$OUT/${prog}_log_asan" "$OUT/${prog}_log_tsan"
  mkdir -p "$OUT/${prog}_log_asan" "$OUT/${prog}_log_tsan"
  extra=""
  [ "$prog" = runtime_stress2 ] && extra="$TLS"
  echo "== $prog (ASan + UBSan)"
  ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 "$OUT/${prog}_asan" "$OUT/${prog}_log_asan" $extra
  echo "== $prog (TSan)"
  TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/${prog}_tsan" "$OUT/${prog}_log_tsan" $extra
done
echo "sanitizers clean"
