#!/bin/bash
# Builds the native host runtime (log, offsets, ingest, HTTP front end) with the two stress
# drivers under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer, and
# runs them (host code only: GPU sanitizers are not available on the MI355X pool).
#   runtime_stress.cpp:  producers / partition readers / offsets / ingest parser
#   runtime_stress2.cpp: append_fill writers + frame and text readers across segment rolls,
#                        the HTTP server under concurrent, pipelined, chunked and abusive
#                        clients, oryx_topn_prep from several threads, the native thread pool,
#                        the HTTPS server (OpenSSL) under concurrent and abusive TLS clients,
#                        and the JKS / PKCS#12 keystore readers (threads, damaged files)
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-/tmp/oryx_sanitize}
mkdir -p "$OUT"
RT="csrc/runtime/oryx_log.cpp csrc/runtime/oryx_ingest.cpp csrc/runtime/oryx_http.cpp csrc/runtime/oryx_hostbuf.cpp csrc/runtime/oryx_keystore.cpp"
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
  # the same key as a PKCS#12 and a JKS keystore (password oryxpass) for the keystore readers
  if [ -n "$TLS" ] && openssl pkcs12 -export -in "$OUT/cert.pem" -inkey "$OUT/key.pem" \
      -out "$OUT/store.p12" -passout pass:oryxpass > /dev/null 2>&1 &&
      python3 -c "
import subprocess, sys
sys.path.insert(0, '.')
from tests.test_serving_keystore import _write_jks
out = sys.argv[1]
k = subprocess.run(['openssl', 'pkcs8', '-topk8', '-nocrypt', '-in', out + '/key.pem',
                    '-outform', 'DER'], capture_output=True, check=True).stdout
c = subprocess.run(['openssl', 'x509', '-in', out + '/cert.pem', '-outform', 'DER'],
                   capture_output=True, check=True).stdout
_write_jks(out + '/store.jks', 'oryxpass', 'oryxtest', k, [c])
" "$OUT"; then
    TLS="$TLS $OUT/store.p12 $OUT/store.jks"
  fi
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
