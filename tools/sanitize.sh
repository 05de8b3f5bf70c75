#!/bin/bash
# CPU sanitizer runs of the native runtime: ThreadSanitizer over the loader
# ring + concurrent engine, AddressSanitizer+UBSan over the same driver.  Host code only
# (GPU ASan / XNACK are not available on the MI355X pool).
set -e -o pipefail
cd "$(dirname "$0")/.."
OUTDIR=${TMPDIR:-/tmp}/dg_sanitize; mkdir -p $OUTDIR
SRC="csrc/engine/tests/stress_main.cpp csrc/engine/loader.cpp csrc/engine/go_engine.cpp csrc/engine/features.cpp csrc/engine/t7.cpp csrc/engine/sgf.cpp"
for SAN in thread address,undefined; do
  OUT=$OUTDIR/stress_${SAN//,/_}
  g++ -std=c++17 -O1 -g -pthread -fno-omit-frame-pointer -fsanitize=$SAN $SRC -o $OUT
  echo "== -fsanitize=$SAN"
  TSAN_OPTIONS="halt_on_error=1" ASAN_OPTIONS="detect_leaks=1:halt_on_error=1" \
    UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1" timeout 600 $OUT
done
