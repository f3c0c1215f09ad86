#!/usr/bin/env bash
# Build the host runtime (netsdb_amd/csrc/runtime) into a standalone self-test with sanitizers and run it:
#   * ASan + UBSan: memory errors / undefined behaviour in the parser, allocator, page files, buffer pool
#   * TSan: data races between buffer-manager users and the native WorkerQueue (page prefetch / flush)
# Host code only (GPU sanitizers are not available on the MI355X pool).  Usage: scripts/sanitize_native.sh [outdir]
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
OUT="${1:-${TMPDIR:-/tmp}/nsdb_sanitize}"
mkdir -p "$OUT"
RT="$ROOT/netsdb_amd/csrc/runtime"
SRCS=("$RT/tcap_parser.cpp" "$RT/storage.cpp" "$RT/work.cpp" "$ROOT/tests/native/runtime_selftest.cpp")
CXX="${CXX:-g++}"

"$CXX" -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -I"$RT" "${SRCS[@]}" -o "$OUT/selftest_asan" -lpthread
mkdir -p "$OUT/asan_data"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/selftest_asan" "$OUT/asan_data"

"$CXX" -std=c++17 -O1 -g -fsanitize=thread -I"$RT" "${SRCS[@]}" -o "$OUT/selftest_tsan" -lpthread
mkdir -p "$OUT/tsan_data"
TSAN_OPTIONS=halt_on_error=1 "$OUT/selftest_tsan" "$OUT/tsan_data"
echo "sanitizers clean"
