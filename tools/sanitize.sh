#!/bin/bash
# Host sanitizer runs: CPU only, in this container -- GPU ASan
# is not available on the pool, so device code is never instrumented.
#   bash tools/sanitize.sh [OUTDIR]      (default profiles/r06/sanitize)
# 1. ASan + UBSan builds of the library's HOST code (make -C
#    krylov_robustness_amd/csrc sanitize), the C oracles (make -C oracle
#    sanitize) and the MEX shim + stand-in runtime (make -C tests/mexstub
#    sanitize), all with clang so one sanitizer runtime serves the process;
#    the CPU test suite (-m "not gpu") runs against them (KT_LIB,
#    KT_ORACLE_DIR, KT_MEXSTUB_BUILD) with that runtime preloaded.
# 2. ThreadSanitizer: the host worker pool under concurrent callers
#    (tests/native/pool_stress.cpp, make -C krylov_robustness_amd/csrc tsan).
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$ROOT/profiles/r06/sanitize}
mkdir -p "$OUT"
cd "$ROOT"
make -s -j8 -C krylov_robustness_amd/csrc sanitize tsan > "$OUT/build.log" 2>&1 || { tail -30 "$OUT/build.log"; exit 1; }
make -s -C oracle sanitize >> "$OUT/build.log" 2>&1 || { tail -30 "$OUT/build.log"; exit 1; }
make -s -j8 -C tests/mexstub sanitize >> "$OUT/build.log" 2>&1 || { tail -30 "$OUT/build.log"; exit 1; }
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
SAN=$ROOT/build/sanitize
{
    echo "# ASan + UBSan: CPU suite against build/sanitize/libkrylov_hip.so, oracle/_san, tests/mexstub/_build_san"
    echo "# LD_PRELOAD=$RT"
} > "$OUT/asan_ubsan.log"
# which libraries a test process maps (the sanitized ones, and the ASan runtime)
LD_PRELOAD=$RT KT_LIB=$SAN/libkrylov_hip.so KT_ORACLE_DIR=$ROOT/oracle/_san ASAN_OPTIONS=detect_leaks=0 \
    python -c "
import sys; sys.path.insert(0, '$ROOT')
from krylov_robustness_amd import _lib; _lib.load()
from oracle import slq_ref, mctrace_ref; slq_ref.load(); mctrace_ref.load()
maps = open('/proc/self/maps').read()
for k in ('build/sanitize/libkrylov_hip.so', 'oracle/_san/libslq_ref.so', 'oracle/_san/libmctrace_ref.so', 'libclang_rt.asan'):
    print('mapped', k, k in maps)
    assert k in maps
" >> "$OUT/asan_ubsan.log" 2>&1 || { echo "sanitized libraries not mapped"; tail -5 "$OUT/asan_ubsan.log"; exit 1; }
LD_PRELOAD=$RT KT_LIB=$SAN/libkrylov_hip.so KT_ORACLE_DIR=$ROOT/oracle/_san \
KT_MEXSTUB_BUILD=$ROOT/tests/mexstub/_build_san \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:log_path=$OUT/asan_report \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path=$OUT/ubsan_report \
    timeout 3000 python -m pytest tests -m "not gpu" -q -p no:cacheprovider >> "$OUT/asan_ubsan.log" 2>&1
rc=$?
tail -3 "$OUT/asan_ubsan.log"
echo "# TSan: host worker pool under 4 concurrent callers" > "$OUT/tsan_pool.log"
TSAN_OPTIONS=halt_on_error=1 timeout 600 "$SAN/pool_stress_tsan" >> "$OUT/tsan_pool.log" 2>&1
rt=$?
tail -2 "$OUT/tsan_pool.log"
reports=$(ls "$OUT" | grep -c -E "asan_report|ubsan_report")
echo "sanitizer reports: $reports; pytest rc $rc; tsan rc $rt"
[ $rc -eq 0 ] && [ $rt -eq 0 ] && [ "$reports" -eq 0 ]
