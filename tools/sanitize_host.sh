#!/bin/bash
# Host-code sanitizer run (SURVEY §5 "race detection / sanitizers"): AddressSanitizer +
# UndefinedBehaviorSanitizer on the C-ABI library's host code (csrc/polyproc.cpp -- the
# DataProcessor restatement -- and the host side of uampath.hip) and on the C oracle, then the
# CPU tests that drive that code.  CPU only: -fsanitize goes to the host compilation alone
# (-Xarch_host), device code is built as usual and never runs here.  Both libraries use
# clang's ASan runtime, preloaded into the (uninstrumented) python.
#   usage: bash tools/sanitize_host.sh [pytest args]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/san
LLVM=/opt/rocm/lib/llvm/bin
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer"
$LLVM/clang -O1 -g -std=c99 -fPIC -shared -ffp-contract=off $SAN -o "$OUT/liboracle.so" \
    "$ROOT/oracle/uam_oracle.c" -lm
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 \
    -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
    -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer \
    -o "$OUT/libuampath.so" "$ROOT/uam_path_planning_amd/csrc/uampath.hip" \
    "$ROOT/uam_path_planning_amd/csrc/polyproc.cpp" "$ROOT/uam_path_planning_amd/csrc/tiles.cpp" \
    -lz
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$ROOT"
LD_PRELOAD=$RT${LD_PRELOAD:+:$LD_PRELOAD} \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:verify_asan_link_order=0 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
UAM_LIB_PATH=$OUT/libuampath.so UAM_ORACLE_LIB=$OUT/liboracle.so \
python -m pytest -x -q -p no:cacheprovider -m "not gpu" \
    tests/test_polygons_cpu.py tests/test_oracle_golden.py tests/test_refine_cpu.py \
    tests/test_crs_cpu.py tests/test_host_cpu.py tests/test_map_generation_cpu.py "$@"
