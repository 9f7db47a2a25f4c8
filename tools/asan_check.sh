#!/bin/bash
# CPU sanitizer run: ASan + UBSan on the host code of libsbo
# (frontier.cpp, polygeom.cpp, the host paths of sbo_api.cpp; GPU code not
# instrumented) and on the oracle, driven by the CPU test suite
# (pytest -m "not gpu").  One ASan runtime (clang's) is preloaded into python.
# Usage: tools/asan_check.sh [pytest args]   -> exit status of pytest
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/safe_bayesian_optimization_amd" -j8 asan 2>&1 | grep -v packed-fp32 || true
make -s -C "$ROOT/oracle" asan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$ROOT"
# detect_leaks=0: python and torch keep allocations for the process lifetime
# (not ours); halt_on_error: any report fails the run
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=97
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1:exitcode=98
SBO_LIB="$ROOT/safe_bayesian_optimization_amd/lib/libsbo_asan.so" ORC_LIB="$ROOT/oracle/liboracle_asan.so" \
LD_PRELOAD="$RT" python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
