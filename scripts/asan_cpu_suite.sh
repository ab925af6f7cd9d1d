#!/bin/bash
# The CPU test suite under AddressSanitizer + UndefinedBehaviorSanitizer: the oracle
# (oracle/_build_asan, `make -C oracle asan`) and the engine's host code (lib/libsdr-asan.so, device
# code unchanged) built with ROCm's clang, whose ASan runtime is preloaded into python.  Host only:
# GPU sanitizers are not used on this pool.  usage: bash scripts/asan_cpu_suite.sh [pytest args]
set -e
cd "$(dirname "$0")/.."
make -C oracle asan
python -m stereo_depth_ruler_amd.build --host-asan > /dev/null
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export SDR_ORACLE_LIB=$PWD/oracle/_build_asan/liboracle.so
export SDR_TEST_ENGINE_LIB=$PWD/stereo_depth_ruler_amd/lib/libsdr-asan.so
LD_PRELOAD="$RT${LD_PRELOAD:+ $LD_PRELOAD}" python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@"
