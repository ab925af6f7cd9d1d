#!/bin/bash
# round 5: LDS-staged sequential FGS passes: parity, then per-kernel durations (scene and noise guides)
set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_wls.py \
    > $O/wls_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o fgs -- \
    python -u scripts/fgs_bench.py 50 --thomas-only > $O/fgs_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_noise -o fgs -- \
    python -u scripts/fgs_bench.py 50 --thomas-only --noise-guide > $O/fgs_bench_noise.log 2>&1
