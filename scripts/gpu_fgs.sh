#!/bin/bash
# The sequential FGS (SDR_FGS_THOMAS): WLS parity, then per-launch durations on a scene and a noise guide
# (python scripts/th_trace.py gpurun_out/fgs/prof/fgs_kernel_trace.csv)
set -o pipefail
O=gpurun_out/fgs
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_wls.py \
    > $O/wls_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o fgs -- \
    python -u scripts/fgs_bench.py 50 --thomas-only > $O/fgs_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_noise -o fgs -- \
    python -u scripts/fgs_bench.py 50 --thomas-only --noise-guide > $O/fgs_bench_noise.log 2>&1
