#!/bin/bash
# round 5: packed sequential-FGS passes; sweep shape A/B (two libraries per kbench: 32-frame scratch)
set -o pipefail
O=gpurun_out/r5e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wls.py \
    > $O/wls_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 \
    --no-cpu-baseline > $O/bench_c4s1.json 2> $O/bench_c4s1.err &&
timeout -k 10 300 python -u scripts/kbench.py --libs stereo_depth_ruler_amd/lib/libsdr.so \
    stereo_depth_ruler_amd/lib/libsdr-dnmh1.so --config c3b32 --rounds 2 --iters 2 > $O/kbench_dnmh1.log 2>&1 &&
timeout -k 10 300 python -u scripts/kbench.py --libs stereo_depth_ruler_amd/lib/libsdr.so \
    stereo_depth_ruler_amd/lib/libsdr-upmo1.so --config c3b32 --rounds 2 --iters 2 > $O/kbench_upmo1.log 2>&1 &&
timeout -k 10 300 python -u scripts/kbench.py --libs stereo_depth_ruler_amd/lib/libsdr.so \
    stereo_depth_ruler_amd/lib/libsdr-dnmo2.so --config c3b32 --rounds 2 --iters 2 > $O/kbench_dnmo2.log 2>&1
