#!/bin/bash
# round 5: sequential FGS (THOMAS, now the default) with precomputed coefficients; sweep shape A/B
set -o pipefail
O=gpurun_out/r5d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wls.py \
    > $O/wls_tests.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 \
    --no-cpu-baseline > $O/bench_c4s1.json 2> $O/bench_c4s1.err &&
timeout -k 10 400 python -u scripts/kbench.py --libs stereo_depth_ruler_amd/lib/libsdr.so \
    stereo_depth_ruler_amd/lib/libsdr-dnmh1.so stereo_depth_ruler_amd/lib/libsdr-upmo1.so \
    stereo_depth_ruler_amd/lib/libsdr-dnmo2.so --config c3b32 --rounds 3 --iters 2 > $O/kbench_c3b32.log 2>&1
