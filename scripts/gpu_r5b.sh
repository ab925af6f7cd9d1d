#!/bin/bash
# round 5: the 16-lane sweeps (up pass + down pass with the WTA): parity first, then speed
set -o pipefail
O=gpurun_out/r5b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sweep.py \
    tests/test_gpu_configs.py > $O/sweep_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/kbench.py --libs stereo_depth_ruler_amd/lib/libsdr.so \
    stereo_depth_ruler_amd/lib/libsdr-r3.so --config c3 --rounds 3 --iters 5 > $O/kbench_c3.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c3 --steps 6 --warmup 2 --streams 1 --iso-steps 3 \
    --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err
