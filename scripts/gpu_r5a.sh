#!/bin/bash
# round 5, first box: the new tests, the k_south_wta A/B against the round-3 build, bench lines
set -o pipefail
O=gpurun_out/r5a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/kbench.py --libs stereo_depth_ruler_amd/lib/libsdr.so \
    stereo_depth_ruler_amd/lib/libsdr-r3.so --config c2 --rounds 5 > $O/kbench_c2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c3 --steps 6 --warmup 2 --streams 1 --iso-steps 3 \
    --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 \
    --no-cpu-baseline > $O/bench_c4s1.json 2> $O/bench_c4s1.err &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
