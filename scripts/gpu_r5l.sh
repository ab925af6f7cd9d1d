#!/bin/bash
# round 5: WLS parity + C4 single-stream bench (per-kernel times)
set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_wls.py \
    > $O/wls_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    > $O/bench_c4s1.json 2> $O/bench_c4s1.err
