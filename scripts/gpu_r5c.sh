#!/bin/bash
# round 5: the full GPU suite on the 16-lane sweeps, C3 bench + rocprof stats
set -o pipefail
O=gpurun_out/r5c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c3 --steps 6 --warmup 2 --streams 1 --iso-steps 3 \
    --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 -- python -u bench.py --config c3 --steps 4 \
    --warmup 1 --streams 1 --iso-steps 2 --no-cpu-baseline --no-stream-probe > $O/prof_c3.json 2> $O/prof_c3.err &&
timeout -k 10 300 python -u scripts/kbench.py --libs stereo_depth_ruler_amd/lib/libsdr.so \
    stereo_depth_ruler_amd/lib/libsdr-r3.so --config c5b8 --rounds 3 --iters 3 > $O/kbench_c5.log 2>&1
