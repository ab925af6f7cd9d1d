#!/bin/bash
# voxel grid scratch: the cloud tests, the host phases (libsdr-vtime.so, SDR_VOXEL_TIMING) inside
# C5's bench, then C5's bench line on the product library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_vtime}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cloud.py -m gpu -q -x --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1 &&
SDR_BENCH_LIB=$PWD/stereo_depth_ruler_amd/lib/libsdr-vtime.so timeout -k 10 300 python -u bench.py --config c5 \
    --steps 6 --warmup 2 --no-cpu-baseline --no-stream-probe --no-kernel-timing > $O/c5_vtime.json 2> $O/c5_vtime.err &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
echo vtime-done
