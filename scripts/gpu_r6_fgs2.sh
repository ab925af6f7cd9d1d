#!/bin/bash
# k_fgs_lr iteration: WLS parity, the stamps of its passes, C4 one stream
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_fgs2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wls.py \
    > $O/wls_tests.log 2>&1 &&
timeout -k 10 120 python -u scripts/lr_stamps.py stereo_depth_ruler_amd/lib/libsdr-thstamps.so > $O/lr_stamps.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    --no-stream-probe > $O/c4s1.json 2> $O/c4s1.err
echo fgs2-done
