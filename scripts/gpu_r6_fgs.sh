#!/bin/bash
# Round 6: the line-resident FGS pass (k_fgs_lr) -- WLS parity, the class-path frame tests, then
# C4 on one stream with the new pass and with the round-5 pass (SDR_FGS_LR=0) for the A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_fgs}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wls.py \
    > $O/wls_tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rectify.py \
    tests/test_gpu_parity.py -k "class or live_loop" > $O/live_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    --no-stream-probe > $O/c4s1.json 2> $O/c4s1.err &&
SDR_FGS_LR=0 timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 \
    --no-cpu-baseline --no-stream-probe > $O/c4s1_th.json 2> $O/c4s1_th.err
echo fgs-done
