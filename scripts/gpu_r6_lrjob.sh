#!/bin/bash
# k_fgs_lrjob (the FGS coefficient jobs the k_fgs_lr way): WLS / class-path parity, then C4 on one
# stream with the jobs on k_fgs_lrjob and on k_fgs_th (SDR_FGS_LRJOB=0), and C4's default line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_lrjob}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wls.py tests/test_gpu_rectify.py tests/test_gpu_parity.py tests/test_gpu_display.py tests/test_gpu_configs.py -m gpu -q -x \
    --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline --no-stream-probe \
    > $O/c4s1_lrjob.json 2> $O/c4s1_lrjob.err &&
SDR_FGS_LRJOB=0 timeout -k 10 200 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    --no-stream-probe > $O/c4s1_th.json 2> $O/c4s1_th.err &&
timeout -k 10 200 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline --no-stream-probe \
    > $O/c4s1_lrjob2.json 2> $O/c4s1_lrjob2.err &&
timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --no-stream-probe > $O/c4.json 2> $O/c4.err
echo lrjob-done
