#!/bin/bash
# A wider parity survey than the suite's: the hypothesis tests at SDR_HYP_SCALE times their example
# counts (derandomized, so reproducible), each file under its own limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_survey}
S=${2:-8}
mkdir -p $O
export SDR_HYP_SCALE=$S
timeout -k 10 900 python -u -m pytest tests/test_gpu_sweep.py -m gpu -v --hypothesis-show-statistics -k hypothesis --timeout 800 --timeout-method thread \
    > $O/sweep.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_wls.py -m gpu -v --hypothesis-show-statistics -k hypothesis --timeout 800 --timeout-method thread \
    > $O/wls.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --hypothesis-show-statistics -k two_chain_paths_randomized --timeout 800 --timeout-method thread \
    > $O/parity.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_gpu_adversarial.py -m gpu -v --hypothesis-show-statistics --timeout 800 --timeout-method thread \
    > $O/adversarial.log 2>&1
echo survey-done
