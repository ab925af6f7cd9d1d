#!/bin/bash
# Class path parity (WLS, live loop, display, facade) + C4 latency/profile.
# usage (via gpurun): bash scripts/gpu_class_iter.sh <tag>
set -e
TAG=${1:-cls}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wls.py tests/test_gpu_rectify.py tests/test_gpu_display.py tests/test_gpu_parity.py tests/test_gpu_distributed.py -x -q -s \
  --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
bash scripts/gpu_c4lat.sh "$TAG/c4"
