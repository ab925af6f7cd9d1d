#!/bin/bash
# WLS / class-path parity on the GPU, then the C4 single-stream latency and its kernel stats.
# usage (via gpurun): bash scripts/gpu_wls_iter.sh <tag>
set -e
TAG=${1:-wls}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wls.py tests/test_gpu_rectify.py tests/test_gpu_display.py -x -v -s \
  --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
grep "PCR - THOMAS" "$O/tests.log" || true
bash scripts/gpu_c4lat.sh "$TAG/c4"
