#!/bin/bash
# FGS parity (both solvers) + FGS kernel timing.  usage (via gpurun): bash scripts/gpu_fgs_iter.sh <tag>
set -e
TAG=${1:-fgs}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wls.py -x -q -s --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"; grep "PCR - THOMAS" "$O/tests.log" || true
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 scripts/fgs_bench.py 50 > "$O/prof.log" 2>&1
python3 scripts/kstats.py "$O/prof"
