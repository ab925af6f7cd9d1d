#!/bin/bash
# Pooled scratch (sdr::scratch_alloc): the GPU suite, then C5's bench line and its kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_pool}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
    python3 bench.py --config c5 --steps 6 --warmup 2 --streams 1 --iso-steps 2 --no-cpu-baseline \
    --no-stream-probe > $O/prof_c5.json 2> $O/prof_c5.err
echo pool-done
