#!/bin/bash
# C5 with the voxel stage one step behind across streams: config / cloud parity, then C5's default
# line (3 streams), one stream, and C2 (unchanged path) for scale
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_c5pipe}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_cloud.py -m gpu -q -x --timeout 240 \
    --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-stream-probe > $O/c5.json 2> $O/c5.err &&
timeout -k 10 300 python -u bench.py --config c5 --streams 1 --steps 30 --warmup 4 --no-cpu-baseline --no-stream-probe \
    > $O/c5s1.json 2> $O/c5s1.err &&
timeout -k 10 300 python -u bench.py --config c5 --streams 2 --no-cpu-baseline --no-stream-probe > $O/c5s2.json 2> $O/c5s2.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-stream-probe > $O/c2.json 2> $O/c2.err
echo c5pipe-done
