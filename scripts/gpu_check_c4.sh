#!/bin/bash
# after a class-path change: the GPU suite, smoke, and the C4 line on one stream and at its default 6
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/check_c4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    > $O/c4s1.json 2> $O/c4s1.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 300 --warmup 30 --no-cpu-baseline --no-kernel-timing \
    > $O/c4s6a.json 2> $O/c4s6a.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 300 --warmup 30 --no-cpu-baseline --no-kernel-timing \
    > $O/c4s6b.json 2> $O/c4s6b.err
