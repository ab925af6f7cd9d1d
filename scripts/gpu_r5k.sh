#!/bin/bash
# round 5: full GPU suite on the new sequential FGS, smoke, C4 single-stream and default bench lines
set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    > $O/bench_c4s1.json 2> $O/bench_c4s1.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --no-cpu-baseline \
    > $O/bench_c4.json 2> $O/bench_c4.err
