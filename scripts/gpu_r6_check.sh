#!/bin/bash
# Round 6 checkpoint: the whole GPU suite, smoke, and every config's bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 900 bash scripts/gpu_bench_all.sh ${1:-r6_check}/bench ${2:-nocpu} > $O/bench_all.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    > $O/c4s1.json 2> $O/c4s1.err
echo check-done
