#!/bin/bash
# Round 6 last check on the final build: the GPU suite, smoke, C2's default line, C4 on one stream and
# its default line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/c2.json 2> $O/c2.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline > $O/c4s1.json 2> $O/c4s1.err &&
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/c4.json 2> $O/c4.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4s1 -o run -- \
    python3 bench.py --config c4 --steps 60 --warmup 10 --streams 1 --no-cpu-baseline --no-stream-probe \
    > $O/prof_c4s1.json 2> $O/prof_c4s1.err
echo final3-done
