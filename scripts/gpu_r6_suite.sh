#!/bin/bash
# the GPU suite and smoke on the current tree, then the C5 and C2 default lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c5 > $O/c5.json 2> $O/c5.err &&
timeout -k 10 300 python -u bench.py > $O/c2.json 2> $O/c2.err
echo suite-done
