#!/bin/bash
# The whole -m gpu suite, smoke, then the C4 latency run and the C2 driver-command bench.
# usage (via gpurun): bash scripts/gpu_all.sh <tag>
set -e
TAG=${1:-all}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gputests.log" 2>&1 || { tail -40 "$O/gputests.log"; exit 1; }
tail -2 "$O/gputests.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 && cat "$O/smoke.log"
bash scripts/gpu_c4lat.sh "$TAG/c4"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$O/c2.json" 2> "$O/c2.err"
python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2', d['fps'], 'fps', d['value'], 'Mpix/s', d['roofline']['frac'])"
