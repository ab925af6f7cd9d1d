#!/bin/bash
# What the driver runs at round end, on one box: the -m gpu suite, smoke(), and the bench command
# (N=1, 20 steps, 5 warmup).  usage (via gpurun): bash scripts/gpu_validate.sh <tag>
set -e
TAG=${1:-val}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$O/gputests.log" 2>&1 || { tail -40 "$O/gputests.log"; exit 1; }
tail -1 "$O/gputests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['fps'], 'fps', d['value'], 'Mpix/s', d['roofline']['frac'])"
