#!/bin/bash
# Class-path parity tests, then the C4 bench line.  usage (via gpurun): bash scripts/gpu_c4.sh <tag>
set -e
TAG=${1:-c4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gputests.log" 2>&1
tail -2 "$O/gputests.log"
timeout -k 10 300 python3 bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline > "$O/c4.json" 2> "$O/c4.err"
python3 -c "import json; d=json.load(open('$O/c4.json')); print('c4', d['fps'], 'fps', d['value'], d['roofline']['frac'])"
