#!/bin/bash
# Frames-in-flight sweep for C2 and C4.  usage (via gpurun): bash scripts/gpu_sweep_streams.sh <tag>
set -e
TAG=${1:-sweep}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
for cfg in c2 c4; do
  for ns in 2 3 4 6; do
    timeout -k 10 200 python3 bench.py --config $cfg --streams $ns --steps 150 --warmup 10 --no-cpu-baseline --no-kernel-timing > "$O/$cfg.s$ns.json" 2> "$O/$cfg.s$ns.err"
    python3 -c "import json; d=json.load(open('$O/$cfg.s$ns.json')); print('$cfg', 'streams $ns', d['fps'], 'fps')"
  done
done
