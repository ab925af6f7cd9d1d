#!/bin/bash
# Experiment: frames in flight (streams) x path-cost store policy on C2.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-streams}
mkdir -p "$O"
for cfg in "2 0" "2 1" "3 0" "3 1" "4 1"; do
  set -- $cfg
  SDR_EXP_NT=$2 timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-kernel-timing --streams $1 > "$O/s$1_nt$2.json" 2> "$O/s$1_nt$2.err"
  python3 -c "import json; d=json.load(open('$O/s$1_nt$2.json')); print('streams=$1 nt=$2 fps', d['fps'])"
done
