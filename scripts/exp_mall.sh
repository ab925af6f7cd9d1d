#!/bin/bash
# Experiment: does keeping the cost volume in the Infinity Cache pay?  Path-cost stores plain vs
# non-temporal, one path launch vs one launch per direction; single stream, isolated timings.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-mall}
mkdir -p "$O"
for cfg in "0 0" "1 0" "0 1" "1 1"; do
  set -- $cfg
  SDR_EXP_NT=$1 SDR_EXP_SEQ=$2 timeout -k 10 120 python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline --streams 1 > "$O/b_nt$1_seq$2.json" 2> "$O/b_nt$1_seq$2.err"
  python3 -c "import json,sys; d=json.load(open('$O/b_nt$1_seq$2.json')); k=d['kernels']; print('nt=$1 seq=$2 fps', d['fps'], {n: v['avg_us'] for n, v in k.items()})"
done
