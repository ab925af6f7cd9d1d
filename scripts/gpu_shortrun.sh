#!/bin/bash
# The driver's bench command (20 steps, 5 warmup) against longer runs, on one box, after the parity
# suite.  usage (via gpurun): bash scripts/gpu_shortrun.sh <tag>
set -e
TAG=${1:-sr}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gputests.log" 2>&1 || { tail -40 "$O/gputests.log"; exit 1; }
tail -1 "$O/gputests.log"
f() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], "fps", d["fps"], "Mpix/s", d["value"], "ms", d["ms_per_step"])' "$1"; }
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/drv$i.json" 2> "$O/drv$i.err"; f "$O/drv$i.json"
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > "$O/nkt.json" 2> "$O/nkt.err"; f "$O/nkt.json"
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-kernel-timing > "$O/long.json" 2> "$O/long.err"; f "$O/long.json"
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > "$O/longkt.json" 2> "$O/longkt.err"; f "$O/longkt.json"
