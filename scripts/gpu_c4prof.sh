#!/bin/bash
# C4 (class path live loop): frames-in-flight sweep and a single-stream kernel profile.
set -e
TAG=${1:-c4prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
for ns in 1 2 3; do
  timeout -k 10 200 python3 bench.py --config c4 --streams $ns --steps 150 --warmup 10 --no-cpu-baseline --no-kernel-timing > "$O/c4.s$ns.json" 2> "$O/c4.s$ns.err"
  python3 -c "import json; d=json.load(open('$O/c4.s$ns.json')); print('c4 streams $ns', d['fps'], 'fps')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 bench.py --config c4 --steps 60 --warmup 10 --no-cpu-baseline --streams 1 --no-kernel-timing > "$O/prof.log" 2>&1
echo prof-done
