#!/bin/bash
# Quick GPU iteration: full parity suite, then kernel-trace stats of a short bench.
# usage (via gpurun): bash scripts/gpu_quick.sh <tag> [pytest -k expr]
set -e
TAG=${1:-q}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
if [ -n "$2" ]; then
  timeout -k 10 600 python3 -m pytest tests -m gpu -x -q -k "$2" > "$O/gputests.log" 2>&1 || { tail -30 "$O/gputests.log"; exit 1; }
else
  timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > "$O/gputests.log" 2>&1 || { tail -30 "$O/gputests.log"; exit 1; }
fi
tail -1 "$O/gputests.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-kernel-timing > "$O/prof.log" 2>&1
grep '^{' "$O/prof.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fps", d["fps"], "ms", d["ms_per_step"])'
python3 scripts/kstats.py "$O/prof"
