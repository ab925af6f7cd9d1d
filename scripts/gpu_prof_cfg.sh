#!/bin/bash
# rocprofv3 kernel-trace stats of one bench config.  usage: bash scripts/gpu_prof_cfg.sh <tag> <config> [extra bench args]
set -e
TAG=${1:-pc}; CFG=${2:-c2}; shift 2 || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 bench.py --config $CFG --no-cpu-baseline --no-kernel-timing "$@" > "$O/prof.log" 2>&1
grep '^{' "$O/prof.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fps", d["fps"], "ms", d["ms_per_step"])'
python3 scripts/kstats.py "$O/prof"
