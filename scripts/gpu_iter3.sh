#!/bin/bash
# Round-3 iteration: GPU parity suite (or a -k subset), C2 single-stream kernel stats, C2 bench.
# usage (via gpurun): bash scripts/gpu_iter3.sh <tag> [pytest -k expr] [config]
set -e
TAG=${1:-it}
CFG=${3:-c2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" > "$O/gputests.log" 2>&1 || { tail -40 "$O/gputests.log"; exit 1; }
tail -1 "$O/gputests.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof1" -o run -- \
  python3 bench.py --config "$CFG" --streams 1 --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-timing > "$O/prof1.log" 2>&1
python3 scripts/kstats.py "$O/prof1"
timeout -k 10 300 python3 bench.py --config "$CFG" --steps 200 --warmup 20 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['fps'], 'fps', d['value'], d['unit'], d['roofline']['frac'])"
