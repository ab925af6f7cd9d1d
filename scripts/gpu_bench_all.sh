#!/bin/bash
# Bench lines for every BASELINE config on one GPU (each step under its own time limit).
# usage (via gpurun): bash scripts/gpu_bench_all.sh <tag> [cpu]
set -e
TAG=${1:-ball}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
CPU="--no-cpu-baseline"
[ "$2" = "cpu" ] && CPU=""
timeout -k 10 300 python3 bench.py $CPU > "$O/c2.json" 2> "$O/c2.err"
python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2', d['fps'], 'fps', d['value'], d['roofline']['frac'], (d['cpu_baseline'] or {}).get('value'))"
timeout -k 10 300 python3 bench.py --config c4 --steps 100 --warmup 10 $CPU > "$O/c4.json" 2> "$O/c4.err"
python3 -c "import json; d=json.load(open('$O/c4.json')); print('c4', d['fps'], 'fps', d['value'], d['roofline']['frac'], (d['cpu_baseline'] or {}).get('value'))"
timeout -k 10 300 python3 bench.py --config c3 --steps 6 --warmup 2 --streams 1 --iso-steps 2 $CPU > "$O/c3.json" 2> "$O/c3.err"
python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3', d['fps'], 'fps', d['value'], d['roofline']['frac'], (d['cpu_baseline'] or {}).get('value'))"
timeout -k 10 300 python3 bench.py --config c5 --steps 6 --warmup 2 --streams 1 --iso-steps 2 $CPU > "$O/c5.json" 2> "$O/c5.err"
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['fps'], 'fps', d['value'], d['roofline']['frac'], (d['cpu_baseline'] or {}).get('value'))"
