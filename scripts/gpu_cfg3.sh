#!/bin/bash
# Round-3 config measurements: C3 and C5 bench lines (with kernel stats), then C2 quick check.
set -e
TAG=${1:-cfg}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
for c in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$c" -o run -- \
    python3 bench.py --config $c --streams 1 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing > "$O/prof_$c.log" 2>&1
  python3 scripts/kstats.py "$O/prof_$c" | head -6
  timeout -k 10 400 python3 bench.py --config $c --streams 1 --steps 6 --warmup 2 > "$O/bench_$c.json" 2> "$O/bench_$c.err"
  python3 -c "import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', d['fps'], 'fps', d['value'], d['unit'], r['kernel'][:30], r['frac'], r['avg_launch_us'])"
done
