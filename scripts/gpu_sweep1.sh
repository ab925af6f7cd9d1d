#!/bin/bash
# First run of the MODE_HH row sweeps: their own parity tests under a short limit, then the suite.
set -e
TAG=${1:-sw}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 150 python3 -u -m pytest tests/test_gpu_sweep.py -x -v --timeout 100 --timeout-method thread > "$O/sweep.log" 2>&1 || { tail -40 "$O/sweep.log"; exit 1; }
tail -3 "$O/sweep.log"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gputests.log" 2>&1 || { tail -40 "$O/gputests.log"; exit 1; }
tail -1 "$O/gputests.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof1" -o run -- \
  python3 bench.py --config c3 --streams 1 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing > "$O/prof1.log" 2>&1
python3 scripts/kstats.py "$O/prof1"
timeout -k 10 300 python3 bench.py --config c3 --steps 6 --warmup 2 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['fps'], 'fps', d['value'], d['unit'], d['roofline']['frac'])"
