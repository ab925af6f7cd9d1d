#!/bin/bash
# C4 (class path live loop) single-frame latency: one stream, one frame in flight, as the
# reference's loop calls it (stereo_displayer.cpp:145-198), plus the rocprofv3 kernel stats of the
# same single-stream command.  usage (via gpurun): bash scripts/gpu_c4lat.sh <tag>
set -e
TAG=${1:-c4lat}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 200 python3 bench.py --config c4 --streams 1 --steps 200 --warmup 20 --no-cpu-baseline > "$O/c4.s1.json" 2> "$O/c4.s1.err"
python3 -c "import json; d=json.load(open('$O/c4.s1.json')); print('c4 streams 1', d['fps'], 'fps', d['ms_per_step'], 'ms/frame')"
timeout -k 10 200 python3 bench.py --config c4 --streams 3 --steps 200 --warmup 20 --no-cpu-baseline --no-kernel-timing > "$O/c4.s3.json" 2> "$O/c4.s3.err"
python3 -c "import json; d=json.load(open('$O/c4.s3.json')); print('c4 streams 3', d['fps'], 'fps', d['ms_per_step'], 'ms/step')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline --streams 1 --no-kernel-timing > "$O/prof.log" 2>&1
python3 scripts/kstats.py "$O/prof"
