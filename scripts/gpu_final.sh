#!/bin/bash
# Round-end measurement on one box: every BASELINE config's bench line (C2 with the CPU baseline),
# then the C2 rocprofv3 kernel-trace stats (default 3-stream run and single stream) and the
# trace split into the timed and single-stream segments.  Each GPU step has its own time limit.
# usage (via gpurun): bash scripts/gpu_final.sh <tag>
set -e
TAG=${1:-fin}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 bash scripts/gpu_bench_all.sh "$TAG" cpu
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline > "$O/prof.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_s1" -o run -- \
  python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline --streams 1 > "$O/prof_s1.log" 2>&1
python3 scripts/trace_segments.py "$O/prof" --iso 30 --out "$O/segments.md" > /dev/null
python3 scripts/kstats.py "$O/prof_s1"
echo final-done
