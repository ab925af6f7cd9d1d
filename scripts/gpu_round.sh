#!/bin/bash
# One GPU session: parity suite -> bench line -> kernel-trace stats (default and single-stream)
# -> PMC passes (single-stream).  usage (via gpurun): bash scripts/gpu_round.sh <tag> [skip-tests]
# Every GPU step has its own time limit; the first failure ends the script (set -e).
set -e
TAG=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > "$O/gputests.log" 2>&1
  tail -3 "$O/gputests.log"
fi
timeout -k 10 300 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline > "$O/prof.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_s1" -o run -- \
  python3 bench.py --steps 60 --warmup 10 --no-cpu-baseline --streams 1 > "$O/prof_s1.log" 2>&1
python3 scripts/trace_segments.py "$O/prof" --iso 30 --out "$O/segments.md" > /dev/null
echo prof-done
timeout -k 10 900 bash scripts/pmc_profile.sh "$O/pmc"
