#!/bin/bash
# One build->measure iteration on the GPU box: parity suite (or a -k subset), single-stream bench
# with per-kernel HIP-event times, default bench, kernel-trace stats.  Every GPU step has its own
# time limit and the first failure ends the script.
# usage (via gpurun): bash scripts/gpu_iter.sh <tag> [pytest -k expr | none] [bench --config]
set -e
TAG=${1:-it}
K=${2:-}
CFG=${3:-c2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
if [ "$K" != "none" ]; then
  ARGS=(tests -m gpu -x -q --timeout 120 --timeout-method thread)
  [ -n "$K" ] && ARGS+=(-k "$K")
  timeout -k 10 600 python3 -u -m pytest "${ARGS[@]}" > "$O/gputests.log" 2>&1 || { tail -40 "$O/gputests.log"; exit 1; }
  tail -1 "$O/gputests.log"
fi
summ() {
  python3 - "$1" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "fps", d.get("fps"), "Mpix/s", d["value"], "ms", d["ms_per_step"])
for k, v in (d.get("kernels") or {}).items():
    print(f"  {k:10s} {v['avg_us']:9.2f} us x{v['launches']}")
EOF
}
timeout -k 10 300 python3 bench.py --config "$CFG" --steps 100 --warmup 10 --no-cpu-baseline --streams 1 > "$O/s1.json" 2> "$O/s1.err"
summ "$O/s1.json"
timeout -k 10 300 python3 bench.py --config "$CFG" --steps 200 --warmup 20 --no-cpu-baseline --no-kernel-timing > "$O/s3.json" 2> "$O/s3.err"
summ "$O/s3.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
  python3 bench.py --config "$CFG" --steps 60 --warmup 10 --no-cpu-baseline --no-kernel-timing --streams 1 > "$O/prof.log" 2>&1
python3 scripts/kstats.py "$O/prof"
