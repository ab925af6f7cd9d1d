#!/bin/bash
# Single-stream per-kernel HIP-event times of experiment builds, interleaved rounds.
# usage (via gpurun): bash scripts/exp_iso.sh <tag> <config> <variant|default> ...
set -e
TAG=$1; CFG=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
for round in 1 2; do
  for v in "$@"; do
    V=$v; [ "$v" = default ] && V=
    SDR_LIB_VARIANT=$V timeout -k 10 120 python3 bench.py --config "$CFG" --steps 100 --warmup 10 --no-cpu-baseline --streams 1 > "$O/$v.r$round.json" 2> "$O/$v.r$round.err"
    python3 - "$O/$v.r$round.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
print(f"{sys.argv[2]:8s} fps={d.get('fps')} " + " ".join(f"{n}={v['avg_us']:.0f}" for n, v in k.items()))
PY
  done
done
