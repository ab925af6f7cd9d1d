#!/bin/bash
# GPU parity suite, then single-stream and 3-stream A/B of experiment builds.
# usage (via gpurun): bash scripts/gpu_ab.sh <tag> <config> <variant|default> ...
set -e
TAG=$1; CFG=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gputests.log" 2>&1 || { tail -30 "$O/gputests.log"; exit 1; }
tail -1 "$O/gputests.log"
bash scripts/exp_iso.sh "$TAG/iso" "$CFG" "$@"
for v in "$@"; do
  V=$v; [ "$v" = default ] && V=
  SDR_LIB_VARIANT=$V timeout -k 10 120 python3 bench.py --config "$CFG" --steps 200 --warmup 20 --no-cpu-baseline --no-kernel-timing > "$O/$v.s3.json" 2> "$O/$v.s3.err"
  python3 -c "import json; d=json.load(open('$O/$v.s3.json')); print('$v', 'streams 3', d['fps'], 'fps')"
done
