#!/bin/bash
# Kernel-trace stats (single stream) of experiment builds: one rocprofv3 run per variant.
# usage (via gpurun): bash scripts/exp_prof.sh <tag> <config> <variant|default> ...
set -e
TAG=$1; CFG=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
for v in "$@"; do
  V=$v; [ "$v" = default ] && V=
  SDR_LIB_VARIANT=$V timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$v" -o run -- \
    python3 bench.py --config "$CFG" --steps 40 --warmup 5 --no-cpu-baseline --no-kernel-timing --streams 1 > "$O/$v.log" 2>&1
  echo "== $v"; python3 scripts/kstats.py "$O/$v" | head -4
done
