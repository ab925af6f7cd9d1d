#!/bin/bash
# A/B of experiment builds (lib/libsdr-<variant>.so) in ONE process session, interleaved rounds.
# usage (via gpurun): bash scripts/exp_variants.sh <tag> <config> <variant|default> ...
set -e
TAG=$1; CFG=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
for round in 1 2; do
  for v in "$@"; do
    V=$v; [ "$v" = default ] && V=
    for ns in 3 1; do
      SDR_LIB_VARIANT=$V timeout -k 10 120 python3 bench.py --config "$CFG" --steps 200 --warmup 20 --no-cpu-baseline --streams $ns $EXTRA > "$O/$v.s$ns.r$round.json" 2> "$O/$v.s$ns.r$round.err"
      python3 - "$O/$v.s$ns.r$round.json" "$v" "$ns" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels") or {}
ks = " ".join(f"{n}={v['avg_us']:.0f}" for n, v in k.items() if n in ("k_cost", "k_paths", "k_wta_lr"))
print(f"{sys.argv[2]:8s} streams={sys.argv[3]} fps={d.get('fps')} {ks}")
PY
    done
  done
done
