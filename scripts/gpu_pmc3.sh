#!/bin/bash
# Round-3 PMC traffic passes for C3 (the MODE_HH row sweeps) and C2 (fused LR check), one
# counter group per run; then the same commands' kernel stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in c3 c2; do
  O=gpurun_out/pmc3_$c
  mkdir -p "$O"
  steps=6; [ $c = c3 ] && steps=2
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$O/p$i" -o run -- \
      python3 bench.py --config $c --steps $steps --warmup 1 --no-cpu-baseline --no-kernel-timing --streams 1 > "$O/p$i.log" 2>&1
  done
done
echo pmc-done
