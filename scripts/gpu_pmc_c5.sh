#!/bin/bash
# C5 PMC traffic passes (FETCH_SIZE, WRITE_SIZE: one counter group per run) over the row-sweep
# pipeline, then the same command's single-stream kernel stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc3_c5
mkdir -p "$O"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$O/p$i" -o run -- \
    python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --streams 1 > "$O/p$i.log" 2>&1
done
echo pmc-done
