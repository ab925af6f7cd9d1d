#!/bin/bash
# Round measurement of every BASELINE config: bench lines (with the CPU baseline), single-stream
# kernel stats, and the HBM-traffic PMC passes for C4 and C5.
# usage (via gpurun): bash scripts/gpu_measure_configs.sh <tag>
set -e
TAG=${1:-meas}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
bash scripts/gpu_bench_all.sh "$TAG/bench" cpu
for c in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$c" -o run -- \
    python3 bench.py --config $c --steps 4 --warmup 1 --streams 1 --no-cpu-baseline --no-kernel-timing > "$O/prof_$c.log" 2>&1
  python3 scripts/kstats.py "$O/prof_$c" | head -8
done
for c in c4 c5; do
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$O/pmc_$c/p$i" -o run -- \
      python3 bench.py --config $c --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-kernel-timing > "$O/pmc_$c.p$i.log" 2>&1
  done
done
echo measure-done
