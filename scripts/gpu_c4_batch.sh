#!/bin/bash
# C4 frames per launch (--batch) against frames in flight (--streams): "B:S B:S ..." in RUNS
set -o pipefail
O=gpurun_out/c4_batch
mkdir -p $O
export TMPDIR=/tmp
for bs in ${RUNS:-1:6 2:3 2:4 4:2 4:3}; do
  b=${bs%:*}; s=${bs#*:}
  timeout -k 10 200 python -u bench.py --config c4 --batch $b --streams $s --steps $((600 / b)) --warmup 10 \
      --no-cpu-baseline --no-kernel-timing > $O/b${b}s${s}.json 2> $O/b${b}s${s}.err || exit 1
done
