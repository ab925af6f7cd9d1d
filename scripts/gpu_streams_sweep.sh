#!/bin/bash
# bench line against the number of frames in flight: CONFIG=c2 NS="2 3 4 6" bash scripts/gpu_streams_sweep.sh
set -o pipefail
C=${CONFIG:-c2}
O=gpurun_out/streams_$C
mkdir -p $O
export TMPDIR=/tmp
for n in ${NS:-2 3 4 6}; do
  timeout -k 10 200 python -u bench.py --config $C --steps 200 --warmup 20 --streams $n --no-cpu-baseline \
      --no-kernel-timing > $O/s$n.json 2> $O/s$n.err || exit 1
done
