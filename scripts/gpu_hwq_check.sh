#!/bin/bash
# C4 / C2 at a few stream counts with 8 hardware queues a process instead of HIP's default 4
set -o pipefail
O=gpurun_out/hwq
mkdir -p $O
export TMPDIR=/tmp
run() {  # name hwq config streams
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 python -u bench.py --config $3 --steps 200 --warmup 20 --streams $4 \
      --no-cpu-baseline --no-kernel-timing > $O/$1.json 2> $O/$1.err
}
run c4_q8_s3 8 c4 3 && run c4_q8_s6 8 c4 6 && run c4_q8_s8 8 c4 8 && run c4_q4_s3 4 c4 3 && run c2_q8_s3 8 c2 3
