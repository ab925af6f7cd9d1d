#!/bin/bash
# C4 at $NS frames in flight, A/B over engine builds: LIBS="base lib/libsdr-x.so ..." (base = libsdr.so)
set -o pipefail
O=gpurun_out/ab_c4
mkdir -p $O
export TMPDIR=/tmp
i=0
for rep in 1 2; do
  for L in ${LIBS:-base}; do
    i=$((i+1))
    if [ "$L" = base ]; then unset SDR_BENCH_LIB; else export SDR_BENCH_LIB=stereo_depth_ruler_amd/$L; fi
    timeout -k 10 200 python -u bench.py --config c4 --steps 300 --warmup 30 --streams ${NS:-6} --no-cpu-baseline \
        --no-kernel-timing > $O/$i.$(basename $L .so).json 2> $O/$i.err || exit 1
  done
done
