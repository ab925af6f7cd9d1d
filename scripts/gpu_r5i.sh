#!/bin/bash
# round 5: per-chunk stamps of the sequential FGS (diagnostic libraries)
set -o pipefail
O=gpurun_out/r5i
mkdir -p $O
for v in thstamps; do
  SDR_TH_STAMP_LAUNCH=21 timeout -k 10 120 python -u scripts/th_stamps.py stereo_depth_ruler_amd/lib/libsdr-$v.so \
      > $O/stamps_${v}_21.txt 2>&1 || exit 1
done
