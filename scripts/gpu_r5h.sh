#!/bin/bash
# round 5: sequential FGS pass A/B (library variants), per-kernel durations
set -o pipefail
O=gpurun_out/r5h
mkdir -p $O
export TMPDIR=/tmp
for v in "" thnochain thnorows thlpb32 thlpb64; do
  lib=stereo_depth_ruler_amd/lib/libsdr${v:+-$v}.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v:-base} -o fgs -- \
      python -u scripts/fgs_bench.py 30 --lib $lib --thomas-only > $O/fgs_${v:-base}.log 2>&1 || exit 1
done
