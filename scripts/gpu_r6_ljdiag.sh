#!/bin/bash
# k_fgs_lrjob diagnostics: C4 one stream with the product library, without the chain, without the solver's stores
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_ljdiag}
mkdir -p $O
L=$PWD/stereo_depth_ruler_amd/lib
for v in "" ljnochain ljnostore; do
  lib=$L/libsdr.so; [ -n "$v" ] && lib=$L/libsdr-$v.so
  SDR_BENCH_LIB=$lib timeout -k 10 200 python -u bench.py --config c4 --steps 100 --warmup 10 --streams 1 --no-cpu-baseline \
      --no-stream-probe > $O/c4s1_${v:-prod}.json 2> $O/c4s1_${v:-prod}.err || exit 1
done
echo ljdiag-done
