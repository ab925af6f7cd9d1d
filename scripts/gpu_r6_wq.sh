#!/bin/bash
# the down sweep's deferred per-pixel epilogue: sweep / config / parity tests on the product library,
# then C3 and C5 lines alternating with the previous build (libsdr-base.so) on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_wq}
mkdir -p $O
L=$PWD/stereo_depth_ruler_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q -x \
    --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
for rep in 1 2; do
  for v in prod base; do
    lib=$L/libsdr.so; [ "$v" != prod ] && lib=$L/libsdr-$v.so
    SDR_BENCH_LIB=$lib timeout -k 10 200 python -u bench.py --config c3 --steps 60 --warmup 6 --no-cpu-baseline \
        --no-stream-probe > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 1
    SDR_BENCH_LIB=$lib timeout -k 10 200 python -u bench.py --config c5 --steps 60 --warmup 6 --no-cpu-baseline \
        --no-stream-probe > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 1
  done
done
echo wq-done
