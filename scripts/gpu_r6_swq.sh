#!/bin/bash
# k_south_wta's deferred per-pixel epilogue: parity suites on the product library, then C2, C4 (one
# stream) and C4 (6 streams) alternating with the previous build (libsdr-base.so) on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_swq}
mkdir -p $O
L=$PWD/stereo_depth_ruler_amd/lib
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adversarial.py tests/test_gpu_configs.py \
    tests/test_gpu_cloud.py tests/test_gpu_speckle.py -m gpu -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
for rep in 1 2; do
  for v in prod base; do
    lib=$L/libsdr.so; [ "$v" != prod ] && lib=$L/libsdr-$v.so
    SDR_BENCH_LIB=$lib timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-stream-probe \
        > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 1
    SDR_BENCH_LIB=$lib timeout -k 10 200 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 \
        --no-cpu-baseline --no-stream-probe > $O/c4s1_${v}_$rep.json 2> $O/c4s1_${v}_$rep.err || exit 1
    SDR_BENCH_LIB=$lib timeout -k 10 200 python -u bench.py --config c4 --steps 200 --warmup 20 \
        --no-cpu-baseline --no-stream-probe --no-kernel-timing > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || exit 1
  done
done
echo swq-done
