#!/bin/bash
# A/B on one box: the up sweep's cost-row ring 2 (product) against 3 (libsdr-upring3.so): sweep
# parity with the variant, then C3 and C5 lines alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_upring}
mkdir -p $O
L=$PWD/stereo_depth_ruler_amd/lib
SDR_TEST_ENGINE_LIB=$L/libsdr-upring3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_configs.py \
    -m gpu -q -x --timeout 240 --timeout-method thread > $O/parity.log 2>&1 &&
for rep in 1 2; do
  for v in prod upring3; do
    lib=$L/libsdr.so; [ "$v" != prod ] && lib=$L/libsdr-$v.so
    SDR_BENCH_LIB=$lib timeout -k 10 200 python -u bench.py --config c3 --steps 60 --warmup 6 --no-cpu-baseline \
        --no-stream-probe > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 1
  done
done
echo upring-done
