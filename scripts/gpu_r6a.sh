#!/bin/bash
# Round 6, first GPU pass: the round's new tests (stream lifetime, status count, pcd_write geometry,
# all reciprocal exponents), then C2 and C4 bench lines with the new roofline fields.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_streams.py tests/test_gpu_sweep.py::test_sweep_timeout_reported_once_unsynchronised \
    tests/test_gpu_sweep.py::test_sweep_timeout_reported_by_next_call \
    tests/test_gpu_cloud.py::test_pcd_write_pipeline tests/test_gpu_wls.py::test_fgs_reciprocal_exact_every_mantissa \
    > $O/tests_new.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 > $O/c2.json 2> $O/c2.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    > $O/c4s1.json 2> $O/c4s1.err
echo r6a-done
