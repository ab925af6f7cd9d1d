#!/bin/bash
# halo ring written lane-contiguous: sweep parity, C3/C5 bench lines, C3 PMC traffic
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_ring}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_configs.py -m gpu -q -x --timeout 240 \
    --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err &&
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_c3_$grp -o run -- \
      python3 bench.py --config c3 --steps 3 --warmup 1 --streams 1 --iso-steps 1 --no-cpu-baseline \
      --no-kernel-timing --no-stream-probe > $O/pmc_c3_$grp.log 2>&1 || exit 1
done
echo ring-done
