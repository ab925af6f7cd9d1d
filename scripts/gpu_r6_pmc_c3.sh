#!/bin/bash
# C3 HBM PMC passes (FETCH_SIZE / WRITE_SIZE, one a run) under the environment given
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_pmc_c3}
mkdir -p $O
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_c3_$grp -o run -- \
      python3 bench.py --config c3 --steps 3 --warmup 1 --streams 1 --iso-steps 1 --no-cpu-baseline \
      --no-kernel-timing --no-stream-probe > $O/pmc_c3_$grp.log 2>&1 || exit 1
done
echo pmc-done
