#!/bin/bash
# A/B on one box: the sweeps' tile -> XCD mapping (SDR_SWEEP_XCD 0: linear, 1: a frame's tiles on one XCD)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_xcd_ab}
mkdir -p $O
for rep in 1 2; do
  for x in ${XS:-0 1}; do
    SDR_SWEEP_XCD=$x timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline --no-stream-probe \
        > $O/c3_x${x}_$rep.json 2> $O/c3_x${x}_$rep.err || exit 1
    SDR_SWEEP_XCD=$x timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline --no-stream-probe \
        > $O/c5_x${x}_$rep.json 2> $O/c5_x${x}_$rep.err || exit 1
  done
done
echo ab-done
