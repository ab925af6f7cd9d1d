#!/bin/bash
# A/B on one box: the batched MODE_HH sweeps' frames in flight (SDR_SWEEP_SLOTS caps nslots), C3
# and C5 at their default 3 streams, so that the other streams' kernels can use the CUs left free
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_slots}
mkdir -p $O
for cap in 0 6 4 3; do
  SDR_SWEEP_SLOTS=$cap timeout -k 10 200 python -u bench.py --config c3 --steps 60 --warmup 6 --no-cpu-baseline \
      --no-stream-probe > $O/c3_s$cap.json 2> $O/c3_s$cap.err || exit 1
done
for cap in 0 4 3; do
  SDR_SWEEP_SLOTS=$cap timeout -k 10 200 python -u bench.py --config c5 --steps 60 --warmup 6 --no-cpu-baseline \
      --no-stream-probe > $O/c5_s$cap.json 2> $O/c5_s$cap.err || exit 1
done
echo slots-done
