#!/bin/bash
# A/B on one box: C4's frames in flight x hardware queues a process (GPU_MAX_HW_QUEUES, HIP's
# default 4 on this pool)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_c4q}
mkdir -p $O
for q in 4 8; do
  for s in 4 6 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --config c4 --steps 200 --warmup 20 --streams $s \
        --no-cpu-baseline --no-stream-probe --no-kernel-timing > $O/c4_q${q}_s$s.json 2> $O/c4_q${q}_s$s.err || exit 1
  done
done
echo c4q-done
