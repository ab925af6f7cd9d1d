#!/bin/bash
# C2 with 2 and 3 frames in flight, plain and over RCCL at world size 1, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_streams}
mkdir -p $O
B="--steps 300 --warmup 20 --no-cpu-baseline --no-stream-probe --no-hbm-only --no-kernel-timing"
D="python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29543"
for r in 1 2; do
  for s in 2 3; do
    timeout -k 10 200 python -u bench.py $B --streams $s > $O/plain_s${s}_$r.json 2> $O/e &&
    timeout -k 10 200 $D bench.py --dist-world1 $B --streams $s > $O/dist_s${s}_$r.json 2> $O/e || exit 1
  done
done
echo streams-done
