#!/bin/bash
# The RCCL world-1 line against the plain one with HIP's 4 hardware queues and with 8
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_dist_hwq}
mkdir -p $O
B="--steps 200 --warmup 20 --no-cpu-baseline --no-stream-probe --no-hbm-only --no-kernel-timing"
D="python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541"
timeout -k 10 200 python -u bench.py $B > $O/plain_q4.json 2> $O/e1 &&
timeout -k 10 200 $D bench.py --dist-world1 $B > $O/dist_q4.json 2> $O/e2 &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py $B > $O/plain_q8.json 2> $O/e3 &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $D bench.py --dist-world1 $B > $O/dist_q8.json 2> $O/e4 &&
timeout -k 10 200 $D bench.py --dist-world1 $B --streams 2 > $O/dist_q4_s2.json 2> $O/e5 &&
timeout -k 10 200 $D bench.py --dist-world1 $B --status-every 100000 > $O/dist_q4_nostatus.json 2> $O/e6 &&
timeout -k 10 60 scripts/probe/fgs_rows > $O/fgs_rows.txt 2>&1
echo hwq-done
