#!/bin/bash
# rocprofv3 kernel trace of the RCCL world-1 C2 line (bench.py --dist-world1 with the rank's
# environment set by hand: no launcher under the profiler) and of the plain C2 line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_distprof}
mkdir -p $O
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dist -o run -- python3 bench.py --dist-world1 \
    --steps 100 --warmup 10 --no-cpu-baseline --no-stream-probe --no-hbm-only --no-kernel-timing \
    > $O/dist.json 2> $O/dist.err &&
unset RANK LOCAL_RANK WORLD_SIZE LOCAL_WORLD_SIZE MASTER_ADDR MASTER_PORT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/plain -o run -- python3 bench.py \
    --steps 100 --warmup 10 --no-cpu-baseline --no-stream-probe --no-hbm-only --no-kernel-timing \
    > $O/plain.json 2> $O/plain.err
echo distprof-done
