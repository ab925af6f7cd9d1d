#!/bin/bash
# Round 6: the batched gather -- the distributed GPU tests, then C2 plain vs C2 over RCCL at world 1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6_dist}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_distributed.py \
    > $O/dist_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-stream-probe --no-hbm-only \
    > $O/c2.json 2> $O/c2.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --dist-world1 --steps 200 --warmup 20 --no-cpu-baseline --no-stream-probe \
    --no-hbm-only > $O/c2_dist_world1.json 2> $O/c2_dist_world1.err &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-stream-probe --no-hbm-only \
    > $O/c2b.json 2> $O/c2b.err
echo dist-done
