#!/bin/bash
# Round 5 end, part A: the GPU suite, smoke, every config's bench line (C2 with the CPU baseline),
# C4 on one stream, and the RCCL world-1 line.  Each GPU step under its own limit, chained.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round_end_a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 900 bash scripts/gpu_bench_all.sh round_end_a cpu > $O/bench_all.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    > $O/c4s1.json 2> $O/c4s1.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --dist-world1 --steps 100 --warmup 10 --no-cpu-baseline \
    > $O/c2_dist_world1.json 2> $O/c2_dist_world1.err
echo finA-done
