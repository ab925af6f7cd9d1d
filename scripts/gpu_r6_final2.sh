#!/bin/bash
# Round 6 final, second pass (after the sweep epilogue queue and the C5 voxel stage): the GPU suite,
# smoke, the default lines of C2 (with the CPU baseline), C3, C4, C5, C4 on one stream, and a
# rocprofv3 kernel-trace summary of C3 and C5 on one stream
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/c2.json 2> $O/c2.err &&
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/c3.json 2> $O/c3.err &&
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/c4.json 2> $O/c4.err &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline > $O/c4s1.json 2> $O/c4s1.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --config c3 --steps 6 --warmup 2 --streams 1 --iso-steps 2 --no-cpu-baseline --no-stream-probe \
    > $O/prof_c3.json 2> $O/prof_c3.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- \
    python3 bench.py --config c5 --steps 6 --warmup 2 --streams 1 --iso-steps 2 --no-cpu-baseline --no-stream-probe \
    > $O/prof_c5.json 2> $O/prof_c5.err
echo final2-done
