#!/bin/bash
# Round 6 final: the GPU suite, smoke, every config's bench line with the CPU baselines, C4 on one
# stream, the RCCL world-1 line, rocprofv3 kernel-trace stats of the lines, then the HBM PMC passes
# (FETCH_SIZE / WRITE_SIZE, one counter group a run, no tracing) of C2, C3, C4 and C5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_final
mkdir -p $O
prof() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- \
      python3 bench.py "$@" > $O/prof_$n.json 2> $O/prof_$n.err
}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 1500 bash scripts/gpu_bench_all.sh r6_final/bench cpu > $O/bench_all.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 200 --warmup 20 --streams 1 --no-cpu-baseline \
    > $O/c4s1.json 2> $O/c4s1.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --dist-world1 --steps 200 --warmup 20 --no-cpu-baseline \
    > $O/c2_dist_world1.json 2> $O/c2_dist_world1.err &&
prof c2s1 --steps 60 --warmup 10 --no-cpu-baseline --streams 1 --no-stream-probe &&
prof c3 --config c3 --steps 6 --warmup 2 --streams 1 --iso-steps 2 --no-cpu-baseline --no-stream-probe &&
prof c4s1 --config c4 --steps 60 --warmup 10 --streams 1 --no-cpu-baseline --no-stream-probe &&
prof c5 --config c5 --steps 6 --warmup 2 --streams 1 --iso-steps 2 --no-cpu-baseline --no-stream-probe &&
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_c2_$grp -o run -- \
      python3 bench.py --steps 6 --warmup 2 --streams 1 --no-cpu-baseline --no-kernel-timing \
      --no-stream-probe > $O/pmc_c2_$grp.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_c3_$grp -o run -- \
      python3 bench.py --config c3 --steps 3 --warmup 1 --streams 1 --iso-steps 1 --no-cpu-baseline \
      --no-kernel-timing --no-stream-probe > $O/pmc_c3_$grp.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_c4_$grp -o run -- \
      python3 bench.py --config c4 --steps 6 --warmup 2 --streams 1 --no-cpu-baseline --no-kernel-timing \
      --no-stream-probe > $O/pmc_c4_$grp.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_c5_$grp -o run -- \
      python3 bench.py --config c5 --steps 3 --warmup 1 --streams 1 --iso-steps 1 --no-cpu-baseline \
      --no-kernel-timing --no-stream-probe > $O/pmc_c5_$grp.log 2>&1 || exit 1
done
echo r6final-done
