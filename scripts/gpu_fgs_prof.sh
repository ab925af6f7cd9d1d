#!/bin/bash
# FGS kernel timing + PMC counters.  usage (via gpurun): bash scripts/gpu_fgs_prof.sh <tag>
set -e
TAG=${1:-fgs}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 120 python3 scripts/fgs_bench.py 50 > "$O/bench.log" 2>&1
cat "$O/bench.log"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 scripts/fgs_bench.py 50 > "$O/prof.log" 2>&1
python3 scripts/kstats.py "$O/prof"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT --kernel-include-regex fgs_pcr --output-format csv -d "$O/pmc1" -o run -- python3 scripts/fgs_bench.py 5 > "$O/pmc1.log" 2>&1
python3 scripts/pmc_quick.py "$O/pmc1"
