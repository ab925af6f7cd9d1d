#!/bin/bash
# C4 single-stream PMC passes (stall breakdown of the class path's kernels).
# usage (via gpurun): bash scripts/gpu_c4pmc.sh <tag>
set -e
TAG=${1:-c4pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
CMD="python3 bench.py --config c4 --streams 1 --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d "$O/pmc1" -o run -- $CMD > "$O/pmc1.log" 2>&1
python3 scripts/pmc_quick.py "$O/pmc1"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS --output-format csv -d "$O/pmc2" -o run -- $CMD > "$O/pmc2.log" 2>&1
python3 scripts/pmc_quick.py "$O/pmc2"
