#!/bin/bash
# FGS PCR PMC passes.  usage (via gpurun): bash scripts/gpu_fgs_pmc.sh <tag>
set -e
TAG=${1:-fgspmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex fgs_pcr --output-format csv -d "$O/pmc1" -o run -- python3 scripts/fgs_bench.py 5 > "$O/pmc1.log" 2>&1
python3 scripts/pmc_quick.py "$O/pmc1"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-include-regex fgs_pcr --output-format csv -d "$O/pmc2" -o run -- python3 scripts/fgs_bench.py 5 > "$O/pmc2.log" 2>&1
python3 scripts/pmc_quick.py "$O/pmc2"
