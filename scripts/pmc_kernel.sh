#!/bin/bash
# PMC passes over the in-process A/B harness (one library, one config), one counter group per
# rocprofv3 run (--pmc is never combined with tracing domains).
# usage (via gpurun): bash scripts/pmc_kernel.sh <outdir> <lib.so> <config>
set -e
OUT=$1; LIB=$2; CFG=${3:-c2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 scripts/kbench.py --libs "$LIB" --config "$CFG" --rounds 1 --iters 5 > "$OUT/p$i.log" 2>&1
done
echo pmc-done
