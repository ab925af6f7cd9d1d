# PMC passes (SQ issue/wait counters) for the path kernels at C2, single stream.
# usage (via gpurun): bash scripts/pmc_south.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_south; mkdir -p $O
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -io "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_INST_CYCLES_[A-Z_]*\|SQ_WAIT_INST_[A-Z_]*\|SQ_BUSY_CU_CYCLES\|SQ_INSTS_[A-Z_]*" $O/avail.txt | sort -u | tr '\n' ' ' > $O/names.txt || true
cat $O/names.txt | head -c 3000; echo
ARGS="--config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing --streams 1"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" "SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$O/p$i" -o run -- python3 bench.py $ARGS > "$O/p$i.log" 2>&1 || echo "pass $i failed"
done
echo pmc-done
